#!/bin/bash
# GPU tests only (optionally a -k selection first): bash tools/r06_tests.sh TAG [pytest args...]
set -o pipefail
P=${1:-r06t}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread "$@" > gpurun_out/${P}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${P}_tests.log
exit $rc
