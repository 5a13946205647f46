#!/bin/bash
# round-6 tree check: full GPU suite, smoke, default bench line (the driver's round-end sequence)
#   bash tools/r06_final.sh TAG [bench args...]
set -o pipefail
P=${1:-r06x}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${P}_tests.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 || exit 1
timeout -k 10 700 python bench.py "$@" > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/${P}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${P}_bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['legs']))"
exit $rc
