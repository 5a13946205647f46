#!/bin/bash
# One rocprofv3 counter pass of tools/pmc_run.py: tools/pmc_one.sh TAG "COUNTERS" [LIB]
set -o pipefail
TAG=$1; C=$2; L=${3:-keyhunt_amd/lib/libkh_gpu.so}
O=gpurun_out/pmc1/$TAG; mkdir -p $O
KH_LIB=$L timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $O -o run -- python3 tools/pmc_run.py > $O.log 2>&1 \
  || { echo "pmc $TAG rc=$?"; tail -20 $O.log; exit 1; }
echo "pmc $TAG ok"
