#!/bin/bash
# A/B timing of library variants on the GPU box: tools/ab_variants.sh NAME... (variants/NAME/libkh_gpu.so)
set -o pipefail
mkdir -p gpurun_out
for n in "$@"; do
  KH_LIB=variants/$n/libkh_gpu.so timeout -k 10 300 python tools/quick_perf.py > gpurun_out/ab_$n.log 2>&1 || { echo "$n failed rc=$?"; tail -5 gpurun_out/ab_$n.log; exit 1; }
  cat gpurun_out/ab_$n.log
done
