#!/bin/bash
# rmd160 A/B of library variants: tools/ab_rmd.sh NAME... (variants/NAME/libkh_gpu.so)
set -o pipefail
mkdir -p gpurun_out
for n in "$@"; do
  KH_LIB=variants/$n/libkh_gpu.so timeout -k 10 300 python tools/perf_rmd.py > gpurun_out/abr_$n.log 2>&1 || { echo "$n failed rc=$?"; tail -5 gpurun_out/abr_$n.log; exit 1; }
  cat gpurun_out/abr_$n.log
done
