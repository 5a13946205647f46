#!/bin/bash
# A/B of library builds with the real bench line: tools/ab_bench.sh NAME... where NAME is "main"
# (keyhunt_amd/lib) or a variant built by tools/build_variants.sh (variants/NAME/libkh_gpu.so).
# Prints, per build: wall G giant pts/s, BSGS walk ms per launch, rmd160 and xpoint G pts/s in kernel.
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
for v in "$@"; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  KH_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { echo "bench $v rc=$?"; tail -20 $O/$v.err; exit 1; }
done
python - "$@" <<'P'
import json, sys
for n in sys.argv[1:]:
    d = json.load(open(f"gpurun_out/ab/{n}.json"))
    print(n, d["giant_points_per_s"] / 1e9, d["roofline"]["mean_launch_ms"],
          d["secondary"]["points_per_s_in_kernel"] / 1e9, d["tertiary"]["points_per_s_in_kernel"] / 1e9)
P
