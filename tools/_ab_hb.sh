set -o pipefail
O=gpurun_out/r01h; mkdir -p $O
for v in main addsub; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  KH_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 20 > $O/$v.json 2> $O/$v.err || { echo "bench $v rc=$?"; tail -20 $O/$v.err; exit 1; }
done
python - <<'P'
import json
for n in ("main","addsub"):
    d=json.load(open(f"gpurun_out/r01h/{n}.json")); r=d["roofline"]
    print(n, d["giant_points_per_s"]/1e9, r["mean_launch_ms"], r["giant_points_per_launch"], r["frac"], d["first_level_candidates"])
P
