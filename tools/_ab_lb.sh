set -o pipefail
O=gpurun_out/r01m; mkdir -p $O
for v in main pad; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  KH_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { echo "bench $v rc=$?"; tail -20 $O/$v.err; exit 1; }
done
python - <<'P'
import json
for n in ("main","pad"):
    d=json.load(open(f"gpurun_out/r01m/{n}.json"))
    print(n, d["giant_points_per_s"]/1e9, d["roofline"]["mean_launch_ms"], d["secondary"]["kernel"]["points_per_s_in_kernel"]/1e9, d["tertiary"]["kernel"]["points_per_s_in_kernel"]/1e9)
P
