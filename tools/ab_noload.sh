set -o pipefail
mkdir -p gpurun_out/ab
for v in main noload; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  KH_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { echo "bench $v rc=$?"; tail -20 gpurun_out/ab/$v.err; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));print('$v', d['giant_points_per_s']/1e9, d['roofline']['mean_launch_ms'])"
done
