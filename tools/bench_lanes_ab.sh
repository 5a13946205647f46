# BSGS bench leg (30 s timed, no CPU baseline, no address legs) with the wide-lane path (default)
# against KH_BSGS_NARROW=1 (2^18 lanes), interleaved in pairs on one box
set -e
P=${1:-r05q}
mkdir -p gpurun_out
for i in $(seq 1 ${2:-2}); do
  KH_BSGS_NARROW=1 timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --seconds 30 > gpurun_out/${P}_bench_narrow_$i.json 2>> gpurun_out/${P}_bench_ab.err
  timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --seconds 30 > gpurun_out/${P}_bench_wide_$i.json 2>> gpurun_out/${P}_bench_ab.err
done
