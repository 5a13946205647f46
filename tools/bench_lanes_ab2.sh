# BSGS bench leg (30 s timed, no CPU baseline, no address legs): KH_BSGS_LANES=$3 against the
# default lanes, interleaved pairs, one process per run
set -e
P=${1:-r05x}
N=${2:-3}
W=${3:-2097152}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --seconds 30 > gpurun_out/${P}_bench_base_$i.json 2>> gpurun_out/${P}_bench_ab.err
  KH_BSGS_LANES=$W timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --seconds 30 > gpurun_out/${P}_bench_alt_$i.json 2>> gpurun_out/${P}_bench_ab.err
done
