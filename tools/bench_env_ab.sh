# bench.py BSGS leg (30 s timed, no CPU baseline, no address legs): the default against one
# environment setting ($3, e.g. KH_BSGS_ROUND_POINTS=34359738368), interleaved pairs, one process per run
set -e
P=${1:-r05ab}
N=${2:-3}
ENVSET=$3
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --seconds 30 > gpurun_out/${P}_bench_base_$i.json 2>> gpurun_out/${P}_bench_ab.err
  env $ENVSET timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --seconds 30 > gpurun_out/${P}_bench_alt_$i.json 2>> gpurun_out/${P}_bench_ab.err
done
