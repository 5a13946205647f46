#!/bin/bash
# N separate processes of the bench's BSGS leg (each a fresh placement draw): rate and calibration
#   bash tools/r06_bench_runs.sh TAG N [bench args...]
set -o pipefail
T=${1:-r06g}; N=${2:-3}; shift 2
O=gpurun_out/$T; mkdir -p $O
for i in $(seq 1 $N); do
  timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --seconds 30 --steps 5 --warmup 2 "$@" \
    > $O/run$i.json 2> $O/run$i.err || { echo "bench run $i rc=$?"; tail -5 $O/run$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.json').read().strip().splitlines()[-1]); print($i, round(d['giant_points_per_s']/1e9,3), d['config'].get('placement_calibration'), d['sustained']['board'].get('board_gfxclk_mhz'), d['sustained']['board'].get('socket_power_w'))"
done
