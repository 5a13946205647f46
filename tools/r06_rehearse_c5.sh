#!/bin/bash
# config 5 (-b 130 -k 512) with two ranks stacked on one GPU (bench.py starts its
# own ranks; --rehearse lets them share device 0).  Exercises the per-rank memory plan (2^21-lane pad +
# k = 512 tables per rank) and the k = 512 known-answer check on every rank.
#   bash tools/r06_rehearse_c5.sh TAG
set -o pipefail
T=${1:-r06c5}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python bench.py --gpus 2 --rehearse --config 5 --steps 4 --warmup 1 --seconds 20 \
  --no-cpu-baseline --no-secondary > $O/n2_config5.json 2> $O/n2_config5.err \
  || { echo "rehearse c5 rc=$?"; tail -30 $O/n2_config5.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/n2_config5.json').read().strip().splitlines()[-1]); print(json.dumps({k: d.get(k) for k in ('value','n_gpus','devices_used','rehearsal','known_answers_all_ranks_match','giant_points_per_s','ranks')}))"
