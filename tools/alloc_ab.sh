#!/bin/bash
# BSGS walk with layer 1 in different HIP memory types (KH_L1_ALLOC, kh_capi.cpp): power and rate
#   tools/alloc_ab.sh TAG SECONDS TYPE...   (TYPE: default | fine | uncached)
set -o pipefail
TAG=$1; SECS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for v in "$@"; do
  rc=0
  if [ $v = default ]; then E=""; else E="$v"; fi
  KH_L1_ALLOC=$E timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-secondary --seconds $SECS > $O/$v.json 2> $O/$v.err || rc=$?
  if [ $rc -ne 0 ]; then echo "bench $v rc=$rc"; tail -20 $O/$v.err; exit 1; fi
  python3 -c "
import json;d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); s=d['sustained']; b=s.get('board') or {}
print('$v', 'G pts/s %.3f walk ms %.3f clock MHz %.0f power W %.0f ppt %.2f pts/J %.3g ka %s' % (d['giant_points_per_s']/1e9, d['roofline']['mean_launch_ms'], b.get('board_gfxclk_mhz') or 0, b.get('socket_power_w') or 0, b.get('ppt_residency_frac') or -1, s.get('points_per_joule') or 0, d['known_answers_all_ranks_match']))"
done
