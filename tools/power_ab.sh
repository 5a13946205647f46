#!/bin/bash
# BSGS walk variants A/B with the board's power and power-limit residency (round 4): timing builds
# (tools/build_variants.sh) whose known answers fail are expected to exit 3.
#   tools/power_ab.sh TAG SECONDS NAME...   (main = keyhunt_amd/lib)
set -o pipefail
TAG=$1; SECS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for v in "$@"; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  rc=0
  KH_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-secondary --seconds $SECS > $O/$v.json 2> $O/$v.err || rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "bench $v rc=$rc"; tail -20 $O/$v.err; exit 1; fi
  python3 -c "
import json;d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); s=d['sustained']; b=s.get('board') or {}
print('$v', 'G pts/s %.3f walk ms %.3f clock MHz %.0f power W %.0f ppt %.2f pts/J %.3g' % (d['giant_points_per_s']/1e9, d['roofline']['mean_launch_ms'], b.get('board_gfxclk_mhz') or 0, b.get('socket_power_w') or 0, b.get('ppt_residency_frac') or -1, s.get('points_per_joule') or 0))"
done
