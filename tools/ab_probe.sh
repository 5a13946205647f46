#!/bin/bash
# BSGS walk A/B of probe-load variants (timing builds whose known answers fail are expected to exit
# 3 -- any other failure stops the run): tools/ab_probe.sh TAG NAME...  (main = keyhunt_amd/lib)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for v in "$@"; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  rc=0
  KH_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --seconds 15 > $O/$v.json 2> $O/$v.err || rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "bench $v rc=$rc"; tail -20 $O/$v.err; exit 1; fi
  python3 -c "
import json;d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); s=d['sustained']
print('$v', 'G pts/s %.3f walk ms %.3f clock MHz %.0f/%.0f ka %s' % (d['giant_points_per_s']/1e9, d['roofline']['mean_launch_ms'], s['first_quarter']['board_gfxclk_mhz'], s['last_quarter']['board_gfxclk_mhz'], d['known_answers_all_ranks_match']))"
done
