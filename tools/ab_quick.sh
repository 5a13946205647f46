#!/bin/bash
# Quick GPU check of a library change: the primitive / scan / BSGS parity tests, then an
# interleaved A/B of bench lines (short sustained windows) between builds.
#   tools/ab_quick.sh TAG "TESTS" NAME...   (NAME: main = keyhunt_amd/lib, else variants/NAME)
set -o pipefail
TAG=$1; TESTS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTS" ]; then
  # a failing test does not stop the A/B; a crash or a time-out (rc > 1) does
  rc=0
  timeout -k 10 900 python -u -m pytest $TESTS -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || rc=$?
  tail -3 $O/tests.log
  [ $rc -gt 1 ] && { echo "tests rc=$rc"; tail -30 $O/tests.log; exit 1; }
fi
i=0
for v in "$@"; do
  i=$((i + 1))
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  KH_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --seconds 12 --seconds-secondary 6 > $O/ab${i}_$v.json 2> $O/ab${i}_$v.err \
    || { echo "ab $v rc=$?"; tail -20 $O/ab${i}_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/ab${i}_$v.json'))
print('$v', 'bsgs G pts/s %.3f walk ms %.3f | rmd160 G pts/s kern %.4f | xpoint %.3f | ka %s' % (d['giant_points_per_s']/1e9, d['roofline']['mean_launch_ms'], d['secondary']['points_per_s_in_kernel']/1e9, d['tertiary']['points_per_s_in_kernel']/1e9, d['known_answers_all_ranks_match']))"
done
