#!/bin/bash
# Round-3 exploration on one GPU box: clock-true class costs (ubench_cost), the new bench line, the
# s_nop price in the BSGS walk (A/B against a build with one more s_nop per carry count), and the
# new PMC pass (VALU thread-cycles, dual issue, wave-time split) on the shipped and the no-probe-load
# builds.  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${1:-r03b}; mkdir -p $O
timeout -k 10 120 tools/ubench_cost > $O/ubench_cost.txt 2>&1 || { echo "ubench rc=$?"; cat $O/ubench_cost.txt; exit 1; }
cat $O/ubench_cost.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for v in main xnops main xnops; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  KH_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --seconds 15 > $O/ab_$v.json 2> $O/ab_$v.err || { echo "ab $v rc=$?"; tail -20 $O/ab_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$v.json'));print('$v', d['giant_points_per_s']/1e9, d['roofline']['mean_launch_ms'])"
done
cd /tmp && export TMPDIR=/tmp
for v in main noload; do
  if [ $v = main ]; then L=$R/keyhunt_amd/lib/libkh_gpu.so; else L=$R/variants/$v/libkh_gpu.so; fi
  i=0
  for c in "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    KH_LIB=$L timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$v/p$i -o run -- \
      python3 $R/tools/pmc_run.py > $O/pmc_${v}_p$i.log 2>&1 || { echo "pmc $v pass $i rc=$?"; tail -20 $O/pmc_${v}_p$i.log; exit 1; }
  done
done
echo explore ok
