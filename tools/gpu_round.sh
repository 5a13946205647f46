#!/bin/bash
# One GPU session: GPU tests, bench, rocprofv3 kernel-trace stats of the bench, PMC counter passes.
# Usage (on the box, from the repo root): bash tools/gpu_round.sh TAG [parts]
#   parts: any of tests,bench,prof,pmc,ubench,config5 (default tests,bench,prof,pmc).  Every GPU step has its own time limit and
#   the script stops at the first failure.
set -o pipefail
TAG=${1:-r01}
PARTS=${2:-tests,bench,prof,pmc}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
has() { [[ ",$PARTS," == *",$1,"* ]]; }
TESTS_RC=0
if has tests; then
  # a failing test does not stop the measurements; a crash or a time-out (rc > 1) does
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || TESTS_RC=$?
  tail -12 $O/tests.log
  [ $TESTS_RC -gt 1 ] && { echo "tests rc=$TESTS_RC"; exit 1; }
fi
if has bench; then
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
cd /tmp && export TMPDIR=/tmp
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.json 2> $O/prof.err \
    || { echo "prof rc=$?"; tail -20 $O/prof.err; exit 1; }
  echo "prof ok"
fi
if has pmc; then
  i=0
  for c in "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE" "FETCH_SIZE" \
           "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc/p$i -o run -- \
      python3 $R/tools/pmc_run.py > $O/pmc_p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -20 $O/pmc_p$i.log; exit 1; }
  done
  # the same workload's kernel durations (a run of its own, no counters)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc/trace -o run -- \
    python3 $R/tools/pmc_run.py > $O/pmc_trace.log 2>&1 || { echo "pmc trace rc=$?"; tail -20 $O/pmc_trace.log; exit 1; }
  echo "pmc ok"
fi
if has ubench; then
  timeout -k 10 120 $R/tools/ubench_cost > $O/ubench_cost.txt 2>&1 || { echo "ubench rc=$?"; tail -5 $O/ubench_cost.txt; exit 1; }
  cat $O/ubench_cost.txt
fi
if has config5; then
  timeout -k 10 600 python $R/bench.py --config 5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 rc=$?"; tail -20 $O/bench_c5.err; exit 1; }
  cat $O/bench_c5.json
fi
exit $TESTS_RC
