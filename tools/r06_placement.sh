#!/bin/bash
# Round-6 placement study: BSGS walk processes at the bench geometry, each one
# sample of the per-process placement state.  Bare runs (rate, board clock/power, buffer addresses),
# then rocprofv3 counter passes over the same workload (translation, L2-request latency, L2/fabric).
#   tools/r06_placement.sh TAG [REPEATS]
set -o pipefail
T=${1:-r06a}; N=${2:-4}
O=gpurun_out/$T; mkdir -p $O
W="python3 tools/placement_pmc.py"
[ -f $O/avail.txt ] || timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list rc=$?"
for i in $(seq 1 $N); do
  timeout -k 10 150 $W --tag bare$i >> $O/bare.jsonl 2>> $O/bare.err || { echo "bare $i rc=$?"; tail $O/bare.err; exit 1; }
done
pass() {  # pass NAME COUNTERS...
  local n=$1; shift
  for i in $(seq 1 $N); do
    timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n$i -o run -- \
      $W --no-board --tag $n$i >> $O/pmc.jsonl 2> $O/$n$i.err || { echo "pmc $n $i rc=$?"; tail $O/$n$i.err; exit 1; }
  done
}
pass tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum \
  TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY || exit 1
pass lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum \
  TCP_UTCL1_STALL_LFIFO_NO_RES_sum GRBM_GUI_ACTIVE || exit 1
pass l2 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
echo "placement $T done"
