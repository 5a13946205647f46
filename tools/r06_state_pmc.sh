#!/bin/bash
# Counters that separate the BSGS walk's fast and slow states.  Re-allocating the
# walk's pad alternates the state inside one process, so each counter pass is ONE process of
# tools/state_pmc.py (4 pad allocations, 2 timed dispatches each) under rocprofv3.
#   bash tools/r06_state_pmc.sh TAG
set -o pipefail
T=${1:-r06f}
O=gpurun_out/$T; mkdir -p $O
pass() {  # pass NAME COUNTERS...
  local n=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o run -- \
    python3 tools/state_pmc.py --allocs 4 --calls 2 --tag $n >> $O/pmc.jsonl 2> $O/$n.err \
    || { echo "pmc $n rc=$?"; tail $O/$n.err; exit 1; }
}
pass rd TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum \
  GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
pass wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
  GRBM_GUI_ACTIVE || exit 1
pass lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum \
  GRBM_GUI_ACTIVE || exit 1
pass tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum \
  TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY || exit 1
pass tlb2 TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_SERIALIZATION_STALL_sum \
  TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_GUI_ACTIVE || exit 1
pass val SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE || exit 1
echo "state pmc $T done"
