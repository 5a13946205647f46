#!/bin/bash
# ISA of the BSGS giant walk alone (KH_ISA_ONLY_BSGSB): tools/isa_bsgs.sh OUT.s [-DFLAG ...]
# then python tools/isa_hot.py OUT.s _Z6k_walkILi7ELi2048EEv9walk_args
set -e
OUT=$1; shift
cd "$(dirname "$0")/../keyhunt_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DKH_WALK_H=512 -DKH_WALK_LB=4 -DKH_WALK_LB_HASH=3 \
  -DKH_ISA_ONLY_BSGSB -DKH_ISA_MARKS "$@" --cuda-device-only -S csrc/kh_kernels.hip -I../include -Icsrc -o "$OUT"
