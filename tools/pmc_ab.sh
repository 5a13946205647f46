#!/bin/bash
# PMC A/B: passes 4-5 of gpu_round.sh for two library builds
set -o pipefail
O=gpurun_out/pmcab; mkdir -p $O
for v in ${PMC_VARIANTS:-main red0}; do
  if [ $v = main ]; then L=keyhunt_amd/lib/libkh_gpu.so; else L=variants/$v/libkh_gpu.so; fi
  i=0
  for c in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i + 1))
    KH_LIB=$L timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $O/$v/p$i -o run -- \
      python3 tools/pmc_run.py > $O/${v}_p$i.log 2>&1 || { echo "pmc $v $i rc=$?"; tail -20 $O/${v}_p$i.log; exit 1; }
  done
done
echo pmc ok
