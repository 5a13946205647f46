#!/bin/bash
# Interleaved processes of the bench's BSGS leg, one per variant per round (PAIRS rounds):
#   nocal: no calibration (2^21 lanes, the first placements); pad2: the pad stage only, 2 candidates;
#   lanes: 2^21 against 2^20 lanes on one pad; mix3: two pads at 2^21 and the first at 2^20; l20: 2^20 lanes;
#   move: the pad moved (once or twice) after one uncalibrated call; lanesd: lanes after one uncalibrated call;
#   nocalb / lanesb: nocal / the default calibration after a 1-s VALU burn ahead of the first walk;
#   both2: pad then layer-1 stage, 2 pad candidates; pad3: the pad stage only, 3 candidates
#   bash tools/r06_cal_ab.sh TAG PAIRS [VARIANTS...]
set -o pipefail
T=${1:-r06n}; P=${2:-2}; shift 2
V=${*:-"nocal pad2 both2 pad3"}
O=gpurun_out/$T; mkdir -p $O
for i in $(seq 1 $P); do
  for v in $V; do
    case $v in
      nocal) E="KH_BSGS_CALIBRATE=0";; pad2) E="KH_CAL_STAGES=1 KH_PAD_CANDIDATES=2";;
      both2) E="KH_CAL_STAGES=2 KH_PAD_CANDIDATES=2";; pad3) E="KH_CAL_STAGES=1 KH_PAD_CANDIDATES=3";;
      lanes) E="KH_CAL_STAGES=1 KH_PAD_CANDIDATES=1";;
      mix3) E="KH_CAL_STAGES=1 KH_PAD_CANDIDATES=2 KH_CAL_LANES=1";;
      l20) E="KH_BSGS_LANES=1048576";;
      move) E="KH_CAL_STAGES=1 KH_CAL_MOVE=1 KH_CAL_DEFER=1";;
      lanesd) E="KH_CAL_STAGES=1 KH_PAD_CANDIDATES=1 KH_CAL_DEFER=1";;
      nocalb) E="KH_BSGS_CALIBRATE=0 KH_BURN_MS=1000";;
      lanesb) E="KH_BURN_MS=1000";;
    esac
    env $E timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --seconds 30 --steps 5 --warmup 2 \
      > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v $i rc=$?"; tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]); c=d['config']['placement_calibration']; print('$v', $i, round(d['giant_points_per_s']/1e9,3), [round(x/1e9,2) for x in (c['pad_giant_points_per_s_kept'], c['pad_other'], c['layer1_giant_points_per_s_kept'], c['layer1_other'])], round(d['sustained']['board'].get('board_gfxclk_mhz') or 0))"
  done
done
