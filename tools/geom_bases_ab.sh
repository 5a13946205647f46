# BSGS lanes per launch vs call size: bench-sized calls (7274496 bases -> 1039214 lanes) against
# 2^23-base calls (2^20 lanes), interleaved, one invocation of tools/geom_ab.py each
set -e
P=${1:-r05q}
mkdir -p gpurun_out
i=0
for nb in 7274496 8388608 7274496 8388608; do
  i=$((i + 1))
  timeout -k 10 200 python -u tools/geom_ab.py --seconds 15 --bsgs-bases $nb bsgs:0:0:1 > gpurun_out/${P}_geom_$i.json 2>> gpurun_out/${P}_geom.err
done
