# the CLI's BSGS rates (sequential, -B random, -B both), 100 s each
set -e
P=${1:-r05ai}
mkdir -p gpurun_out
for m in bsgs bsgs_random bsgs_both; do
  timeout -k 10 150 python tools/cli_rate.py --mode $m --seconds 100 --skip 20 --out gpurun_out/${P}_cli_rate_$m.json > gpurun_out/${P}_$m.txt 2>&1
done
