# round-5 closing measurements, part 2: PMC passes (bench geometry) and the CLI's BSGS rates
set -e
P=${1:-r05u}
bash tools/gpu_round.sh $P pmc > gpurun_out/${P}_pmc_round.txt 2>&1
for m in bsgs bsgs_random bsgs_both; do
  timeout -k 10 150 python tools/cli_rate.py --mode $m --seconds 100 --skip 20 --out gpurun_out/${P}_cli_rate_$m.json > gpurun_out/${P}_$m.txt 2>&1
done
