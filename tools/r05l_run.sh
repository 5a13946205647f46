# round-5 BSGS list/geometry GPU step: BSGS tests, the list-call probe, CLI rates (-B sequential/random/both)
set -e
mkdir -p gpurun_out
P=${1:-r05o}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsgs.py tests/test_gpu_stdout.py tests/test_gpu_multictx.py > gpurun_out/${P}_tests.log 2>&1
timeout -k 10 200 python -u tools/bsgs_list_probe.py --calls 3 --out gpurun_out/${P}_list_probe.json > gpurun_out/${P}_probe.txt 2>&1
for m in bsgs bsgs_random bsgs_both; do
  timeout -k 10 120 python tools/cli_rate.py --mode $m --seconds 70 --skip 20 --out gpurun_out/${P}_cli_rate_$m.json > gpurun_out/${P}_$m.txt 2>&1
done
