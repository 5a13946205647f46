# BSGS tests with the lane-tiling changes, then the default bench (and its rocprof stats)
set -e
P=${1:-r05r}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsgs.py tests/test_gpu_multictx.py tests/test_gpu_integration.py > gpurun_out/${P}_tests.log 2>&1
bash tools/gpu_round.sh $P bench,prof > gpurun_out/${P}_round.txt 2>&1
