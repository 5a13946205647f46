set -o pipefail
timeout -k 10 900 python -m pytest tests/test_gpu_bsgs.py -q -m gpu > gpurun_out/t14_bsgs.log 2>&1; echo "bsgs tests rc=$?"; tail -3 gpurun_out/t14_bsgs.log
timeout -k 10 300 python tools/bsgs_k_sweep.py 128:1 > gpurun_out/sweep14.log 2>&1; cat gpurun_out/sweep14.log
