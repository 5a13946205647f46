set -o pipefail
timeout -k 10 1100 python -m pytest tests/test_gpu_scan.py tests/test_gpu_primitives.py -q -m gpu > gpurun_out/t15_scan.log 2>&1; echo "scan tests rc=$?"; tail -15 gpurun_out/t15_scan.log
