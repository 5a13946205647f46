# 4-rank rehearsal of the driver's N>1 bench on a 1-GPU box (both ranks share device 0), then the
# default 1-GPU bench with the tertiary leg
set -o pipefail
O=gpurun_out/r01q; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 4 --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc=$?"; tail -30 $O/n2.err; exit 1; }
cat $O/n2.json
