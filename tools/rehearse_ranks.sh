#!/bin/bash
# Rehearsal of the driver's N>1 bench on a 1-GPU box: all ranks share device 0 (d % ndev).
#   bash tools/rehearse_ranks.sh TAG N       torchrun launch, as the driver does
#   bash tools/rehearse_ranks.sh TAG N self  bench.py --gpus N starting its own ranks
set -o pipefail
TAG=${1:-rehearse}; N=${2:-2}; MODE=${3:-torchrun}
O=gpurun_out/$TAG; mkdir -p $O
if [ "$MODE" = self ]; then
  timeout -k 10 600 python bench.py --gpus $N --steps 4 --warmup 1 --no-cpu-baseline > $O/n$N.json 2> $O/n$N.err \
    || { echo "self n$N rc=$?"; tail -30 $O/n$N.err; exit 1; }
else
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus $N --steps 4 --warmup 1 > $O/n$N.json 2> $O/n$N.err \
    || { echo "torchrun n$N rc=$?"; tail -30 $O/n$N.err; exit 1; }
fi
cat $O/n$N.json
