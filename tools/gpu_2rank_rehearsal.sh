#!/bin/bash
# the bench's N-rank path on a one-GPU box: 2 ranks under torchrun, gloo, both
# on the one GPU (DV_SHARE_GPU=1); checks the barrier / max-over-ranks timing
# and the one JSON line rank 0 prints.  The driver's multi-GPU runs use RCCL.
export TMPDIR=/tmp
tag=${1:-r2}
mkdir -p gpurun_out
DV_DIST_BACKEND=gloo DV_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline --no-sampling \
  --no-fp32 > gpurun_out/${tag}.log 2>&1 || exit 1
tail -1 gpurun_out/${tag}.log
