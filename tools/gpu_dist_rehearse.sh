#!/bin/bash
# Multi-rank rehearsal of bench.py on a one-GPU box: 2 ranks under torchrun sharing cuda:0 over gloo
# (the driver's N>1 runs use one GPU per rank over RCCL).  Checks the barrier / max-over-ranks /
# rank-0-only legs end to end.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp EDGEDET_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps ${STEPS:-200} --warmup 10 > gpurun_out/dist_rehearse.log 2>&1 || exit 5
exit 0
