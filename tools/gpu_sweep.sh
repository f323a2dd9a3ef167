#!/bin/bash
# SSD step-shape sweep: HIP hardware queues x chains per batch x batches in flight (bench.py --model
# ssd, device rate only).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/sweep.log
for q in ${QUEUES:-4 8 16}; do
for ch in ${CHAINS:-2 4}; do
  for inf in ${INFL:-2 3 4}; do
    v=$(GPU_MAX_HW_QUEUES=$q EDGEDET_SSD_CHAINS=$ch timeout -k 10 300 python bench.py --model ssd --steps 300 --warmup 20 --no-cpu --no-e2e --inflight $inf 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 6
    echo "queues=$q chains=$ch inflight=$inf $v" >> gpurun_out/sweep.log
  done
done
done
exit 0
