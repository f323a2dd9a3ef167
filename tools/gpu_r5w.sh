#!/bin/bash
# round-5 session w: batches in flight re-measured on the round-5 kernels (FRCNN 2 / 3 / 4, SSD 3 / 4 / 5 / 6), alternated
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5w_steps.log
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r5w_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5w_$name.log | head -1)" >> gpurun_out/r5w_steps.log; [ $rc -ne 0 ] && exit $rc; return 0; }
F="python -u bench.py --model frcnn --steps 300 --warmup 10 --no-cpu --no-e2e --no-roofline"
S="python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline"
for r in 1 2; do
  for n in 3 2 4; do run frcnn_if${n}_$r $F --inflight $n; done
  for n in 4 5 6 3; do run ssd_if${n}_$r $S --inflight $n; done
done
exit 0
