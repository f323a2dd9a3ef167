#!/bin/bash
# FRCNN batches in flight on the final tree.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3af.txt
for inf in 2 3 4 2 3; do
  x=$(timeout -k 10 200 python bench.py --model frcnn --steps 300 --warmup 20 --no-cpu --no-e2e --no-roofline --inflight $inf 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d = d.get('frcnn', d); print(d['value'], d['ms_per_step'])") || exit 6
  echo "inflight=$inf $x" >> gpurun_out/r3af.txt
done
