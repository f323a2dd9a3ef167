#!/bin/bash
# FRCNN A/B: RPN head levels on four stream lanes (default) or all on the caller stream.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3ab.txt
for v in 1 0 1 0; do
  for inf in 1 2; do
    x=$(EDGEDET_RPN_LANES=$v timeout -k 10 200 python bench.py --model frcnn --steps 300 --warmup 20 --no-cpu --no-e2e --no-roofline --inflight $inf 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d = d.get('frcnn', d); print(d['value'], d['ms_per_step'])") || exit 6
    echo "rpn_lanes=$v inflight=$inf $x" >> gpurun_out/r3ab.txt
  done
done
