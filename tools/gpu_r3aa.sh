#!/bin/bash
# FRCNN: one instance in flight, with and without the small launches (diagnostic skips, wrong results).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3aa.txt
for sk in none 11 10 none; do
  [ $sk = none ] && unset EDGEDET_DIAG_SKIP || export EDGEDET_DIAG_SKIP=$sk
  for inf in 1 2; do
    v=$(timeout -k 10 200 python bench.py --model frcnn --steps 300 --warmup 20 --no-cpu --no-e2e --no-roofline --inflight $inf 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d = d.get('frcnn', d); print(d['value'], d['ms_per_step'])") || exit 6
    echo "skip=$sk inflight=$inf $v" >> gpurun_out/r3aa.txt
  done
done
