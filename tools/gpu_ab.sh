#!/bin/bash
# Alternated A/B of one environment switch: VAR=<name> VALUES="a b ..." [MODEL=ssd|frcnn] [ROUNDS=2]
# [STEPS=750]; round r runs the values in order, round r+1 reversed (ABBA), each a fresh process.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/ab.log
m=${MODEL:-ssd}
for r in $(seq 1 ${ROUNDS:-2}); do
  o="$VALUES"; [ $((r % 2)) = 0 ] && o=$(echo $VALUES | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $o; do
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --model $m --steps ${STEPS:-750} --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline > gpurun_out/ab_${v}_r$r.log 2>&1
    rc=$?
    echo "$VAR=$v r$r rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_r$r.log | head -1)" >> gpurun_out/ab.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
