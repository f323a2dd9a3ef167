#!/bin/bash
# round-5 session g: SSD head 1x1 group tiles (A/B, alternated): one group on tile 31 (default) / tile 29;
# cls on 31 and the narrow reg members in their own group on tile 38 / on the tuned per-shape tile
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5g_steps.log
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r5g_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5g_$name.log | head -1)" >> gpurun_out/r5g_steps.log; [ $rc -ne 0 ] && exit $rc; return 0; }
B="python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline"
for r in 1 2; do
  run base_$r $B
  run reg38_$r env EDGEDET_SSD_HEAD_REG_TILE=38 $B
  run cls29_$r env EDGEDET_SSD_HEAD_TILE=29 $B
  run reg0_$r env EDGEDET_SSD_HEAD_REG_TILE=0 $B
done
run ops_reg38 env EDGEDET_SSD_HEAD_REG_TILE=38 python -u bench.py --model ssd --steps 100 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5g_ops_reg38.json
run frcnn_if3 python -u bench.py --model frcnn --steps 750 --no-cpu --no-e2e --no-roofline
run frcnn_if2 python -u bench.py --model frcnn --steps 750 --no-cpu --no-e2e --no-roofline --inflight 2
run frcnn_if2b python -u bench.py --model frcnn --steps 750 --no-cpu --no-e2e --no-roofline --inflight 2
run frcnn_if3b python -u bench.py --model frcnn --steps 750 --no-cpu --no-e2e --no-roofline
