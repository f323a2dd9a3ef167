#!/bin/bash
# Grid-cap sweep of the streaming 1x1 tiles (EDGEDET_PWS_WG), SSD device rate, twice interleaved.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/pws_grid.log
for rep in 1 2; do
for g in 2048 512 1024 4096; do
  EDGEDET_PWS_WG=$g timeout -k 10 300 python bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/pws_ops_$g.json 2>/dev/null | grep '"metric"' > gpurun_out/pws_b_$g.json || exit 7
  python3 -c "import json; d=json.load(open('gpurun_out/pws_b_$g.json')); print('$g', d['value'], d['ms_per_step'])" >> gpurun_out/pws_grid.log
done
done
exit 0
