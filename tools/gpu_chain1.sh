#!/bin/bash
# One 32-image chain per batch with more batches in flight: tune the B=32 keys (EDGEDET_SSD_CHAINS=1),
# then compare against the default two 16-image chains x two in flight.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
cp edgeml-object-detection_amd/data/conv_tiles_gfx950.json gpurun_out/tiles_c1.json
EDGEDET_SSD_CHAINS=1 timeout -k 10 900 python -u tools/tune_conv.py --models ssd --out gpurun_out/tiles_c1.json > gpurun_out/c1_tune.log 2>&1 || exit 7
cp gpurun_out/tiles_c1.json edgeml-object-detection_amd/data/conv_tiles_gfx950.json
: > gpurun_out/c1_sweep.log
for cfg in "2 2" "1 2" "1 3" "1 4" "2 2"; do
  set -- $cfg
  v=$(EDGEDET_SSD_CHAINS=$1 timeout -k 10 300 python bench.py --model ssd --steps 500 --warmup 20 --no-cpu --no-e2e --inflight $2 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 6
  echo "chains=$1 inflight=$2 $v" >> gpurun_out/c1_sweep.log
done
exit 0
