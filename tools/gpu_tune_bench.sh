#!/bin/bash
# tools/gpu_tune.sh, then the bench on the re-tuned table (copied over the box's copy of the data
# file; the Python host reads it at import).
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/gpu_tune.sh || exit $?
cp gpurun_out/tiles_new.json edgeml-object-detection_amd/data/conv_tiles_gfx950.json
timeout -k 10 300 python bench.py --model both --no-cpu --no-e2e > gpurun_out/tb_bench.log 2>&1 || exit 7
exit 0
