#!/bin/bash
# New-tile check and re-tune: the bf16x6 kernel tests, then tools/tune_conv.py over $MODELS
# (merging into a copy of the committed table, written to gpurun_out/tiles_new.json).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bf16x6" > gpurun_out/tune_pytest.log 2>&1 || exit 5
cp edgeml-object-detection_amd/data/conv_tiles_gfx950.json gpurun_out/tiles_new.json
timeout -k 10 900 python -u tools/tune_conv.py --models ${MODELS:-ssd,frcnn} --out gpurun_out/tiles_new.json > gpurun_out/tune.log 2>&1 || exit 6
exit 0
