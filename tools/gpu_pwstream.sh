#!/bin/bash
# Streaming pointwise tiles (33-35): kernel tests, SSD re-tune with the new candidates, bench on the
# committed table and on the re-tuned one.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "pointwise_stream or bf16x6 or direct_pointwise or matches_torch" > gpurun_out/pws_pytest.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/pws_ops_old.json 2>/dev/null | grep '"metric"' > gpurun_out/pws_bench_old.json || exit 6
cp edgeml-object-detection_amd/data/conv_tiles_gfx950.json gpurun_out/tiles_new.json
timeout -k 10 900 python -u tools/tune_conv.py --models ${MODELS:-ssd} --out gpurun_out/tiles_new.json > gpurun_out/pws_tune.log 2>&1 || exit 7
cp gpurun_out/tiles_new.json edgeml-object-detection_amd/data/conv_tiles_gfx950.json
timeout -k 10 300 python bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/pws_ops_new.json 2>/dev/null | grep '"metric"' > gpurun_out/pws_bench_new.json || exit 8
exit 0
