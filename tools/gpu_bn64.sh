#!/bin/bash
# 128 x 64 x6b tile (38): bf16x6 kernel tests, conv microbench on the Cout = 64 shapes, FRCNN re-tune
# and the bench on the committed and the re-tuned table.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bf16x6" > gpurun_out/bn64_pytest.log 2>&1 || exit 5
timeout -k 10 300 python tools/conv_bench.py --tiles 27,31,38 --shapes layer1_3x3,layer1_1x1_in,stem_7x7,ssd_02_project --reps 20 > gpurun_out/bn64_conv.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --model both --no-cpu --no-e2e 2>/dev/null | grep '"metric"' > gpurun_out/bn64_bench_old.json || exit 7
cp edgeml-object-detection_amd/data/conv_tiles_gfx950.json gpurun_out/tiles_bn64.json
timeout -k 10 900 python -u tools/tune_conv.py --models frcnn,ssd --out gpurun_out/tiles_bn64.json > gpurun_out/bn64_tune.log 2>&1 || exit 8
cp gpurun_out/tiles_bn64.json edgeml-object-detection_amd/data/conv_tiles_gfx950.json
timeout -k 10 300 python bench.py --model both --no-cpu --no-e2e 2>/dev/null | grep '"metric"' > gpurun_out/bn64_bench_new.json || exit 9
exit 0
