#!/bin/bash
# Two-register-stage tiles (30 / 32) in the 16x16x32 form: x6b tests, conv microbench, re-tune of
# both models and the bench on the committed and on the re-tuned table.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bf16x6" > gpurun_out/pf2_pytest.log 2>&1 || exit 5
timeout -k 10 300 python tools/conv_bench.py --tiles 29,30,31,32 --shapes ssd_head_cls0,ssd_head_cls1,ssd_f13,layer3_3x3 --reps 50 > gpurun_out/pf2_conv.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --model both --no-cpu --no-e2e 2>/dev/null | grep '"metric"' > gpurun_out/pf2_bench_old.json || exit 7
cp edgeml-object-detection_amd/data/conv_tiles_gfx950.json gpurun_out/tiles_pf2.json
timeout -k 10 900 python -u tools/tune_conv.py --models ssd,frcnn --out gpurun_out/tiles_pf2.json > gpurun_out/pf2_tune.log 2>&1 || exit 8
cp gpurun_out/tiles_pf2.json edgeml-object-detection_amd/data/conv_tiles_gfx950.json
timeout -k 10 300 python bench.py --model both --no-cpu --no-e2e 2>/dev/null | grep '"metric"' > gpurun_out/pf2_bench_new.json || exit 9
exit 0
