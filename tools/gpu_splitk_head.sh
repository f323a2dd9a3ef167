#!/bin/bash
# Split-K 128x128 / 64x128 tiles (36 / 37): tests, then the SSD cls-head shapes in the conv microbench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "split_k" > gpurun_out/sk_pytest.log 2>&1 || exit 5
timeout -k 10 300 python tools/conv_bench.py --tiles 29,31,26,36,37 --shapes ssd_head_cls0,ssd_head_cls1,ssd_f13 --reps 50 > gpurun_out/sk_conv.log 2>&1 || exit 6
exit 0
