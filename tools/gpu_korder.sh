#!/bin/bash
# A/B of the conv_x6b_kernel K stage order (EDGEDET_X6B_KORDER): conv kernel tests, tile-25
# microbench on the 3x3 shapes, FRCNN bench, both orders.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "x6 or bf16 or conv" > gpurun_out/ko_pytest.log 2>&1 || exit 5
for ko in 0 1; do
  EDGEDET_X6B_KORDER=$ko timeout -k 10 300 python tools/conv_bench.py --tiles 25 --shapes box_head_3x3,fpn_p2_3x3,layer3_3x3,layer4_3x3 > gpurun_out/ko_conv_$ko.log 2>&1 || exit 6
  EDGEDET_X6B_KORDER=$ko timeout -k 10 300 python bench.py --model frcnn --steps 40 --warmup 10 --no-cpu --no-e2e > gpurun_out/ko_bench_$ko.log 2>&1 || exit 7
done
exit 0
