#!/bin/bash
# A/B of the pointwise conv_x6b specialisation (EDGEDET_X6B_P1): kernel tests, tile microbench on the
# SSD 1x1 shapes and the SSD/FRCNN bench, both ways.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bf16x6" > gpurun_out/p1_pytest.log 2>&1 || exit 5
: > gpurun_out/p1.log
for rep in 1 2; do
for v in 0 1; do
  EDGEDET_X6B_P1=$v timeout -k 10 300 python tools/conv_bench.py --tiles 29,31 --shapes ssd_head_cls0,ssd_f13,ssd_12_3,ssd_head_cls1 --reps 50 | sed "s/^/P1=$v /" >> gpurun_out/p1.log 2>&1 || exit 6
  EDGEDET_X6B_P1=$v timeout -k 10 300 python bench.py --model both --steps 600 --warmup 20 --no-cpu --no-e2e 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('P1=$v bench ssd', d['value'], 'frcnn', d['frcnn']['value'])" >> gpurun_out/p1.log || exit 7
done
done
exit 0
