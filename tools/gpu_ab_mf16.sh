#!/bin/bash
# A/B of the 16x16x32 bf16x6 form (X6B_MF16=1, build/variants/lib_mf16.so) against the default
# build: x6b kernel tests on the variant, conv microbench and the device-rate bench for both.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/ab_mf16.log
export EDGEDET_LIB=build/variants/lib_${VAR:-mf16}.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${K:-bf16x6 or every_lds}" > gpurun_out/ab_pytest.log 2>&1 || exit 5
for v in base ${VAR:-mf16}; do
  if [ $v = base ]; then unset EDGEDET_LIB; else export EDGEDET_LIB=build/variants/lib_$v.so; fi
  timeout -k 10 300 python tools/conv_bench.py --tiles ${TILES:-25,29,31} --shapes ${SHAPES:-box_head_3x3,fpn_p2_3x3,layer3_3x3,ssd_head_cls0,ssd_f13} > gpurun_out/ab_conv_$v.log 2>&1 || exit 6
  timeout -k 10 300 python bench.py --model both --no-cpu --no-e2e 2>/dev/null | grep '"metric"' > gpurun_out/ab_bench_$v.json || exit 7
  python3 -c "import json; d=json.load(open('gpurun_out/ab_bench_$v.json')); print('$v', 'ssd', d['value'], d['ms_per_step'], 'frcnn', d['frcnn']['value'], d['frcnn']['ms_per_step'], 'boxhead_ms', d['frcnn']['roofline']['launch_ms'], 'ssd_roof_ms', d['roofline']['launch_ms'])" >> gpurun_out/ab_mf16.log
done
exit 0
