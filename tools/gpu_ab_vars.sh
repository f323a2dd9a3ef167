#!/bin/bash
# A/B over library variants (build/variants/lib_$v.so for v in $VARS): x6b kernel tests on each,
# then the device-rate bench (both models) for the default build and each variant, interleaved twice.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/ab_vars.log
for v in $VARS; do
  EDGEDET_LIB=build/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${K:-bf16x6}" > gpurun_out/ab_pytest_$v.log 2>&1 || exit 5
done
for rep in 1 2; do
for v in base $VARS; do
  if [ $v = base ]; then unset EDGEDET_LIB; else export EDGEDET_LIB=build/variants/lib_$v.so; fi
  timeout -k 10 300 python bench.py --model both --no-cpu --no-e2e 2>/dev/null | grep '"metric"' > gpurun_out/ab_bench_$v.json || exit 7
  python3 -c "import json; d=json.load(open('gpurun_out/ab_bench_$v.json')); print('$v', 'ssd', d['value'], d['ms_per_step'], 'frcnn', d['frcnn']['value'], d['frcnn']['ms_per_step'], 'boxhead_ms', d['frcnn']['roofline']['launch_ms'], 'ssd_roof_ms', d['roofline']['launch_ms'])" >> gpurun_out/ab_vars.log
done
done
exit 0
