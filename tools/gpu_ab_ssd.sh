#!/bin/bash
# SSD A/B over library variants: bench (device rate) + per-op dump for the default build and each
# build/variants/lib_$v.so in $VARS.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/ab_ssd.log
for v in base $VARS; do
  if [ $v = base ]; then unset EDGEDET_LIB; else export EDGEDET_LIB=build/variants/lib_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${K:-dw}" > gpurun_out/ab_pytest_$v.log 2>&1 || exit 5
  timeout -k 10 300 python bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/ab_ops_$v.json 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" >> gpurun_out/ab_ssd.log || exit 7
done
exit 0
