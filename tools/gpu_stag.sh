#!/bin/bash
# A/B of conv_x6b_kernel variants: kernel tests on every build, then the tile-25 microbench and the
# FRCNN bench on the default build (arm "base") and on build/variants/lib_$v.so for v in $VARS.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
VARS=${VARS:-stag2 stag3}
for v in base $VARS; do
  if [ $v = base ]; then unset EDGEDET_LIB; else export EDGEDET_LIB=build/variants/lib_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "x6 or bf16" > gpurun_out/st_pytest_$v.log 2>&1 || exit 5
done
for rep in 1 2; do
  for v in base $VARS; do
    if [ $v = base ]; then unset EDGEDET_LIB; else export EDGEDET_LIB=build/variants/lib_$v.so; fi
    timeout -k 10 300 python tools/conv_bench.py --tiles 25 --shapes box_head_3x3,fpn_p2_3x3,layer3_3x3 >> gpurun_out/st_conv_$v.log 2>&1 || exit 6
    timeout -k 10 300 python bench.py --model frcnn --steps 40 --warmup 10 --no-cpu --no-e2e >> gpurun_out/st_bench_$v.log 2>&1 || exit 7
  done
done
exit 0
