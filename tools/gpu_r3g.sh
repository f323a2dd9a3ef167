#!/bin/bash
# 8-wave fused MBConv + 16-byte SE staging: parity, SSD A/B (MBConv on / off), the step with SE /
# MBConv left out, then the config-4 pipeline stages (5000 synthetic COCO JPEGs, GPU decode).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3g.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "mbconv or se_ or squeeze" > gpurun_out/r3g_test0.log 2>&1 || { echo "kernel tests failed" >> gpurun_out/r3g.txt; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py > gpurun_out/r3g_test.log 2>&1 || { echo "model tests failed" >> gpurun_out/r3g.txt; exit 1; }
echo "tests ok" >> gpurun_out/r3g.txt
for mb in 1 0; do
  EDGEDET_MB_BLOCK=$mb timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --no-alt \
      --dump-ops gpurun_out/ops_g_mb$mb.json > gpurun_out/bench_g_mb$mb.log 2>&1 || { echo "bench mb=$mb failed" >> gpurun_out/r3g.txt; exit 1; }
  echo "mb=$mb $(tail -1 gpurun_out/bench_g_mb$mb.log | cut -c1-200)" >> gpurun_out/r3g.txt
done
EDGEDET_MB_BLOCK=1 SKIPS="none 6 22 3" STEPS=400 bash tools/gpu_skip.sh || exit 6
timeout -k 10 600 python -u tools/config4_full.py --n 5000 --subset 0 > gpurun_out/r3g_config4.log 2>&1; echo "config4 rc=$?" >> gpurun_out/r3g.txt
