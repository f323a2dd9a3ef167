#!/bin/bash
# Grouped SSD heads with a real prefetch: head tests, then the SSD A/B (EDGEDET_SSD_HEADS off / on).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3w.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_models.py -k "head or ssd" > gpurun_out/r3w_t.log 2>&1 || { echo "tests failed" >> gpurun_out/r3w.txt; tail -20 gpurun_out/r3w_t.log >> gpurun_out/r3w.txt; exit 1; }
echo "tests $(tail -1 gpurun_out/r3w_t.log)" >> gpurun_out/r3w.txt
EDGEDET_SSD_HEADS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_parity_configs.py -k "ssd or SSD" > gpurun_out/r3w_t2.log 2>&1 || { echo "heads=1 tests failed" >> gpurun_out/r3w.txt; tail -20 gpurun_out/r3w_t2.log >> gpurun_out/r3w.txt; exit 1; }
echo "heads=1 tests $(tail -1 gpurun_out/r3w_t2.log)" >> gpurun_out/r3w.txt
for v in 0 1 0 1; do
  EDGEDET_SSD_HEADS=$v timeout -k 10 200 python -u bench.py --model ssd --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r3w_ops$v.json > gpurun_out/r3w_$v.log 2>&1 || exit 1
  echo "heads=$v $(tail -1 gpurun_out/r3w_$v.log | cut -c100-190)" >> gpurun_out/r3w.txt
done
