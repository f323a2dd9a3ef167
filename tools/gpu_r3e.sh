#!/bin/bash
# Grouped SSD heads / fused MBConv (prefetched chunk operands) parity + A/B; conv picture; the ingest
# bench under faulthandler.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "mbconv or bf16x6" > gpurun_out/r3e_test0.log 2>&1 || { echo "kernel tests failed" >> gpurun_out/r3e.txt; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py -k "grouped or ssd" > gpurun_out/r3e_test.log 2>&1 || { echo "model tests failed" >> gpurun_out/r3e.txt; exit 1; }
echo "tests ok" >> gpurun_out/r3e.txt
for cfg in "1 0" "1 1" "0 0"; do
  set -- $cfg
  EDGEDET_SSD_HEADS=$1 EDGEDET_MB_BLOCK=$2 timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --no-alt \
      --dump-ops gpurun_out/ops_h$1_mb$2.json > gpurun_out/bench_h$1_mb$2.log 2>&1 || { echo "bench $cfg failed" >> gpurun_out/r3e.txt; exit 1; }
  echo "heads=$1 mb=$2 $(tail -1 gpurun_out/bench_h$1_mb$2.log | cut -c1-200)" >> gpurun_out/r3e.txt
done
bash tools/gpu_r3d.sh; echo "r3d rc=$?" >> gpurun_out/r3e.txt
timeout -k 10 400 python -u -X faulthandler tools/ingest_bench.py --n 400 > gpurun_out/ingest.log 2>&1; echo "ingest rc=$?" >> gpurun_out/r3e.txt
