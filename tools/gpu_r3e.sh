#!/bin/bash
# Grouped SSD heads (prefetched, register-blocked) parity + A/B; the ingest bench under faulthandler.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py -k "grouped or ssd" > gpurun_out/r3e_test.log 2>&1 || { echo "tests failed" >> gpurun_out/r3e.txt; exit 1; }
echo "tests ok" >> gpurun_out/r3e.txt
for h in 1 0; do
  EDGEDET_SSD_HEADS=$h timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --no-alt \
      --dump-ops gpurun_out/ops_h$h.json > gpurun_out/bench_h$h.log 2>&1 || { echo "bench $h failed" >> gpurun_out/r3e.txt; exit 1; }
  echo "heads=$h $(tail -1 gpurun_out/bench_h$h.log | cut -c1-200)" >> gpurun_out/r3e.txt
done
bash tools/gpu_r3d.sh; echo "r3d rc=$?" >> gpurun_out/r3e.txt
timeout -k 10 400 python -u -X faulthandler tools/ingest_bench.py --n 400 > gpurun_out/ingest.log 2>&1; echo "ingest rc=$?" >> gpurun_out/r3e.txt
