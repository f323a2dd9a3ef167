#!/bin/bash
# Round-3 SSD step A/B: parity of the fused InvertedResidual and the grouped small-heads launch, then
# the SSD bench over EDGEDET_MB_BLOCK x EDGEDET_SSD_HEADS (per-op times dumped), then the ingest bench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_models.py > gpurun_out/r3c_test.log 2>&1 || { echo "tests failed" >> gpurun_out/r3c.txt; exit 1; }
echo "tests ok" >> gpurun_out/r3c.txt
for cfg in "0 0" "0 1" "1 1" "1 0"; do
  set -- $cfg
  EDGEDET_MB_BLOCK=$1 EDGEDET_SSD_HEADS=$2 timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --no-alt \
      --dump-ops gpurun_out/ops_mb$1_h$2.json > gpurun_out/bench_mb$1_h$2.log 2>&1 || { echo "bench $cfg failed" >> gpurun_out/r3c.txt; exit 1; }
  echo "mb=$1 heads=$2 $(tail -1 gpurun_out/bench_mb$1_h$2.log | cut -c1-200)" >> gpurun_out/r3c.txt
done
timeout -k 10 300 python -u bench.py --model frcnn --no-cpu --no-e2e --dump-ops gpurun_out/ops_frcnn.json > gpurun_out/bench_frcnn.log 2>&1 || { echo "frcnn bench failed" >> gpurun_out/r3c.txt; exit 1; }
echo "frcnn $(tail -1 gpurun_out/bench_frcnn.log | cut -c1-300)" >> gpurun_out/r3c.txt
timeout -k 10 600 python -u tools/ingest_bench.py --n 2000 > gpurun_out/ingest.log 2>&1; echo "ingest rc=$?" >> gpurun_out/r3c.txt
