#!/bin/bash
# A/B of the fused InvertedResidual (MBCONV, csrc/layers.hip mbconv_kernel) on SSDLite blocks 0.2 / 0.3:
# the unit test, then the SSD bench with EDGEDET_MB_BLOCK=0 / 1 alternated (per-op times dumped).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k mbconv_block -q > gpurun_out/mb_test.log 2>&1 || exit 1
for v in 0 1 0 1; do
  EDGEDET_MB_BLOCK=$v timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --no-alt \
      --dump-ops gpurun_out/ops_mb$v.json > gpurun_out/mb_bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/mb_bench_$v.log | cut -c1-160 >> gpurun_out/mb_ab.txt
done
