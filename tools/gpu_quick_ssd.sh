#!/bin/bash
# Quick SSD check: depthwise/SE kernel tests, then the SSD bench with the per-op dump.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${K:-dw or se}" > gpurun_out/q_pytest.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/ops_ssd.json > gpurun_out/q_bench.log 2>&1 || exit 7
exit 0
