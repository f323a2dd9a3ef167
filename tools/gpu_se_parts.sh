#!/bin/bash
# SE partial-sum splits (SE_PARTS 32): SE / depthwise / model tests, then the SSD bench with the per-op dump.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_native_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sep_pytest.log 2>&1 || exit 5
for rep in 1 2; do
timeout -k 10 300 python bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/sep_ops_$rep.json 2>/dev/null | grep '"metric"' > gpurun_out/sep_bench_$rep.json || exit 6
done
exit 0
