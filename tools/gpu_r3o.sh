#!/bin/bash
# SE squeeze means once per launch: SE / model tests, then the SSD bench with the per-op dump.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3o.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "se_ or dwconv" > gpurun_out/r3o_t0.log 2>&1 || { echo "kernel tests failed" >> gpurun_out/r3o.txt; tail -20 gpurun_out/r3o_t0.log >> gpurun_out/r3o.txt; exit 1; }
echo "kernels $(tail -1 gpurun_out/r3o_t0.log)" >> gpurun_out/r3o.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_parity_configs.py > gpurun_out/r3o_t1.log 2>&1 || { echo "model tests failed" >> gpurun_out/r3o.txt; exit 3; }
echo "models $(tail -1 gpurun_out/r3o_t1.log)" >> gpurun_out/r3o.txt
timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/r3o_ops.json > gpurun_out/r3o_bench.log 2>&1 || { echo "bench failed" >> gpurun_out/r3o.txt; exit 4; }
tail -1 gpurun_out/r3o_bench.log | cut -c1-200 >> gpurun_out/r3o.txt
