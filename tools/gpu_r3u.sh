#!/bin/bash
# Transform folded into the SSD stem: kernel + model parity tests, SSD bench with the per-op dump.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3u.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "stem" > gpurun_out/r3u_t0.log 2>&1 || { echo "kernel tests failed" >> gpurun_out/r3u.txt; tail -30 gpurun_out/r3u_t0.log >> gpurun_out/r3u.txt; exit 1; }
echo "kernels $(tail -1 gpurun_out/r3u_t0.log)" >> gpurun_out/r3u.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_parity_configs.py tests/test_gpu_pipeline.py tests/test_gpu_native_model.py > gpurun_out/r3u_t1.log 2>&1 || { echo "model tests failed" >> gpurun_out/r3u.txt; tail -30 gpurun_out/r3u_t1.log >> gpurun_out/r3u.txt; exit 3; }
echo "models $(tail -1 gpurun_out/r3u_t1.log)" >> gpurun_out/r3u.txt
for i in 1 2; do
timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/r3u_ops.json > gpurun_out/r3u_bench.log 2>&1 || { echo "bench failed" >> gpurun_out/r3u.txt; exit 4; }
tail -1 gpurun_out/r3u_bench.log | cut -c100-200 >> gpurun_out/r3u.txt
done
