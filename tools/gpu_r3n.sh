#!/bin/bash
# Wave-per-chunk fused MBConv: kernel tests, microbench, SSD model parity, SSD bench with per-op dump.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3n.txt
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k mbconv > gpurun_out/r3n_t0.log 2>&1 || { echo "kernel tests failed" >> gpurun_out/r3n.txt; exit 1; }
timeout -k 10 120 python -u tools/mb_bench.py >> gpurun_out/r3n.txt 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_parity_configs.py -k "ssd or SSD" > gpurun_out/r3n_t1.log 2>&1 || { echo "model tests failed" >> gpurun_out/r3n.txt; exit 3; }
echo "models ok $(tail -1 gpurun_out/r3n_t1.log)" >> gpurun_out/r3n.txt
timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/r3n_ops.json > gpurun_out/r3n_bench.log 2>&1 || { echo "bench failed" >> gpurun_out/r3n.txt; exit 4; }
tail -1 gpurun_out/r3n_bench.log | cut -c1-400 >> gpurun_out/r3n.txt
