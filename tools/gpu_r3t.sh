#!/bin/bash
# uint8 preprocess lookup table: u8 == float paths (pipeline tests), SSD bench with the per-op dump.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3t.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_jpeg.py tests/test_gpu_kernels.py -k "run_batches or decode or preprocess or transform" > gpurun_out/r3t_t.log 2>&1 || { echo "tests failed" >> gpurun_out/r3t.txt; tail -30 gpurun_out/r3t_t.log >> gpurun_out/r3t.txt; exit 1; }
echo "tests $(tail -1 gpurun_out/r3t_t.log)" >> gpurun_out/r3t.txt
timeout -k 10 300 python -u bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/r3t_ops.json > gpurun_out/r3t_bench.log 2>&1 || exit 4
tail -1 gpurun_out/r3t_bench.log | cut -c100-200 >> gpurun_out/r3t.txt
