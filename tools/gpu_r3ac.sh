#!/bin/bash
# FRCNN with the RPN head on one stream: FRCNN / native-model / pipeline / distributed tests, FRCNN bench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3ac.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_parity_configs.py tests/test_gpu_native_model.py tests/test_gpu_pipeline.py tests/test_gpu_distributed.py tests/test_gpu_lanes.py > gpurun_out/r3ac_t.log 2>&1 || { echo "tests failed" >> gpurun_out/r3ac.txt; tail -30 gpurun_out/r3ac_t.log >> gpurun_out/r3ac.txt; exit 1; }
echo "tests $(tail -1 gpurun_out/r3ac_t.log)" >> gpurun_out/r3ac.txt
timeout -k 10 300 python -u bench.py --model frcnn --no-cpu --no-e2e > gpurun_out/r3ac_b.log 2>&1 || exit 2
tail -1 gpurun_out/r3ac_b.log | cut -c90-200 >> gpurun_out/r3ac.txt
