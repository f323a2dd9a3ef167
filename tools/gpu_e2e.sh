#!/bin/bash
# run_batches check: pipeline tests (bit-identity vs model(images)) and the end-to-end rates.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_native_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/e2e_pytest.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --model both --no-cpu --steps 300 > gpurun_out/e2e_bench.log 2>&1 || exit 7
exit 0
