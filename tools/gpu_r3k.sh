#!/bin/bash
# Batched native entropy decode: JPEG / pipeline GPU tests, then the ingest anatomy at config-4 size.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3k.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_jpeg.py tests/test_gpu_pipeline.py > gpurun_out/r3k_test.log 2>&1 || { echo "tests failed" >> gpurun_out/r3k.txt; exit 1; }
echo "tests ok $(tail -1 gpurun_out/r3k_test.log)" >> gpurun_out/r3k.txt
EDGEDET_DETECT_TIMING=1 timeout -k 10 400 python -u -X faulthandler tools/ingest_bench.py --n 5000 > gpurun_out/r3k_ingest.log 2>&1 || { echo "ingest failed" >> gpurun_out/r3k.txt; exit 1; }
echo ok >> gpurun_out/r3k.txt
