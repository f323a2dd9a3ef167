#!/bin/bash
# Full GPU test suite, smoke, default bench (both models), and the ingest bench at config-4 size with
# the detect CLI's phase times.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3i.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3i_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/r3i_pytest_gpu.log)" >> gpurun_out/r3i.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3i_smoke.log 2>&1 || { echo "smoke failed" >> gpurun_out/r3i.txt; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r3i_bench.log 2>&1 || { echo "bench failed" >> gpurun_out/r3i.txt; exit 1; }
echo "bench $(tail -1 gpurun_out/r3i_bench.log | cut -c1-300)" >> gpurun_out/r3i.txt
EDGEDET_DETECT_TIMING=1 timeout -k 10 600 python -u -X faulthandler tools/ingest_bench.py --n 5000 > gpurun_out/r3i_ingest.log 2>&1; echo "ingest rc=$?" >> gpurun_out/r3i.txt
