#!/bin/bash
# FRCNN with three batches in flight: pipeline / distributed tests, FRCNN bench with the end-to-end leg.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3ag.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_distributed.py tests/test_gpu_jpeg.py tests/test_gpu_retinanet.py > gpurun_out/r3ag_t.log 2>&1 || { echo "tests failed" >> gpurun_out/r3ag.txt; tail -30 gpurun_out/r3ag_t.log >> gpurun_out/r3ag.txt; exit 1; }
echo "tests $(tail -1 gpurun_out/r3ag_t.log)" >> gpurun_out/r3ag.txt
timeout -k 10 300 python -u bench.py --model frcnn --no-cpu > gpurun_out/r3ag_b.log 2>&1 || exit 2
tail -1 gpurun_out/r3ag_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['end_to_end']['value'], d['roofline']['frac'])" >> gpurun_out/r3ag.txt
