#!/bin/bash
# Ingest phase anatomy (detect CLI, SSDLite, 5000 synthetic COCO JPEGs, GPU decode) and the per-op
# device times of both models (bench --dump-ops).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3j.txt
EDGEDET_DETECT_TIMING=1 timeout -k 10 400 python -u -X faulthandler tools/ingest_bench.py --n 5000 > gpurun_out/r3j_ingest.log 2>&1 || { echo "ingest failed" >> gpurun_out/r3j.txt; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-alt --steps 300 --dump-ops gpurun_out/r3j_ops.json > gpurun_out/r3j_bench.log 2>&1 || { echo "bench failed" >> gpurun_out/r3j.txt; exit 1; }
echo ok >> gpurun_out/r3j.txt
