#!/bin/bash
# SSD A/B: grouped small heads (EDGEDET_SSD_HEADS) on / off, alternated.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3p.txt
for v in 0 1 0 1; do
  EDGEDET_SSD_HEADS=$v timeout -k 10 200 python -u bench.py --model ssd --no-cpu --no-e2e --no-roofline > gpurun_out/r3p_$v.log 2>&1 || exit 1
  echo "heads=$v $(tail -1 gpurun_out/r3p_$v.log | cut -c100-200)" >> gpurun_out/r3p.txt
done
