#!/bin/bash
# FRCNN A/B: conv_x6b young-half priority (EDGEDET_X6B_PRIO) off / on, alternated.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3r.txt
for v in 0 1 0 1; do
  EDGEDET_X6B_PRIO=$v timeout -k 10 200 python -u bench.py --model frcnn --no-cpu --no-e2e --no-roofline > gpurun_out/r3r_$v.log 2>&1 || exit 1
  echo "prio=$v $(tail -1 gpurun_out/r3r_$v.log | cut -c90-190)" >> gpurun_out/r3r.txt
done
