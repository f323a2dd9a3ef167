#!/bin/bash
# SSD sweep on the round-3 tree: batch chains x batches in flight.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3q.txt
for cfg in "2 3" "2 4" "2 5" "2 6" "4 2" "4 3" "1 6"; do
  set -- $cfg
  EDGEDET_SSD_CHAINS=$1 timeout -k 10 200 python -u bench.py --model ssd --no-cpu --no-e2e --no-roofline --no-alt --inflight $2 > gpurun_out/r3q_$1_$2.log 2>&1 || exit 1
  echo "chains=$1 inflight=$2 $(tail -1 gpurun_out/r3q_$1_$2.log | cut -c100-190)" >> gpurun_out/r3q.txt
done
