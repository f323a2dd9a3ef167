#!/bin/bash
# Depthwise row pipeline: depthwise tests, then the SSD bench with the per-op dump (twice).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3x.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dwconv" > gpurun_out/r3x_t.log 2>&1 || { echo "tests failed" >> gpurun_out/r3x.txt; tail -20 gpurun_out/r3x_t.log >> gpurun_out/r3x.txt; exit 1; }
echo "tests $(tail -1 gpurun_out/r3x_t.log)" >> gpurun_out/r3x.txt
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --model ssd --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r3x_ops.json > gpurun_out/r3x_b.log 2>&1 || exit 1
  echo "$(tail -1 gpurun_out/r3x_b.log | cut -c100-190)" >> gpurun_out/r3x.txt
done
python3 -c "
import json; d=json.load(open('gpurun_out/r3x_ops.json'))['ssd']
fam={}
for o in d: fam[o['family']]=fam.get(o['family'],0)+o['ms']
print({k:round(v,4) for k,v in fam.items()})" >> gpurun_out/r3x.txt
