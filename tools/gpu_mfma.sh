#!/bin/bash
# MFMA utilisation of the conv kernels (tools/mfma_util.py) for both models, one PMC pass each.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for m in ssd frcnn; do
  rm -rf /tmp/mfma_$m
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/mfma_$m -o m -- \
    python3 bench.py --model $m --steps 4 --warmup 1 --no-cpu --no-e2e --no-roofline --inflight 1 > gpurun_out/mfma_$m.log 2>&1 || exit 5
  python3 tools/mfma_util.py /tmp/mfma_$m --model $m > gpurun_out/mfma_util_$m.txt 2>&1 || exit 6
done
exit 0
