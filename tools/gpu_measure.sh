#!/bin/bash
# Measurement extras: a kernel trace of the bench with one batch in flight and the roofline launch
# cross-check against it, the MFMA utilisation passes, and the SSD op-family skip diagnostic.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_if1 -o trace -- python3 bench.py --model both --no-cpu --no-e2e --inflight 1 --steps 200 > gpurun_out/prof_if1.log 2>&1 || exit 5
python3 tools/roofline_check.py gpurun_out/prof_if1 gpurun_out/prof_if1.log -o gpurun_out/roofline_check.json > /dev/null || exit 6
bash tools/gpu_mfma.sh || exit 7
SKIPS="${SKIPS:-none 3 4 6 17 129 133,134,135 121,128,101}" bash tools/gpu_skip.sh || exit 8
exit 0
