#!/bin/bash
# Check-then-measure: the GPU tests matching $PYTEST_K (stop on any failure or crash), then an ABBA
# A/B of $VAR over $VALUES (tools/gpu_ab.sh), then optionally the session of record ($ROUND=1).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "$PYTEST_K" --timeout 120 --timeout-method thread > gpurun_out/pytest_check.log 2>&1
rc=$?
[ $rc -ne 0 ] && { echo "check tests rc=$rc: stopping" >> gpurun_out/pytest_check.log; exit 3; }
bash tools/gpu_ab.sh || exit 4
cp gpurun_out/ab.log gpurun_out/ab_${VAR}.log
[ "${ROUND:-0}" = "1" ] && { TESTS=1 bash tools/gpu_round.sh || exit 5; }
exit 0
