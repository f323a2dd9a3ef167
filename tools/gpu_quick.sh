#!/bin/bash
# Short GPU iteration: GPU tests (optionally filtered) + bench.  Usage: gpu_quick.sh [pytest -k expr] [bench args]
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
K=${1:-}
shift
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/quick_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/quick_pytest.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/quick_bench.log 2>&1
  rc=$?; tail -2 gpurun_out/quick_bench.log | cut -c1-3000
  exit $rc
fi
