#!/bin/bash
# MBConv ablations (EDGEDET_MB_DIAG, wrong results): which phase the time goes to.
cd "$GRAFT_REPO_ROOT" || exit 9
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for d in 0 1 2 3 4 8 12 15; do
  echo "diag=$d $(EDGEDET_MB_DIAG=$d timeout -k 10 60 python -u tools/mb_bench.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
done
