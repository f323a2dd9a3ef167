#!/bin/bash
# MBConv ablations (EDGEDET_MB_DIAG, wrong results) and resident-grid A/B (EDGEDET_MB_PER_CU).
cd "$GRAFT_REPO_ROOT" || exit 9
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for pc in 0 1 3 4 8 64; do
for d in ${DIAGS:-0 15}; do
  echo "per_cu=$pc diag=$d $(EDGEDET_MB_PER_CU=$pc EDGEDET_MB_DIAG=$d timeout -k 10 60 python -u tools/mb_bench.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
done
done
