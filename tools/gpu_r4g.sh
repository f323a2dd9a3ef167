#!/bin/bash
# Round-4 session g: BASELINE configs[3] at full size on one GPU (tools/config4_full.py: 5,000
# synthetic COCO-size JPEGs -> weak + strong files -> ORIE E = 1,000; identity-paired parity on a
# 60-image subset against the CPU oracle pipeline).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 1000 python -u tools/config4_full.py --subset 60 --work /tmp/c4 > gpurun_out/config4_full.log 2>&1
echo "rc=$?" >> gpurun_out/config4_full.log
exit 0
