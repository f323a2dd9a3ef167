#!/bin/bash
# BASELINE configs[3] at full size on one GPU (5,000 synthetic COCO-size JPEGs: SSDLite weak files,
# FRCNN strong files, ORIE E=1000) with the GPU JPEG path, phase times, and ORIE parity on a subset.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp EDGEDET_DETECT_TIMING=1
timeout -k 10 900 python -u tools/config4_full.py --n 5000 --subset 60 > gpurun_out/r3s_config4.log 2>&1; echo "rc=$?" >> gpurun_out/r3s_config4.log
