#!/bin/bash
# FRCNN step anatomy (diagnostic skips, results wrong): RPN NMS, RoIAlign, box scores + NMS, merge, maxpool.
cd "$GRAFT_REPO_ROOT" || exit 9
MODEL=frcnn SKIPS="none 11 12 13,14 10 7 none" STEPS=300 bash tools/gpu_skip.sh || exit 6
cp gpurun_out/skip.log gpurun_out/r3y_skip.log
