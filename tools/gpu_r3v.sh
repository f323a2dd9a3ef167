#!/bin/bash
# SSD step anatomy on the current tree (diagnostic skips, results wrong).
cd "$GRAFT_REPO_ROOT" || exit 9
SKIPS="none 3 4 6 17 22 21 8 129 none" STEPS=400 bash tools/gpu_skip.sh || exit 6
cp gpurun_out/skip.log gpurun_out/r3v_skip.log
