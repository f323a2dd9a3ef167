#!/bin/bash
# SSD step anatomy on the round-3 tree (diagnostic skips, results wrong): what each family costs the
# steady-state step under 4 batches in flight.
cd "$GRAFT_REPO_ROOT" || exit 9
SKIPS="none 3 4 6 17 22 21 8,2 129 3,4,6,17,22,21,8,2" STEPS=400 bash tools/gpu_skip.sh || exit 6
cp gpurun_out/skip.log gpurun_out/r3l_skip.log
