#!/bin/bash
# Two-register-stage x6b tiles (30, 32) against the skewed tiles (29, 31, 25) on the shapes the table
# serves: conv microbench.
cd "$GRAFT_REPO_ROOT" || exit 9
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_bench.py --tiles 25,29,30,31,32 --shapes ssd_head_cls0,ssd_head_cls1,ssd_f13,ssd_12_3,layer3_3x3,layer4_3x3,box_head_3x3 --reps 10 2>&1 | grep -v amdgpu.ids
