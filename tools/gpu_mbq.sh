#!/bin/bash
# MBConv quick loop: kernel tests + microbench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k mbconv > gpurun_out/mbq_t.log 2>&1 || { tail -30 gpurun_out/mbq_t.log; exit 1; }
tail -1 gpurun_out/mbq_t.log
timeout -k 10 120 python -u tools/mb_bench.py 2>&1 | grep -v amdgpu.ids
