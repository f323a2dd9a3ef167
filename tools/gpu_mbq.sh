#!/bin/bash
# MBConv quick loop: kernel tests + microbench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k mbconv > gpurun_out/mbq_t.log 2>&1 || { tail -30 gpurun_out/mbq_t.log; exit 1; }
tail -1 gpurun_out/mbq_t.log
timeout -k 10 120 python -u tools/mb_bench.py 2>&1 | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  --output-format csv -d gpurun_out/mbq_p1 -o c -- python3 tools/mb_bench.py --reps 5 > gpurun_out/mbq_p1.log 2>&1 || exit 2
python3 tools/pmc_kernels.py gpurun_out/mbq_p1 --raw --top 2
