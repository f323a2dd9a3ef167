#!/bin/bash
# Fused MBConv microbench: launch times, then the stall picture from two rocprofv3 PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 120 python -u tools/mb_bench.py > gpurun_out/r3m_mb.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  --output-format csv -d gpurun_out/r3m_p1 -o c -- python3 tools/mb_bench.py --reps 5 > gpurun_out/r3m_p1.log 2>&1 || exit 2
python3 tools/pmc_kernels.py gpurun_out/r3m_p1 --raw --top 4 > gpurun_out/r3m_pmc.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS \
  --output-format csv -d gpurun_out/r3m_p2 -o c -- python3 tools/mb_bench.py --reps 5 > gpurun_out/r3m_p2.log 2>&1 || exit 3
python3 tools/pmc_kernels.py gpurun_out/r3m_p2 --raw --top 4 >> gpurun_out/r3m_pmc.txt 2>&1
exit 0
