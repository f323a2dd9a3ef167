#!/bin/bash
# round-5 session y: stall picture of the FRCNN kernels (one plan in flight, so launches run alone):
# two SQ passes over a short SSD bench, reduced per kernel by tools/pmc_kernels.py --raw
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
B="python3 bench.py --model frcnn --steps 3 --warmup 1 --no-cpu --no-e2e --no-roofline --inflight 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d gpurun_out/r5y_sq1 -o s -- $B > gpurun_out/r5y_sq1.log 2>&1 || exit 5
python3 tools/pmc_kernels.py gpurun_out/r5y_sq1 --raw --top 25 > gpurun_out/r5y_sq1.txt 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/r5y_sq2 -o s -- $B > gpurun_out/r5y_sq2.log 2>&1 || exit 6
python3 tools/pmc_kernels.py gpurun_out/r5y_sq2 --raw --top 25 > gpurun_out/r5y_sq2.txt 2>&1
rm -rf gpurun_out/r5y_sq1 gpurun_out/r5y_sq2
exit 0
