#!/bin/bash
# Stall picture of the bf16x6 conv kernels on single shapes (tools/conv_bench.py under one rocprofv3
# PMC pass): SQ wave-cycle split (active / wait / issue-stall), instruction mix, MFMA busy.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for t in ${TILES:-29 25}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
    --output-format csv -d gpurun_out/pmcc_$t -o c -- python3 tools/conv_bench.py --tiles $t --shapes ${SHAPES:-ssd_head_cls0,box_head_3x3} --reps 5 > gpurun_out/pmcc_$t.log 2>&1 || exit 5
  python3 tools/pmc_kernels.py gpurun_out/pmcc_$t --raw --top 3 >> gpurun_out/pmcc_summary.log 2>&1
done
exit 0
