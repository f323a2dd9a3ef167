#!/bin/bash
# Conv kernel picture after the 16x16-read LDS swizzle: isolated launch times of the dominant shapes,
# then one PMC pass each for LDS bank conflicts and for HBM bytes (FETCH_SIZE / WRITE_SIZE).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
SH=box_head_3x3,fpn_p2_3x3,ssd_head_cls0,ssd_12_3,layer3_3x3,layer4_3x3
timeout -k 10 300 python3 tools/conv_bench.py --tiles 0 --shapes $SH --reps 20 > gpurun_out/r3d_conv.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d gpurun_out/r3d_lds -o c -- python3 tools/conv_bench.py --tiles 0 --shapes box_head_3x3,ssd_head_cls0 --reps 3 > gpurun_out/r3d_lds.log 2>&1 || exit 5
python3 tools/pmc_kernels.py gpurun_out/r3d_lds --raw --top 4 > gpurun_out/r3d_lds_summary.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3d_fetch -o c -- python3 tools/conv_bench.py --tiles 0 --shapes box_head_3x3,fpn_p2_3x3,ssd_head_cls0 --reps 3 > gpurun_out/r3d_fetch.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3d_write -o c -- python3 tools/conv_bench.py --tiles 0 --shapes box_head_3x3,fpn_p2_3x3,ssd_head_cls0 --reps 3 > gpurun_out/r3d_write.log 2>&1 || exit 7
python3 tools/pmc_kernels.py gpurun_out/r3d_fetch --raw --top 4 > gpurun_out/r3d_fetch_summary.txt 2>&1
python3 tools/pmc_kernels.py gpurun_out/r3d_write --raw --top 4 > gpurun_out/r3d_write_summary.txt 2>&1
exit 0
