#!/bin/bash
# SQ stall picture of the SSD kernels (grouped heads + fused MBConv on), then the SSD step with op
# families left out (diagnostic, wrong results) on the fused-MBConv configuration.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
EDGEDET_SSD_HEADS=1 EDGEDET_MB_BLOCK=1 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU \
  --output-format csv -d gpurun_out/r3f_sq -o c -- python3 bench.py --model ssd --steps 30 --warmup 5 --no-cpu --no-e2e --no-alt --no-roofline > gpurun_out/r3f_sq.log 2>&1 || exit 5
python3 tools/pmc_kernels.py gpurun_out/r3f_sq --raw --top 14 > gpurun_out/r3f_sq_summary.txt 2>&1
EDGEDET_SSD_HEADS=0 EDGEDET_MB_BLOCK=1 SKIPS="none 3 4 6 17 22 129 133,134,135 2 8" STEPS=400 bash tools/gpu_skip.sh || exit 6
exit 0
