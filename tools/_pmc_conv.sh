cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -q -x --timeout 200 --timeout-method thread -k miniature 2>&1 | tail -1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_conv1 -o c -- python3 tools/conv_bench.py --tiles 25 --shapes box_head_3x3 --reps 3 > gpurun_out/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES --output-format csv -d gpurun_out/pmc_conv2 -o c -- python3 tools/conv_bench.py --tiles 25 --shapes box_head_3x3 --reps 3 > gpurun_out/pmc2.log 2>&1
echo rc=$?
