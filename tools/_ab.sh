cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
S=box_head_3x3,fpn_p2_3x3,fc6,layer3_3x3
for v in x6b t14 prio t14prio; do echo "== $v"; EDGEDET_LIB=build/variants/lib_$v.so timeout -k 10 120 python tools/conv_bench.py --tiles 25 --shapes $S || exit $?; done
EDGEDET_LIB=build/variants/lib_t14.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bf16x6" 2>&1 | tail -2
EDGEDET_LIB=build/variants/lib_t14prio.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bf16x6" 2>&1 | tail -2
