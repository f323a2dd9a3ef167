cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mbconv" 2>&1 | tail -1 || exit 1
for v in new mbd1; do echo "== $v"; L=build/variants/lib_$v.so; [ $v = new ] && L=edgeml-object-detection_amd/libedgedet.so
  EDGEDET_LIB=$L timeout -k 10 120 python tools/mb_bench.py || exit $?; done
