cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_retinanet.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bf16x6 or retina" 2>&1 | tail -2 || exit 1
S=box_head_3x3,layer3_3x3,layer4_3x3,ssd_f13,ssd_12_3,ssd_head_cls0
for v in base new; do echo "== $v"; L=build/variants/lib_$v.so; [ $v = new ] && L=edgeml-object-detection_amd/libedgedet.so
  EDGEDET_LIB=$L timeout -k 10 120 python tools/conv_bench.py --tiles 21,23 --shapes $S || exit $?; done
for m in frcnn retinanet ssd; do timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 2>&1 | tail -1 || exit 1; done
