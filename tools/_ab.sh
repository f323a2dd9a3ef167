cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_retinanet.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
for m in frcnn retinanet ssd; do timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 --no-cpu --no-roofline 2>&1 | tail -1 | cut -c1-200 || exit 1; done
