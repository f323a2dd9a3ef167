cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -m gpu -x -q --timeout 120 --timeout-method thread -k "se_ or ssd or SSD" 2>&1 | tail -2 || exit 1
timeout -k 10 200 python bench.py --model ssd --steps 30 --warmup 5 --dump-ops gpurun_out/ops_ssd_se.json 2>&1 | tail -1 | cut -c1-300 || exit 1
