cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1 || exit 1
timeout -k 10 300 python -u tools/_detect_prof.py > gpurun_out/detect_prof.log 2>&1; echo rc=$?
