cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u tools/estimator_bench.py > gpurun_out/estimator_bench.log 2>&1; echo "est rc=$?"; cat gpurun_out/estimator_bench.log | grep -v amdgpu.ids
