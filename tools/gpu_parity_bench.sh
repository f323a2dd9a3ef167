#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/box.txt
lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/box.txt
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -q -s -rA > gpurun_out/pytest1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-budget 8 > gpurun_out/bench1.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench1.log
exit 0
