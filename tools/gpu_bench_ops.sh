#!/bin/bash
# Quick perf iteration: build, parity smoke of the models, bench with per-op dump (no CPU baseline).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 8
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_postprocess.py -q -s -rA ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
grep -q "illegal memory access\|Memory access fault" gpurun_out/pytest_quick.log && exit 7
timeout -k 10 600 python bench.py --model ${MODEL:-both} --steps 20 --warmup 5 --no-cpu --dump-ops gpurun_out/ops.json > gpurun_out/bench_quick.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_quick.log

if [ "${TRACE:-1}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_quick -o q -- python3 bench.py --model ${MODEL:-both} --steps 5 --warmup 2 --no-cpu --no-roofline > gpurun_out/trace_quick.log 2>&1
echo "trace rc=$?" >> gpurun_out/trace_quick.log
fi
exit 0
