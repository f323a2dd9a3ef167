#!/bin/bash
# A/B: quick parity, then bench with default tiles and with EDGEDET_BIG_TILE=$BIG for the large convs.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 8
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -q -s -rA > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
grep -q "illegal memory access\|Memory access fault" gpurun_out/pytest_quick.log && exit 7
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu --dump-ops gpurun_out/ops.json > gpurun_out/bench_quick.log 2>&1 || exit 6
EDGEDET_BIG_TILE=${BIG:-4} timeout -k 10 600 python bench.py --model frcnn --steps 20 --warmup 5 --no-cpu --dump-ops gpurun_out/ops_big.json > gpurun_out/bench_big.log 2>&1
echo "done rc=$?" >> gpurun_out/bench_big.log
exit 0
