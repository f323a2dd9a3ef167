#!/bin/bash
# round-5 session zd: four-wave class selection in the SSD postprocess: tests, A/B against the one-wave
# form, solo per-op timings and a short kernel trace of each
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5zd_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5zd_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5zd_$name.log | head -1)" >> gpurun_out/r5zd_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5zd_$name.log; then exit 7; fi; [ $rc -ne 0 ] && exit $rc; return 0; }
st tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_postprocess.py tests/test_gpu_parity_configs.py tests/test_gpu_pipeline.py
F="python -u bench.py --model ssd --steps 300 --warmup 10 --no-cpu --no-e2e --no-roofline"
for r in 1 2 3; do
  st block_$r 300 $F
  st wave_$r 300 env EDGEDET_SSD_SELECT_WAVE=1 $F
done
st ops_block 300 python -u bench.py --model ssd --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5zd_ops_block.json
st ops_wave 300 env EDGEDET_SSD_SELECT_WAVE=1 python -u bench.py --model ssd --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5zd_ops_wave.json
st trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5zd_prof -o trace -- python3 bench.py --model ssd --no-cpu --no-e2e --no-roofline --steps 30
cp $(find /tmp/r5zd_prof -name "*kernel_stats.csv" | head -1) gpurun_out/r5zd_kernel_stats.csv
exit 0
