#!/bin/bash
# round-5 session x: x6b A loads two stages ahead (X6B_APF2 build) against the product: conv tests on the variant,
# FRCNN and SSD A/B alternated, ops dump of the variant
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5x_steps.log
D=$PWD/edgeml-object-detection_amd
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5x_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5x_$name.log | head -1)" >> gpurun_out/r5x_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5x_$name.log; then exit 7; fi; [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 600 env EDGEDET_LIB=$D/libedgedet_apf2.so python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "conv" tests/test_gpu_parity_configs.py tests/test_gpu_plan_records.py
F="python -u bench.py --model frcnn --steps 300 --warmup 10 --no-cpu --no-e2e --no-roofline"
for r in 1 2; do
  run f_apf2_$r 300 env EDGEDET_LIB=$D/libedgedet_apf2.so $F
  run f_base_$r 300 $F
done
run ops_apf2 300 env EDGEDET_LIB=$D/libedgedet_apf2.so python -u bench.py --model frcnn --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5x_ops_apf2.json
S="python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline"
run s_apf2 300 env EDGEDET_LIB=$D/libedgedet_apf2.so $S
run s_base 300 $S
exit 0
