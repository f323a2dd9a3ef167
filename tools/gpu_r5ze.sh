#!/bin/bash
# round-5 session ze: register top-k probes with the popcounts summed in four independent chains
# (product) against the serial chain (-DSEL_SERIAL_COUNT): tests, NMS phase ticks, solo per-op
# times and throughput A/B for both models
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
D=$GRAFT_REPO_ROOT/edgeml-object-detection_amd
: > gpurun_out/r5ze_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5ze_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5ze_$name.log | head -1)" >> gpurun_out/r5ze_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5ze_$name.log; then exit 7; fi; [ $rc -ne 0 ] && exit $rc; return 0; }
st tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_postprocess.py tests/test_gpu_plan_records.py tests/test_gpu_unitops.py tests/test_gpu_parity_configs.py
st nmsprof_chains 200 env EDGEDET_LIB=$D/libedgedet_nmsprof.so python -u tools/nms_profile.py
st nmsprof_serial 200 env EDGEDET_LIB=$D/libedgedet_nmsprofserial.so python -u tools/nms_profile.py
S="python -u bench.py --model ssd --steps 300 --warmup 10 --no-cpu --no-e2e --no-roofline"
F="python -u bench.py --model frcnn --steps 200 --warmup 10 --no-cpu --no-e2e --no-roofline"
for r in 1 2; do
  st ssd_chains_$r 300 $S
  st ssd_serial_$r 300 env EDGEDET_LIB=$D/libedgedet_selserial.so $S
  st frcnn_chains_$r 300 $F
  st frcnn_serial_$r 300 env EDGEDET_LIB=$D/libedgedet_selserial.so $F
done
st ops_chains 300 python -u bench.py --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5ze_ops_chains.json
st ops_serial 300 env EDGEDET_LIB=$D/libedgedet_selserial.so python -u bench.py --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5ze_ops_serial.json
exit 0
