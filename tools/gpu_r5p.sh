#!/bin/bash
# round-5 session p: RPN selection from registers + rank sort (2 keys per thread): tests, FRCNN A/B against
# the previous build (libedgedet_prev.so), ops dump
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5p_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5p_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5p_$name.log | head -1)" >> gpurun_out/r5p_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5p_$name.log; then exit 7; fi; [ $rc -ne 0 ] && exit $rc; return 0; }
st tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan_records.py tests/test_gpu_parity_configs.py tests/test_gpu_postprocess.py tests/test_gpu_models.py
F="python -u bench.py --model frcnn --steps 300 --warmup 10 --no-cpu --no-e2e --no-roofline"
for r in 1 2; do
  st new_$r 300 $F
  st prev_$r 300 env EDGEDET_LIB=$PWD/edgeml-object-detection_amd/libedgedet_prev.so $F
done
st ops_new 300 python -u bench.py --model frcnn --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5p_ops_new.json
exit 0
