#!/bin/bash
# round-5 session n: RPN level NMS split into selection / IoU mask over many workgroups / scan:
# FRCNN + RetinaNet parity, plan-record tests, A/B against EDGEDET_RPN_SPLIT=0 (one workgroup per segment),
# the old kernel's phase profile, ops dump
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5n_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5n_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5n_$name.log | head -1)" >> gpurun_out/r5n_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5n_$name.log; then exit 7; fi; [ $rc -ne 0 ] && exit $rc; return 0; }
st tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan_records.py tests/test_gpu_parity_configs.py tests/test_gpu_models.py tests/test_gpu_redzone.py
st rpnprof 200 env EDGEDET_RPN_SPLIT=0 EDGEDET_LIB=$PWD/edgeml-object-detection_amd/libedgedet_rpnprof.so python -u tools/rpn_profile.py
F="python -u bench.py --model frcnn --steps 300 --warmup 10 --no-cpu --no-e2e --no-roofline"
for r in 1 2; do
  st split_$r 300 $F
  st one_$r 300 env EDGEDET_RPN_SPLIT=0 $F
done
st ops_split 300 python -u bench.py --model frcnn --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5n_ops_split.json
exit 0
