#!/bin/bash
# round-5 session k: SE excitation kernels with staged operands: exactness / parity tests, SSD bench
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5k_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5k_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5k_$name.log | head -1)" >> gpurun_out/r5k_steps.log; [ $rc -ne 0 ] && exit $rc; return 0; }
st tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity_configs.py tests/test_gpu_models.py tests/test_gpu_pipeline.py
B="python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline"
HEADLIB=$PWD/edgeml-object-detection_amd/libedgedet_head.so
st new_1 300 $B
st head_1 300 env EDGEDET_LIB=$HEADLIB $B
st new_2 300 $B
st ops_new 300 python -u bench.py --model ssd --steps 100 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5k_ops_new.json
exit 0
