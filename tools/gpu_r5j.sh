#!/bin/bash
# round-5 session j: uint8 transform fast division (stem + FRCNN transform): exactness tests, A/B against
# the HEAD build alternated (SSD and FRCNN), stem solo time
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5j_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5j_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5j_$name.log | head -1)" >> gpurun_out/r5j_steps.log; [ $rc -ne 0 ] && exit $rc; return 0; }
st tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity_configs.py tests/test_gpu_pipeline.py
for v in base mbe2 mbxm mbdw2 mball base; do
  L=$PWD/edgeml-object-detection_amd/libedgedet_$v.so; [ $v = base ] && L=$PWD/edgeml-object-detection_amd/libedgedet.so
  st mb_$v 120 env EDGEDET_LIB=$L python -u tools/mb_bench.py --reps 50
  grep -h "us" gpurun_out/r5j_mb_$v.log | sed "s/^/$v /" >> gpurun_out/r5j_steps.log
done
HEADLIB=$PWD/edgeml-object-detection_amd/libedgedet_head.so
B="python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline"
F="python -u bench.py --model frcnn --steps 300 --warmup 10 --no-cpu --no-e2e --no-roofline"
for r in 1 2; do
  st new_$r 300 $B
  st head_$r 300 env EDGEDET_LIB=$HEADLIB $B
done
st fnew 300 $F
st fhead 300 env EDGEDET_LIB=$HEADLIB $F
st ops_new 300 python -u bench.py --model ssd --steps 100 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5j_ops_new.json
exit 0
