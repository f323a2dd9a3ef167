#!/bin/bash
# round-5 session l: depthwise rows preloaded (DW_PIPE=1 every K, =2 K = 3 only) against the product, alternated
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5l_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5l_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5l_$name.log | head -1)" >> gpurun_out/r5l_steps.log; [ $rc -ne 0 ] && exit $rc; return 0; }
D=$PWD/edgeml-object-detection_amd
st tests 600 env EDGEDET_LIB=$D/libedgedet_dwpipe.so python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "dwconv or group"
B="python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline"
for r in 1 2; do
  st base_$r 300 $B
  st pipe_$r 300 env EDGEDET_LIB=$D/libedgedet_dwpipe.so $B
  st pipe3_$r 300 env EDGEDET_LIB=$D/libedgedet_dwpipe3.so $B
done
st ops_pipe 300 env EDGEDET_LIB=$D/libedgedet_dwpipe.so python -u bench.py --model ssd --steps 100 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5l_ops_pipe.json
st ops_base 300 python -u bench.py --model ssd --steps 100 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5l_ops_base.json
exit 0
