#!/bin/bash
# round-5 session zg: register top-k bisection started at the block's smallest key (product) against
# key 1 (-DSEL_LO_ONE): NMS phase clocks and solo per-op times, alternated
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
D=$GRAFT_REPO_ROOT/edgeml-object-detection_amd
: > gpurun_out/r5zg_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5zg_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5zg_$name.log | head -1)" >> gpurun_out/r5zg_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5zg_$name.log; then exit 7; fi; [ $rc -ne 0 ] && exit $rc; return 0; }
st nmsprof_min 200 env EDGEDET_LIB=$D/libedgedet_nmsprof.so python -u tools/nms_profile.py
st nmsprof_lo1 200 env EDGEDET_LIB=$D/libedgedet_nmsproflo1.so python -u tools/nms_profile.py
for r in 1 2; do
  st ops_min_$r 300 python -u bench.py --model both --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5zg_ops_min_$r.json
  st ops_lo1_$r 300 env EDGEDET_LIB=$D/libedgedet_lo1.so python -u bench.py --model both --steps 50 --no-cpu --no-e2e --dump-ops gpurun_out/r5zg_ops_lo1_$r.json
done
exit 0
