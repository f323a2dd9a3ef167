#!/bin/bash
# round-5 session t: what the table stem build does to the input buffer (race_bisect detail of 'images'),
# with one chain (no concurrency inside the plan) and with the two chains
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5t_steps.log
D=$PWD/edgeml-object-detection_amd
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5t_$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r5t_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5t_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
st dbg_n1 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 6 --n 1 --detail backbone.features.0.1#
st dbg_n1_chains1 300 env EDGEDET_SSD_CHAINS=1 EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 6 --n 1 --detail backbone.features.0.1
st dbg_n1_eager 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 6 --n 1 --eager --detail backbone.features.0.1#
st prod_n1 300 python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 6 --n 1
exit 0
