#!/bin/bash
# round-5 session v: are the device reference copies of race_bisect changed during the table-stem debug runs?
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5v_steps.log
D=$PWD/edgeml-object-detection_amd
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5v_$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r5v_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5v_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
st dbg_n1 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 6 --n 1
st dbg_n2 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 6 --n 2
st prod_n2 300 python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 6 --n 2
exit 0
