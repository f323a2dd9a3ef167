#!/bin/bash
# round-5 session zb: is the table stem's first replay the odd one?  reference taken after 0 / 3 extra solo runs
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5zb_steps.log
D=$PWD/edgeml-object-detection_amd
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5zb_$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r5zb_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5zb_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
st ref0 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 10 --n 1
st ref3 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 10 --n 1 --ref-after 3
st ref3_eager 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 10 --n 1 --ref-after 3 --eager
exit 0
