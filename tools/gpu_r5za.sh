#!/bin/bash
# round-5 session za: the table stem with every byte load waited for before it indexes the table
# (STEM_TABLE_DEBUG=2) against the plain table stem (=1), race_bisect one plan with two chains
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5za_steps.log
D=$PWD/edgeml-object-detection_amd
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5za_$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r5za_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5za_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
st wait_n2 300 env EDGEDET_LIB=$D/libedgedet_stemdbg2.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 12 --n 2 --stem-debug
st plain_n2 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 12 --n 2 --stem-debug
st wait_n1 300 env EDGEDET_LIB=$D/libedgedet_stemdbg2.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 8 --n 1
exit 0
