#!/bin/bash
# round-5 session u: does a replay change the plan's input buffer (table-stem debug build vs product)?
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5u_steps.log
D=$PWD/edgeml-object-detection_amd
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5u_$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r5u_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5u_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
st dbg_graph 200 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/input_probe.py
st dbg_eager 200 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/input_probe.py --eager
st prod_graph 200 python -u tools/input_probe.py
exit 0
