#!/bin/bash
# round-5 session zc: the table stem with the convs on the exact-fp32 MFMA kernels (EDGEDET_CONV_MATH=f32: no
# bf16x6 / LDS-DMA kernel co-runs with it) against the default math, one plan with its two chains
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5zc_steps.log
D=$PWD/edgeml-object-detection_amd
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5zc_$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r5zc_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5zc_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
st f32_n1 300 env EDGEDET_CONV_MATH=f32 EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 10 --n 1
st f32_n2 300 env EDGEDET_CONV_MATH=f32 EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 10 --n 2
st x6_n1 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 10 --n 1
exit 0
