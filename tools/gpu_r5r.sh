#!/bin/bash
# round-5 session r: the round-4 table stem rebuilt with NaN-poisoned LDS and end-of-kernel
# LDS checks (libedgedet_stemdbg.so), the product stem with the table's LDS footprint only (libedgedet_stempad.so),
# and the product, each through tools/race_bisect.py (one SSD b=32 plan beside a second instance, every buffer
# against its solo run) and the single-kernel stem tests
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5r_steps.log
D=$PWD/edgeml-object-detection_amd
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5r_$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r5r_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5r_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
st dbg_kernel 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "stem or transform"
st dbg_bisect 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 12 --stem-debug
st pad_bisect 300 env EDGEDET_LIB=$D/libedgedet_stempad.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 12
st prod_bisect 300 python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 12
st dbg_bisect_eager 300 env EDGEDET_LIB=$D/libedgedet_stemdbg.so python -u tools/race_bisect.py --kind ssd --B 32 --H 640 --W 640 --trials 8 --eager --stem-debug
exit 0
