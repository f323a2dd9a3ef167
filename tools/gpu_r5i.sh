#!/bin/bash
# round-5 session i: SSD image NMS with the rank sort + ballot class ranks: exactness tests, phase
# profile, A/B against the HEAD build (libedgedet_head.so) alternated, then the SQ stall picture
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5i_steps.log
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/r5i_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5i_$name.log | head -1)" >> gpurun_out/r5i_steps.log; [ $rc -ne 0 ] && exit $rc; return 0; }
st tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_postprocess.py "tests/test_gpu_parity_configs.py::test_ssd_b32_bench_plan_matches_oracle"
st nmsprof 200 env EDGEDET_LIB=$PWD/edgeml-object-detection_amd/libedgedet_nmsprof.so python -u tools/nms_profile.py
B="python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline"
for r in 1 2; do
  st new_$r 300 $B
  st head_$r 300 env EDGEDET_LIB=$PWD/edgeml-object-detection_amd/libedgedet_head.so $B
done
st ops_new 300 python -u bench.py --model ssd --steps 100 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5i_ops_new.json
bash tools/gpu_r5h.sh
exit $?
