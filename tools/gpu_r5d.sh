#!/bin/bash
# round-5 session d: the new GPU tests (end-to-end witness, config-4 world 2, record equivalences,
# redzones), the config-4 subset witness, the bench with the in-pipeline probe, the MFMA rounding probe,
# the SSD image-NMS phase profile
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5d_steps.log
step() { local name=$1 t=$2; shift 2; local t0=$SECONDS; timeout -k 10 "$t" "$@" > gpurun_out/r5d_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $((SECONDS - t0)) s" >> gpurun_out/r5d_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5d_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
step mfma 120 python -u tools/mfma_probe.py
step redzone 300 python -u -m pytest tests/test_gpu_redzone.py tests/test_gpu_plan_records.py -v -s --timeout 200 --timeout-method thread
step nmsprof 120 env EDGEDET_LIB=$GRAFT_REPO_ROOT/edgeml-object-detection_amd/libedgedet_nmsprof.so python -u tools/nms_profile.py
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-e2e
step tests 800 python -u -m pytest tests/test_gpu_frcnn_e2e.py tests/test_gpu_config4.py -v -s --timeout 600 --timeout-method thread
step c4witness 300 python -u tools/config4_witness.py -o gpurun_out/r5d_c4witness.json
