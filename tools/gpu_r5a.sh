#!/bin/bash
# round-5 session a: record-level GPU tests, the LDS canary, the conv accuracy probe and the end-to-end
# FRCNN witness attribution (f32 and f64 references)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_plan_records.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5a_plan_records.log 2>&1; rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 180 python -u tools/lds_canary.py > gpurun_out/r5a_canary.log 2>&1 || exit $?
timeout -k 10 180 python -u tools/accuracy_probe.py > gpurun_out/r5a_accuracy.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/e2e_witness.py --ref f32 --side engine -o gpurun_out/r5a_e2e_f32.json > gpurun_out/r5a_e2e_f32.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/e2e_witness.py --ref f64 --side engine -o gpurun_out/r5a_e2e_f64.json > gpurun_out/r5a_e2e_f64.log 2>&1 || exit $?
