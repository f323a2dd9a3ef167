#!/bin/bash
# Accuracy session: the conv accuracy probe, the FRCNN stage- and layer-error tables, then (TESTS=1) the GPU
# parity tests and (BENCH=1) the bench at the driver's arguments.  Stops on a fault or time limit.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/steps.log
step() {
    local name=$1 t=$2; shift 2
    local t0=$SECONDS
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $((SECONDS - t0)) s" >> gpurun_out/steps.log
    if grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "gpurun_out/$name.log"; then
        echo "fault in $name: stopping" >> gpurun_out/steps.log; exit 7; fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
    return 0
}
step accuracy 300 python -u tools/accuracy_probe.py
step stage_error 600 python -u tools/stage_error.py --images 0,1,2 -o gpurun_out/stage_error.json
step layer_error 600 python -u tools/layer_error.py --image 0
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench_driver 900 python -u bench.py --gpus 1 --steps 20 --warmup 5
fi
exit 0
