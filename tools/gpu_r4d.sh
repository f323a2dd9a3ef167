#!/bin/bash
# Round-4 session d: tests + smoke after the tile-39 / stem changes, then the FRCNN timing check
# (per-pass completion traces with the SSD run before it and without), then the driver-args bench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/steps.log
step() {  # step <name> <timeout> <cmd...>: stop on anything but success / test failure, and on faults
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
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
rm -f gpurun_out/trace_*.jsonl
EDGEDET_BENCH_TRACE=gpurun_out/trace_frcnn.jsonl step tr_frcnn 300 python -u bench.py --model frcnn --steps 200 --warmup 10 --no-cpu --no-e2e --no-roofline --no-alt
EDGEDET_BENCH_TRACE=gpurun_out/trace_both.jsonl step tr_both 300 python -u bench.py --model both --steps 200 --warmup 10 --no-cpu --no-e2e --no-roofline --no-alt
step bench_driver 900 python -u bench.py --gpus 1 --steps 20 --warmup 5
if [ "${STAGE:-1}" = "1" ]; then
  step stage_error 600 python -u tools/stage_error.py --images 0,1,2 -o gpurun_out/stage_error.json
fi
exit 0
