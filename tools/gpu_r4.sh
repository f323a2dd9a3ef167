#!/bin/bash
# Round-4 GPU session: parity tests + smoke, the bench as the driver runs it (--steps 20 --warmup 5)
# and a long run of the same bench (steady-state check), then optional experiments.
#   TESTS=1 (default) pytest -m gpu + smoke;  BENCH=1 driver-args bench + 750-step SSD run;
#   CHAINS="1 2" SSD in-flight sweep per chain count;  EXTRA="cmd" one more step.
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
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x -rA --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench_driver 900 python -u bench.py --gpus 1 --steps 20 --warmup 5
  step bench_long 600 python -u bench.py --model both --steps 750 --warmup 20 --no-cpu --no-e2e --no-roofline
fi
for c in ${CHAINS:-}; do
  for inf in ${INFLIGHTS:-2 4 6}; do
    EDGEDET_SSD_CHAINS=$c step chains${c}_if${inf} 300 python -u bench.py --model ssd --steps 400 --warmup 20 --no-cpu --no-e2e --no-roofline --no-alt --inflight $inf
  done
done
if [ "${LANE_REPRO:-0}" = "1" ]; then  # one variant per process; stop at the first that dies
  [ -x tools/lane_repro ] || hipcc -O2 --offload-arch=gfx950 tools/lane_repro.cpp -o tools/lane_repro || exit 8
  for m in none events streams both; do step lane_repro_$m 60 tools/lane_repro $m; done
fi
if [ -n "${EXTRA:-}" ]; then step extra 900 bash -c "$EXTRA"; fi
exit 0
