#!/bin/bash
# One GPU session: build check, parity tests, smoke, bench, rocprofv3 kernel-trace stats and the
# PMC traffic passes.  Usage: gpu_session.sh [TESTS=1] [PROFILE=1] [PMC=1] (env switches)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/steps.log
step() {  # step <name> <timeout> <cmd...>: stop the script on anything but success/test-failure
    local name=$1 t=$2; shift 2
    local t0=$SECONDS
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc ${SECONDS}s-${t0}s = $((SECONDS - t0)) s" >> gpurun_out/steps.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
    if grep -q "illegal memory access\|Memory access fault" "gpurun_out/$name.log"; then
        echo "fault in $name: stopping" >> gpurun_out/steps.log; exit 7; fi
    return 0
}
if [ "${TESTS:-1}" = "1" ]; then
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -s -rA --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python -u bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = "1" ]; then
step prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python3 bench.py --model all --no-cpu --no-e2e
fi
if [ "${PMC:-1}" = "1" ]; then
for m in ssd frcnn; do
  step bench_fetch_$m 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$m -o fetch -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
  step bench_write_$m 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$m -o write -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
  python tools/pmc_summary.py --bench-log gpurun_out/bench_fetch_$m.log --model $m --fetch gpurun_out/prof_fetch_$m --write gpurun_out/prof_write_$m -o gpurun_out/pmc_$m.json >> gpurun_out/steps.log 2>&1
done
fi
exit 0
