#!/bin/bash
# One GPU session (traces kept in /tmp on the box, only summaries under gpurun_out/): build check, parity tests, smoke, bench, rocprofv3 kernel-trace stats and the
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
step prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_trace -o trace -- python3 bench.py --model all --no-cpu --no-e2e
find /tmp/prof_trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
# the roofline launches against a one-in-flight kernel trace (same kernel, same grid)
step prof_if1 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_if1 -o trace -- python3 bench.py --model both --no-cpu --no-e2e --inflight 1 --steps 200
python3 tools/roofline_check.py /tmp/prof_if1 gpurun_out/prof_if1.log -o gpurun_out/roofline_check.json >> gpurun_out/steps.log 2>&1
find /tmp/prof_if1 -name "*kernel_stats.csv" -exec cp {} gpurun_out/if1_kernel_stats.csv \;
fi
if [ "${PMC:-1}" = "1" ]; then
for m in ssd frcnn; do
  step bench_fetch_$m 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/prof_fetch_$m -o fetch -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
  step bench_write_$m 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/prof_write_$m -o write -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
  python tools/pmc_summary.py --bench-log gpurun_out/bench_fetch_$m.log --model $m --fetch /tmp/prof_fetch_$m --write /tmp/prof_write_$m -o gpurun_out/pmc_$m.json >> gpurun_out/steps.log 2>&1
done
fi
exit 0
