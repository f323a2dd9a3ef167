#!/bin/bash
# Round-4 session b: tests + smoke, the bench as the driver runs it, a long SSD run with per-op times,
# and the SSD A/B of the grouped heads and the chain count (alternated).
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
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_driver 900 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_long 600 python -u bench.py --model both --steps 750 --warmup 20 --no-cpu --no-e2e --dump-ops gpurun_out/ops_long.json
for r in 1 2; do
  for v in 1 0; do
    EDGEDET_HEAD_GROUP=$v step ab_heads${v}_r$r 300 python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-roofline --no-alt
  done
done
for inf in 4 6 8; do
  EDGEDET_SSD_CHAINS=1 step chains1_if$inf 300 python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-roofline --no-alt --inflight $inf
done
exit 0
