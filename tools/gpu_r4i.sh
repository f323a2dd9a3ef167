#!/bin/bash
# Round-4 session i: the one-launch SE excitation for the wide layers (se_wide_kernel): its tests and
# the SSD parity suite, then alternated SSD runs against the fc1 + fc2 pair (EDGEDET_SE_WIDE=0).
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
step pytest_se 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "se_excitation" --timeout 120 --timeout-method thread
grep -q "failed" gpurun_out/pytest_se.log && { echo "se tests failed: stopping" >> gpurun_out/steps.log; exit 0; }
step pytest_ssd 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_configs.py -q -x --timeout 300 --timeout-method thread
SSD_AB="bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt"
for r in 1 2; do
  o="1 0"; [ $r = 2 ] && o="0 1"
  for v in $o; do EDGEDET_SE_WIDE=$v step ab_sew${v}_r$r 300 python -u $SSD_AB --dump-ops gpurun_out/ops_sew${v}_r$r.json; done
done
exit 0
