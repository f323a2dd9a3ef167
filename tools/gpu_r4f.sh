#!/bin/bash
# Round-4 session f: the fused MBConv front (MBFRONT) -- its kernel tests and the SSD parity tests,
# then an ABBA A/B of EDGEDET_MB_FRONT (0 off, 1 expansion <= 240, 2 every eligible block), then the
# hardware-queue count (GPU_MAX_HW_QUEUES 4 vs 8) for both models.
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
SSD_AB="bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-roofline --no-alt"
FRCNN_AB="bench.py --model frcnn --steps 400 --warmup 10 --no-cpu --no-e2e --no-roofline --no-alt"
step pytest_front 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "mbfront or mbconv or dwconv" --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/pytest_front.log && ! grep -q "failed" gpurun_out/pytest_front.log || { echo "front kernel tests failed: stopping" >> gpurun_out/steps.log; exit 0; }
step pytest_ssd 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_configs.py tests/test_gpu_native_model.py -q -x -s --timeout 300 --timeout-method thread
for r in 1 2; do
  o="1 0 2"; [ $r = 2 ] && o="2 0 1"
  for v in $o; do EDGEDET_MB_FRONT=$v step ab_front${v}_r$r 300 python -u $SSD_AB; done
done
for r in 1 2; do
  o="4 8"; [ $r = 2 ] && o="8 4"
  for q in $o; do GPU_MAX_HW_QUEUES=$q step ab_q${q}_ssd_r$r 300 python -u $SSD_AB; done
done
for r in 1 2; do
  o="4 8"; [ $r = 2 ] && o="8 4"
  for q in $o; do GPU_MAX_HW_QUEUES=$q step ab_q${q}_frcnn_r$r 300 python -u $FRCNN_AB; done
done
exit 0
