#!/bin/bash
# One GPU session of record: parity tests + smoke, the bench as the driver runs it and a long run
# (per-op times), the FRCNN stage-error table, the kernel trace, the PMC traffic passes of the
# roofline launches (and the FRCNN box head) and the MFMA utilisation passes.  Steps stop the script
# on a fault, a crash or a time limit.  Switches: TESTS BENCH STAGE PROF (1 = run, default all 1).
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
if [ "${BENCH:-1}" = "1" ]; then
  step bench_driver 900 python -u bench.py --gpus 1 --steps 20 --warmup 5
  step bench_long 600 python -u bench.py --model both --steps 750 --warmup 20 --no-cpu --no-e2e --dump-ops gpurun_out/ops_long.json
fi
if [ "${STAGE:-1}" = "1" ]; then
  step stage_error 600 python -u tools/stage_error.py --images 0,1,2 -o gpurun_out/stage_error.json
fi
if [ "${PROF:-1}" = "1" ]; then
  step prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_trace -o trace -- python3 bench.py --model both --no-cpu --no-e2e --steps 200
  # the raw trace stays on the box (tens of MB): its per-kernel stats and the stretch attribution come back
  find /tmp/prof_trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
  python3 tools/stretch.py /tmp/prof_trace --kernel conv_x6b_group_kernel -o gpurun_out/stretch.txt >> gpurun_out/steps.log 2>&1
  for m in ssd frcnn; do
    step bench_fetch_$m 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$m -o fetch -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
    step bench_write_$m 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$m -o write -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
    python3 tools/pmc_summary.py --bench-log gpurun_out/bench_fetch_$m.log --model $m --fetch gpurun_out/prof_fetch_$m --write gpurun_out/prof_write_$m -o gpurun_out/pmc_$m.json >> gpurun_out/steps.log 2>&1
  done
  python3 tools/pmc_summary.py --bench-log x --model frcnn --fetch gpurun_out/prof_fetch_frcnn --write gpurun_out/prof_write_frcnn -o gpurun_out/pmc_frcnn_boxhead.json --kernel "conv_x6b_kernel<false, true, false, 128, 1, false, 256>" --grid-wg 3063 --algo-bytes 805000000 --launch "roi_heads.box_head.{0..3}.0 (3x3, tile 39)" >> gpurun_out/steps.log 2>&1
  step mfma 600 bash tools/gpu_mfma.sh
fi
exit 0
