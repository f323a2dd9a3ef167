#!/bin/bash
# Round-4 session c: tests + smoke, the bench as the driver runs it, the stem (matrix cores vs vector
# ALUs) and head-tile A/B (alternated 750-step SSD runs), the long bench with per-op times, the FRCNN
# stage-error table, the kernel trace + PMC traffic passes of the roofline kernels, the MFMA
# utilisation passes, and last the lane-destruction repro variants (one per process).
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
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench_driver 900 python -u bench.py --gpus 1 --steps 20 --warmup 5
fi
if [ "${AB:-1}" = "1" ]; then
  # ABBA order (alternated pairs showed the first run of each pair ~1% high whatever its variant)
  for r in 1 2; do
    o="1 0"; [ $r = 2 ] && o="0 1"
    for v in $o; do EDGEDET_STEM_MFMA=$v step ab_stem${v}_r$r 300 python -u $SSD_AB; done
  done
  for r in 1 2; do
    o="29 31"; [ $r = 2 ] && o="31 29"
    for t in $o; do EDGEDET_HEAD_TILE=$t step ab_tile${t}_r$r 300 python -u $SSD_AB; done
  done
fi
if [ "${FAB:-0}" = "1" ]; then  # FRCNN: the Cout = 256 layers (and the RPN head groups) on the 128 x 256 tile
  step pytest_t39 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k bf16x6 --timeout 120 --timeout-method thread
  step conv39 300 python -u tools/conv_bench.py --tiles 25,39 --shapes box_head_3x3,fpn_p2_3x3,layer3_3x3 --reps 20
  FRCNN_AB="bench.py --model frcnn --steps 200 --warmup 10 --no-cpu --no-e2e --no-roofline --no-alt"
  for r in 1 2; do
    step ab_t39_0_r$r 300 python -u $FRCNN_AB
    EDGEDET_TILE39=1 EDGEDET_RPN_TILE=39 step ab_t39_1_r$r 300 python -u $FRCNN_AB
  done
fi
if [ "${MERGE:-0}" = "1" ]; then  # SSD: chains merged after block features.0.<m> (0: never)
  step pytest_merge 300 python -u -m pytest tests/test_gpu_models.py -q -x -k chains_agree -s --timeout 200 --timeout-method thread
  for r in 1 2; do
    o="${MERGES:-0 3 5 7 9 12}"; [ $r = 2 ] && o=$(echo $o | tr ' ' '\n' | tac | tr '\n' ' ')
    for m in $o; do EDGEDET_SSD_MERGE=$m step ab_merge${m}_r$r 300 python -u $SSD_AB; done
  done
fi
if [ "${LONG:-1}" = "1" ]; then
  step bench_long 600 python -u bench.py --model both --steps 750 --warmup 20 --no-cpu --no-e2e --dump-ops gpurun_out/ops_long.json
fi
if [ "${STAGE:-1}" = "1" ]; then
  step stage_error 600 python -u tools/stage_error.py --images 0,1,2 -o gpurun_out/stage_error.json
fi
if [ "${PROF:-1}" = "1" ]; then
  step prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python3 bench.py --model both --no-cpu --no-e2e --steps 200
  for m in ssd frcnn; do
    step bench_fetch_$m 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$m -o fetch -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
    step bench_write_$m 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$m -o write -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
    python3 tools/pmc_summary.py --bench-log gpurun_out/bench_fetch_$m.log --model $m --fetch gpurun_out/prof_fetch_$m --write gpurun_out/prof_write_$m -o gpurun_out/pmc_$m.json >> gpurun_out/steps.log 2>&1
  done
  step mfma 600 bash tools/gpu_mfma.sh
fi
if [ "${LANE_REPRO:-1}" = "1" ]; then  # one variant per process; stop at the first that dies
  for m in streams_during events_during; do step lane_repro_$m 60 tools/lane_repro $m; done
fi
exit 0
