#!/bin/bash
# round-5 session zh: the profiling legs of the session of record (kernel trace + stretch, PMC traffic,
# MFMA utilisation; tools/gpu_r5q.sh steps with r5zh names) on the final tree
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5zh_steps.log
step() {
    local name=$1 t=$2; shift 2
    local t0=$SECONDS
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $((SECONDS - t0)) s $(grep -o '"value": [0-9.]*' gpurun_out/$name.log | head -1)" >> gpurun_out/r5zh_steps.log
    if grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "gpurun_out/$name.log"; then
        echo "fault in $name: stopping" >> gpurun_out/r5zh_steps.log; exit 7; fi
    if [ $rc -ne 0 ]; then echo "stopping after $name rc=$rc" >> gpurun_out/r5zh_steps.log; exit $rc; fi
    return 0
}
step ops_long 400 python -u bench.py --model both --steps 300 --warmup 20 --no-cpu --no-e2e --dump-ops gpurun_out/r5zh_ops_long.json
step prof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_trace -o trace -- python3 bench.py --model both --no-cpu --no-e2e --steps 200
cp "$(find /tmp/prof_trace -name '*kernel_stats.csv' | head -1)" gpurun_out/r5zh_kernel_stats.csv
python3 tools/stretch.py /tmp/prof_trace --kernel conv_x6b_group_kernel --grid-wg 822 -o gpurun_out/r5zh_stretch_ssd.txt >> gpurun_out/r5zh_steps.log 2>&1
python3 tools/stretch.py /tmp/prof_trace --kernel conv_x6b_group_kernel --grid-wg 3333 -o gpurun_out/r5zh_stretch_frcnn.txt >> gpurun_out/r5zh_steps.log 2>&1
rm -rf /tmp/prof_trace
for m in ssd frcnn; do
  step bench_fetch_$m 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/prof_fetch_$m -o fetch -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
  step bench_write_$m 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/prof_write_$m -o write -- python3 bench.py --model $m --steps 2 --warmup 1 --no-cpu --no-e2e
  python3 tools/pmc_summary.py --bench-log gpurun_out/bench_fetch_$m.log --model $m --fetch /tmp/prof_fetch_$m --write /tmp/prof_write_$m -o gpurun_out/pmc_$m.json >> gpurun_out/r5zh_steps.log 2>&1
done
python3 tools/pmc_summary.py --bench-log x --model frcnn --fetch /tmp/prof_fetch_frcnn --write /tmp/prof_write_frcnn -o gpurun_out/pmc_frcnn_boxhead.json --kernel "conv_x6b_kernel<false, true, false, 128, 1, false, 256>" --grid-wg 3063 --algo-bytes 805000000 --launch "roi_heads.box_head.{0..3}.0 (3x3, tile 39)" >> gpurun_out/r5zh_steps.log 2>&1
rm -rf /tmp/prof_fetch_* /tmp/prof_write_*
step mfma 300 bash tools/gpu_mfma.sh
exit 0
