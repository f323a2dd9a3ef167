#!/bin/bash
# round-5 session e: the fixed GPU tests (end-to-end witness, config-4, redzones); the kernel trace of the
# bench and the stretch attribution of the roofline launches
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5e_steps.log
step() { local name=$1 t=$2; shift 2; local t0=$SECONDS; timeout -k 10 "$t" "$@" > gpurun_out/r5e_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $((SECONDS - t0)) s" >> gpurun_out/r5e_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5e_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
step tests 900 python -u -m pytest tests/test_gpu_redzone.py tests/test_gpu_frcnn_e2e.py tests/test_gpu_config4.py -v -s --timeout 600 --timeout-method thread
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5e_prof -o trace -- python3 bench.py --model both --no-cpu --no-e2e --steps 200
python3 tools/stretch.py gpurun_out/r5e_prof --kernel conv_x6b_group_kernel --grid-wg 822 -o gpurun_out/r5e_stretch_ssd.txt >> gpurun_out/r5e_steps.log 2>&1
python3 tools/stretch.py gpurun_out/r5e_prof --kernel conv_x6b_group_kernel --grid-wg 3333 -o gpurun_out/r5e_stretch_frcnn.txt >> gpurun_out/r5e_steps.log 2>&1
exit 0
