#!/bin/bash
# round-5 session f: register bitonic sort -- correctness (NMS / post-processing / parity GPU tests, ORIE
# vs float64) and an alternated A/B against the LDS sort (libedgedet_sortlds.so)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5f_steps.log
step() { local name=$1 t=$2; shift 2; local t0=$SECONDS; timeout -k 10 "$t" "$@" > gpurun_out/r5f_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $((SECONDS - t0)) s $(grep -o '"value": [0-9.]*' gpurun_out/r5f_$name.log | head -2 | tr '\n' ' ')" >> gpurun_out/r5f_steps.log; if grep -q "Memory access fault\|HSA_STATUS_ERROR" gpurun_out/r5f_$name.log; then exit 7; fi; [ $rc -gt 1 ] && exit $rc; return 0; }
step tests 600 python -u -m pytest tests/test_gpu_unitops.py tests/test_gpu_postprocess.py tests/test_gpu_parity_configs.py tests/test_gpu_models.py tests/test_gpu_orie_f64.py -q -s --timeout 300 --timeout-method thread
LDS=$GRAFT_REPO_ROOT/edgeml-object-detection_amd/libedgedet_sortlds.so
step ssd_regs1 300 python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5f_ops_regs.json
step ssd_lds1 300 env EDGEDET_LIB=$LDS python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5f_ops_lds.json
step ssd_lds2 300 env EDGEDET_LIB=$LDS python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
step ssd_regs2 300 python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
step frcnn_regs1 300 python -u bench.py --model frcnn --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
step frcnn_lds1 300 env EDGEDET_LIB=$LDS python -u bench.py --model frcnn --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
step frcnn_lds2 300 env EDGEDET_LIB=$LDS python -u bench.py --model frcnn --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
step frcnn_regs2 300 python -u bench.py --model frcnn --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
