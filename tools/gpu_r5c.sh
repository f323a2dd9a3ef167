#!/bin/bash
# round-5 session c: the bench with the in-pipeline roofline probe; SSD NMS form A/B (image-greedy vs
# per-class + merge); the short-run bias (a 4 s completion trace and settle lengths)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r5c_steps.log
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r5c_$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5c_$name.log | head -1)" >> gpurun_out/r5c_steps.log; [ $rc -ne 0 ] && exit $rc; return 0; }
run probe python -u bench.py --model both --steps 20 --warmup 5 --no-cpu --no-e2e --dump-ops gpurun_out/r5c_ops.json
run nms_image1 python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
run nms_class1 env EDGEDET_SSD_NMS=class python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/r5c_ops_class.json
run nms_class2 env EDGEDET_SSD_NMS=class python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
run nms_image2 python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
run trace env EDGEDET_BENCH_TRACE=gpurun_out/r5c_trace.jsonl python -u bench.py --model ssd --steps 3000 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
run s20_settle05 python -u bench.py --model ssd --steps 20 --warmup 5 --no-cpu --no-e2e --no-alt --no-roofline
run s20_settle2 env EDGEDET_BENCH_SETTLE=2 python -u bench.py --model ssd --steps 20 --warmup 5 --no-cpu --no-e2e --no-alt --no-roofline
run s750_settle2 env EDGEDET_BENCH_SETTLE=2 python -u bench.py --model ssd --steps 750 --warmup 20 --no-cpu --no-e2e --no-alt --no-roofline
run s20_settle05b python -u bench.py --model ssd --steps 20 --warmup 5 --no-cpu --no-e2e --no-alt --no-roofline
