#!/bin/bash
# merge_topk without scratch: merge / FRCNN parity tests, then the FRCNN bench at one and two in flight.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/r3ae.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_postprocess.py tests/test_gpu_models.py tests/test_gpu_parity_configs.py tests/test_gpu_retinanet.py > gpurun_out/r3ae_t.log 2>&1 || { echo "tests failed" >> gpurun_out/r3ae.txt; tail -30 gpurun_out/r3ae_t.log >> gpurun_out/r3ae.txt; exit 1; }
echo "tests $(tail -1 gpurun_out/r3ae_t.log)" >> gpurun_out/r3ae.txt
for inf in 1 2 2; do
  x=$(timeout -k 10 200 python bench.py --model frcnn --steps 300 --warmup 20 --no-cpu --no-e2e --no-roofline --inflight $inf 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d = d.get('frcnn', d); print(d['value'], d['ms_per_step'])") || exit 6
  echo "inflight=$inf $x" >> gpurun_out/r3ae.txt
done
