#!/bin/bash
# A/B: in-loop activation split (default) vs a pre-split pass for every eligible tile-25 conv
# (EDGEDET_CONV_PRESPLIT=2), FRCNN device rate, twice interleaved; FRCNN model tests under the latter.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
EDGEDET_CONV_PRESPLIT=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_native_model.py -x -q --timeout 300 --timeout-method thread -k "frcnn" > gpurun_out/ps_pytest.log 2>&1 || exit 5
: > gpurun_out/ps_ab.log
for rep in 1 2; do
for ps in 1 2; do
  EDGEDET_CONV_PRESPLIT=$ps timeout -k 10 300 python bench.py --model frcnn --no-cpu --no-e2e --dump-ops gpurun_out/ps_ops_$ps.json 2>/dev/null | grep '"metric"' > gpurun_out/ps_b_$ps.json || exit 6
  python3 -c "import json; d=json.load(open('gpurun_out/ps_b_$ps.json')); print('presplit=$ps', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" >> gpurun_out/ps_ab.log
done
done
exit 0
