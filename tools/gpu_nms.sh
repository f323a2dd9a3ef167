#!/bin/bash
# Post-processing check: the exact post-process tests (incl. ties and clusters), then the SSD bench
# with the per-op dump and a kernel trace of the NMS kernels.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_postprocess.py tests/test_gpu_retinanet.py -x -q --timeout 200 --timeout-method thread > gpurun_out/nms_pytest.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --model ssd --no-cpu --no-e2e --dump-ops gpurun_out/nms_ops.json > gpurun_out/nms_bench.log 2>&1 || exit 7
rm -rf gpurun_out/nms_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nms_trace -o t -- python3 bench.py --model both --steps 100 --no-cpu --no-e2e --no-roofline > gpurun_out/nms_trace.log 2>&1 || exit 8
exit 0
