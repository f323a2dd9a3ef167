cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model frcnn --steps 20 --warmup 5 --no-cpu --dump-ops gpurun_out/ops_frcnn.json || exit 1
python - <<'P'
import json; d=json.load(open("gpurun_out/ops_frcnn.json"))
for m,ops in d.items():
    ops=sorted(ops, key=lambda o:-o.get("us",o.get("ms",0)) if isinstance(o,dict) else 0)[:12] if isinstance(ops,list) else ops
    print(m, json.dumps(ops)[:1500])
P
