cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
bash tools/gpu_mb_ab.sh; echo "mb rc=$?" >> gpurun_out/combo.txt
timeout -k 10 600 python -u tools/ingest_bench.py --n 2000 > gpurun_out/ingest.log 2>&1; echo "ingest rc=$?" >> gpurun_out/combo.txt
