cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
EDGEDET_LIB=build/variants/lib_nmsprof.so timeout -k 10 120 python tools/_nmsprof.py 2>&1 | grep -E "nms img0|counts" | tail -3
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread -k "ssd or nms or detect" 2>&1 | tail -1 || exit 1
timeout -k 10 200 python bench.py --model ssd --steps 20 --warmup 5 2>&1 | tail -1 | cut -c1-300
