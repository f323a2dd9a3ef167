cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in rpnprof rpnu2 rpnu4 rpnu8; do echo $v; EDGEDET_LIB=build/variants/lib_$v.so timeout -k 10 300 python bench.py --model frcnn --steps 1 --warmup 0 --no-cpu --no-roofline 2>&1 | grep "rpn level" | sort | uniq | head -3 || exit 1; done
