#!/bin/bash
# Kernel-trace A/B of the post-process kernels over library variants ($VARS).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for v in base $VARS; do
  if [ $v = base ]; then unset EDGEDET_LIB; else export EDGEDET_LIB=build/variants/lib_$v.so; fi
  rm -rf gpurun_out/sel_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sel_$v -o t -- python3 bench.py --model ssd --steps 300 --no-cpu --no-e2e --no-roofline > gpurun_out/sel_$v.log 2>&1 || exit 8
done
exit 0
