#!/bin/bash
# Diagnostic (wrong results): SSD steady-state step with op families left out (EDGEDET_DIAG_SKIP),
# to see what each family costs the step under stream concurrency.  Needs the diagnostic build
# (python -m edgeml_amd.build --diag -> libedgedet_diag.so, made on the CPU side beforehand).
cd "$GRAFT_REPO_ROOT" || exit 9
export EDGEDET_LIB="$PWD/edgeml-object-detection_amd/libedgedet_diag.so"
[ -f "$EDGEDET_LIB" ] || { echo "no diagnostic build"; exit 9; }
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/skip.log
for sk in ${SKIPS:-none 3 4 6 17 8 21 2 4,6 3,4,6,17,8,21,2}; do
  [ $sk = none ] && unset EDGEDET_DIAG_SKIP || export EDGEDET_DIAG_SKIP=$sk
  v=$(timeout -k 10 300 python bench.py --diagnostic --model ${MODEL:-ssd} --steps ${STEPS:-300} --warmup 20 --no-cpu --no-e2e 2>/dev/null | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d=d.get('frcnn', d) if '${MODEL:-ssd}'=='frcnn' else d; print(d['value'], d['ms_per_step'])") || exit 6
  echo "skip=$sk $v" >> gpurun_out/skip.log
done
exit 0
