#!/bin/bash
# Alternated A/B of library builds: LIBS="old new" (edgeml-object-detection_amd/libedgedet_<name>.so;
# "new" = the product libedgedet.so), MODEL=ssd|frcnn|both [ROUNDS=2] [STEPS=300]; round r runs the
# builds in order, round r+1 reversed (ABBA), each a fresh process with per-op times dumped.
# PRE="cmd": a step run first (e.g. the accuracy probe).  Stops on a fault or a time limit.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/libab.log
if [ -n "$PRE" ]; then
  timeout -k 10 600 bash -c "$PRE" > gpurun_out/pre.log 2>&1; rc=$?
  echo "pre rc=$rc" >> gpurun_out/libab.log
  [ $rc -ne 0 ] && exit $rc
fi
m=${MODEL:-frcnn}
for r in $(seq 1 ${ROUNDS:-2}); do
  o="$LIBS"; [ $((r % 2)) = 0 ] && o=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $o; do
    lib="$PWD/edgeml-object-detection_amd/libedgedet_$v.so"; [ "$v" = "new" ] && lib="$PWD/edgeml-object-detection_amd/libedgedet.so"
    EDGEDET_LIB="$lib" timeout -k 10 400 python -u bench.py --model $m --steps ${STEPS:-300} --warmup 20 --no-cpu --no-e2e --no-alt --dump-ops gpurun_out/ops_${v}_r$r.json > gpurun_out/libab_${v}_r$r.log 2>&1
    rc=$?
    echo "$v r$r rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/libab_${v}_r$r.log | tr '\n' ' ')" >> gpurun_out/libab.log
    if grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" gpurun_out/libab_${v}_r$r.log; then exit 7; fi
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
