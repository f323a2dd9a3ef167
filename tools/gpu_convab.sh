#!/bin/bash
# Conv-kernel A/B across library builds: LIBS="old new ..." (libedgedet_<name>.so, "new" = product),
# ROUNDS (ABBA order), TILES, SHAPES for tools/conv_bench.py.  Stops on a fault or a time limit.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/convab.log
for r in $(seq 1 ${ROUNDS:-2}); do
  o="$LIBS"; [ $((r % 2)) = 0 ] && o=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $o; do
    lib="$PWD/edgeml-object-detection_amd/libedgedet_$v.so"; [ "$v" = "new" ] && lib="$PWD/edgeml-object-detection_amd/libedgedet.so"
    echo "== $v r$r" >> gpurun_out/convab.log
    EDGEDET_LIB="$lib" timeout -k 10 300 python -u tools/conv_bench.py --tiles ${TILES:-39} --shapes ${SHAPES:-box_head_3x3} --reps 20 >> gpurun_out/convab.log 2>&1
    rc=$?
    if grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" gpurun_out/convab.log; then exit 7; fi
    [ $rc -ne 0 ] && { echo "rc=$rc" >> gpurun_out/convab.log; exit $rc; }
  done
done
exit 0
