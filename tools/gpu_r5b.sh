#!/bin/bash
# round-5 session b: end-to-end FRCNN witness attribution (f32 and f64 references) and a probe of the
# EVENT record inside a captured graph
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u tools/e2e_witness.py --ref f32 --side engine -o gpurun_out/r5b_e2e_f32.json > gpurun_out/r5b_e2e_f32.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/e2e_witness.py --ref f64 --side engine -o gpurun_out/r5b_e2e_f64.json > gpurun_out/r5b_e2e_f64.log 2>&1 || exit $?
