#!/bin/bash
# HBM bytes of the streaming 1x1 tiles on the SSDLite block 0.3 expand (24 -> 72 at 80^2, 16 images):
# separate FETCH_SIZE / WRITE_SIZE passes over tools/conv_bench.py, mean per dispatch per kernel.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcp_$c -o c -- python3 tools/conv_bench.py --tiles ${TILES:-33,34,35,28} --shapes ${SHAPES:-ssd_03_expand,ssd_03_project} --reps 5 > gpurun_out/pmcp_$c.log 2>&1 || exit 5
done
python3 - <<'P' > gpurun_out/pmcp_summary.txt
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/pmcp_{c}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != c: continue
        key = (r["Kernel_Name"][:60], int(r["Grid_Size"]) if "Grid_Size" in r else 0)
        acc[key].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(c, k, len(v), "mean KiB", round(sum(v) / len(v), 1))
P
exit 0
