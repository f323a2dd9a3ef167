#!/bin/bash
# FRCNN kernel timeline (one plan in flight): per-dispatch start / end for the gap analysis.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl -- python3 bench.py --model frcnn --no-cpu --no-e2e --no-roofline --inflight 1 --steps 40 --warmup 4 > gpurun_out/r3ad.log 2>&1 || exit 5
f=$(find /tmp/tl -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY' > gpurun_out/r3ad_gaps.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 10 steps: find the final merge launches
names = [r["Kernel_Name"] for r in rows]
ends = [i for i, n in enumerate(names) if "merge_topk" in n]
sel = rows[ends[-20] + 1: ends[-2] + 1] if len(ends) >= 20 else rows[-1000:]
t0 = int(sel[0]["Start_Timestamp"])
prev_end = t0
busy = 0
gaps = []
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > prev_end:
        gaps.append((s - prev_end, r["Kernel_Name"][:70]))
    busy += e - s
    prev_end = max(prev_end, e)
span = prev_end - t0
print(f"span {span/1e6:.3f} ms over {len(sel)} dispatches, kernel busy {busy/1e6:.3f} ms")
gaps.sort(reverse=True)
for g, n in gaps[:30]:
    print(f"gap {g/1e3:8.1f} us before {n}")
PY
