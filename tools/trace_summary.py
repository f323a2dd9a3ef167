"""Per-kernel in-graph durations of one replayed step from a rocprofv3 kernel-trace CSV.

    python tools/trace_summary.py gpurun_out/prof_quick [--first preprocess_kernel --last 'ssd_image_nms|merge_topk' --min-len 90]

In a captured graph consecutive kernels of the critical path run back to back, so a kernel's
trace duration includes its launch latency and ramp: this is the breakdown that adds up to the
step time (bench.py's isolated per-op times do not include those).
"""
import argparse
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--first", default="preprocess_kernel")
    ap.add_argument("--last", default="ssd_image_nms|merge_topk")
    ap.add_argument("--min-len", type=int, default=60)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    seqs, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if a.first in n:
            cur = [r]
        elif cur is not None:
            cur.append(r)
            if re.search(a.last, n) and len(cur) >= a.min_len:
                seqs.append(cur)
                cur = None
    if not seqs:
        raise SystemExit("no step found")
    s = seqs[len(seqs) // 2]
    t0, t1 = int(s[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in s)
    print(f"steps found {len(seqs)}; step span {(t1 - t0) / 1e3:.1f} us over {len(s)} kernels")
    agg = {}
    for r in s:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("edgedet::", "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        x = agg.setdefault(n, [0, 0.0])
        x[0] += 1
        x[1] += d
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{d:9.1f} us  x{c:3d}  {n}")


if __name__ == "__main__":
    main()
