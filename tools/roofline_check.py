"""Cross-check of bench.py's roofline launch times against a rocprofv3 kernel trace of the same bench.

    python tools/roofline_check.py <trace dir> <bench json line file> [-o out.json]

For each model's roofline launch (kernel name + workgroup count from the bench JSON) the trace's
dispatches of that kernel with that grid are collected; their mean and median durations are printed
beside the bench's HIP-event time.  With --inflight 1 and one chain the dispatches do not overlap, so
the two must agree; several layers can share a grid (the FRCNN box-head 3x3 convs), so the minimum
over dispatches is reported too.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("-o")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    d = json.loads([l for l in open(a.bench) if '"metric"' in l][0])
    out = {}
    for model, r in (("ssd", d.get("roofline")), ("frcnn", d.get("frcnn", {}).get("roofline"))):
        if not r:
            continue
        grid = r["grid_wg"] * r["wg_threads"]
        durs = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in rows
                if r["kernel"] in x["Kernel_Name"] and int(x["Grid_Size_X"]) * int(x["Grid_Size_Y"]) * int(x["Grid_Size_Z"]) == grid]
        if not durs:
            continue
        out[model] = {"kernel": r["kernel"], "launch": r["launch"], "grid_wg": r["grid_wg"], "bench_launch_ms": r["launch_ms"],
                      "trace_dispatches": len(durs), "trace_mean_ms": statistics.mean(durs),
                      "trace_median_ms": statistics.median(durs), "trace_min_ms": min(durs)}
    print(json.dumps(out, indent=1))
    if a.o:
        json.dump(out, open(a.o, "w"), indent=1)


if __name__ == "__main__":
    main()
