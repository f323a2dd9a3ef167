"""Reduce rocprofv3 PMC passes to HBM bytes per launch of the bench's roofline kernel.

    python tools/pmc_summary.py --bench-log gpurun_out/bench_fetch_ssd.log --model ssd \
        --fetch gpurun_out/prof_fetch_ssd --write gpurun_out/prof_write_ssd -o profiles/pmc_ssd.json

    (--kernel / --grid-wg / --algo-bytes / --launch: the same reduction for another launch, e.g. the
    FRCNN box-head 3x3 convs: conv_x6b_kernel<false, true, false, 128, 1, false, 256>, 3,063 workgroups)

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one pass of TCC
counters).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE on gfx950 reports exactly half of the bytes of
a wide coalesced read, so it is doubled; WRITE_SIZE is taken as is; both are KiB.  The dispatches
averaged are those of the roofline kernel (name match) with the roofline launch's grid size.
"""
import argparse
import csv
import glob
import json
import os


def bench_line(path):
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                return json.loads(line)
    raise SystemExit(f"no bench JSON line in {path}")


def counter_rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    rows = []
    for fn in files:
        with open(fn) as f:
            rows.extend(csv.DictReader(f))
    return rows


def per_dispatch(rows, counter, kernel, grid_items):
    vals = {}
    for r in rows:
        name = r.get("Counter_Name", "")
        if name != counter or kernel not in r.get("Kernel_Name", ""):
            continue
        if grid_items is not None and int(float(r.get("Grid_Size", 0))) != grid_items:
            continue
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[did] = vals.get(did, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench-log", required=True)
    ap.add_argument("--model", default="ssd")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("-o", required=True)
    ap.add_argument("--kernel", default="", help="another launch than the roofline one: kernel name substring")
    ap.add_argument("--grid-wg", type=int, default=0, help="... its grid in workgroups")
    ap.add_argument("--wg-threads", type=int, default=512)
    ap.add_argument("--algo-bytes", type=float, default=0.0, help="... its algorithmic bytes")
    ap.add_argument("--launch", default="", help="... its name (for the record)")
    a = ap.parse_args()
    if a.kernel:
        roof = {"kernel": a.kernel, "grid_wg": a.grid_wg, "wg_threads": a.wg_threads,
                "algorithmic_bytes": a.algo_bytes, "launch": a.launch or a.kernel}
    else:
        line = bench_line(a.bench_log)
        roof = line["roofline"] if a.model == "ssd" else line.get("frcnn", {}).get("roofline")
        if roof is None and a.model == "frcnn":
            roof = line["roofline"]
    kernel = roof["kernel"]
    grid = roof.get("grid_wg")
    items = grid * roof["wg_threads"] if grid else None
    f = per_dispatch(counter_rows(a.fetch), "FETCH_SIZE", kernel, items)
    w = per_dispatch(counter_rows(a.write), "WRITE_SIZE", kernel, items)
    if not f or not w:
        raise SystemExit(f"no dispatches of {kernel} (grid {items}) in the PMC output")
    fetch_kib = sum(f) / len(f)
    write_kib = sum(w) / len(w)
    hbm = (2.0 * fetch_kib + write_kib) * 1024.0
    out = {"model": a.model, "kernel": kernel, "launch": roof["launch"], "grid_wg": grid,
           "dispatches": {"fetch": len(f), "write": len(w)}, "FETCH_SIZE_KiB": fetch_kib,
           "WRITE_SIZE_KiB": write_kib, "hbm_bytes_per_launch": hbm,
           "algorithmic_bytes": roof.get("algorithmic_bytes"),
           "traffic_over_algorithmic": hbm / roof["algorithmic_bytes"] if roof.get("algorithmic_bytes") else None,
           "correction": "FETCH_SIZE x2 (gfx950 half-count on wide reads), KiB -> bytes"}
    os.makedirs(os.path.dirname(a.o), exist_ok=True)
    with open(a.o, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
