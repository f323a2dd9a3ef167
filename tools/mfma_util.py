"""MFMA utilisation of the conv kernels from one rocprofv3 PMC pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d <dir> -o m -- \
        python3 bench.py --model frcnn --steps 2 --warmup 1 --no-cpu --no-roofline --inflight 1
    python tools/mfma_util.py <dir> [--model frcnn]

Per dispatch (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units" and "DVFS give-back"):
  * SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over the chip's 1024 SIMDs
    (32 per 32x32x16 bf16 MFMA);
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs, so GRBM_GUI_ACTIVE / 8 is the dispatch's clock
    cycles at the clock the chip actually held;
  * utilisation = busy / (1024 * GRBM_GUI_ACTIVE / 8): the share of the matrix pipe's cycles in
    use while the dispatch ran, independent of the clock (the spec-peak fraction is this times
    held clock / 2.4 GHz).
Prints per-kernel rows and the cycle-weighted total over the GEMM conv kernels. GRBM_GUI_ACTIVE
over-counts on dispatches shorter than about 0.3 ms (the held clock then reads above 2.4 GHz), so
their utilisation reads low: trust the rows whose held clock is at or below 2.4 GHz.
  * mfma_util_spec = busy / (1024 * dispatch duration * 2.4 GHz): the share of the matrix pipe's
    cycles at the 2.4 GHz spec clock over the dispatch's wall time (the trace's start/end stamps).
    It needs no clock counter, so it is valid for short dispatches too, and it is a lower bound of
    the utilisation at the clock actually held (equal to it when the chip holds 2.4 GHz).
"""
import argparse
import csv
import glob
import json
import os
import re

SIMDS = 1024
XCDS = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--model", default="")
    ap.add_argument("-o", default="")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = {}
    for r in csv.DictReader(open(f)):
        d = disp.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                                "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = {}
    for d in disp.values():
        if ("conv" not in d["name"] and "pw_" not in d["name"]) or "dwconv" in d["name"]:
            continue  # the GEMM-shaped conv kernels only (depthwise runs on the VALU)
        k = re.sub(r"\(edgedet::ConvParams\)|void edgedet::", "", d["name"])
        g = rows.setdefault(k, {"dispatches": 0, "busy": 0.0, "cycles": 0.0, "ns": 0})
        g["dispatches"] += 1
        g["busy"] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        g["cycles"] += d.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        g["ns"] += d["ns"]
    tot_b = sum(g["busy"] for g in rows.values())
    tot_c = sum(g["cycles"] for g in rows.values())
    tot_ns = sum(g["ns"] for g in rows.values())
    spec = lambda b, ns: b / (SIMDS * ns * 1e-9 * 2.4e9) if ns else 0.0  # noqa: E731
    out = {"model": a.model, "source": os.path.relpath(f), "kernels": {}, "conv_total": None}
    for k, g in sorted(rows.items(), key=lambda kv: -kv[1]["cycles"]):
        u = g["busy"] / (SIMDS * g["cycles"]) if g["cycles"] else 0.0
        clk = g["cycles"] / (g["ns"] * 1e-9) / 1e9 if g["ns"] else 0.0
        us = spec(g["busy"], g["ns"])
        out["kernels"][k] = {"dispatches": g["dispatches"], "mfma_util": round(u, 4), "mfma_util_spec": round(us, 4),
                             "held_clock_GHz": round(clk, 3), "us_per_dispatch": round(g["ns"] / g["dispatches"] / 1e3, 2),
                             "share_of_conv_time": round(g["ns"] / tot_ns, 4)}
        print(f"{u:7.3f} (spec-clock {us:6.3f})  clk {clk:5.2f} GHz  {g['ns'] / tot_ns:6.1%} of conv time  "
              f"x{g['dispatches']:4d}  {g['ns'] / g['dispatches'] / 1e3:8.1f} us  {k}")
    out["conv_total"] = {"mfma_util": round(tot_b / (SIMDS * tot_c), 4), "mfma_util_spec": round(spec(tot_b, tot_ns), 4)}
    print(f"conv kernels: cycle-weighted MFMA utilisation {tot_b / (SIMDS * tot_c):.3f}; at the 2.4 GHz spec "
          f"clock over the dispatch wall time {spec(tot_b, tot_ns):.3f}")
    if a.o:
        with open(a.o, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
