"""MFMA utilisation of the conv kernels from one rocprofv3 PMC pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d <dir> -o m -- \
        python3 bench.py --model frcnn --steps 2 --warmup 1 --no-cpu --no-roofline --inflight 1
    python tools/mfma_util.py <dir> [--model frcnn]

Per dispatch (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units"):
  * SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over the chip's 1024 SIMDs
    (32 per 32x32x16 bf16 MFMA);
  * mfma_util_spec = busy / (1024 * dispatch duration * 2.4 GHz): the share of the matrix pipe's
    cycles at the 2.4 GHz spec clock over the dispatch's wall time (the trace's start/end stamps).
    This is the only figure quoted: it needs no clock counter and is a lower bound of the
    utilisation at whatever clock the chip held.
  * held_clock_GHz = (GRBM_GUI_ACTIVE / 8 XCDs) / duration is printed for information only, and only
    for kernels whose mean dispatch is >= 0.3 ms: on shorter dispatches GRBM_GUI_ACTIVE over-counts
    (round 3 read 2.9-4.5 GHz there, above the 2.4 GHz maximum), so no figure is derived from it.
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
    tot_ns = sum(g["ns"] for g in rows.values())
    spec = lambda b, ns: b / (SIMDS * ns * 1e-9 * 2.4e9) if ns else 0.0  # noqa: E731
    out = {"model": a.model, "source": os.path.relpath(f), "basis": "busy / (1024 SIMDs x dispatch ns x 2.4 GHz)",
           "kernels": {}, "conv_total": None}
    for k, g in sorted(rows.items(), key=lambda kv: -kv[1]["ns"]):
        us = spec(g["busy"], g["ns"])
        per = g["ns"] / g["dispatches"] / 1e3
        clk = g["cycles"] / (g["ns"] * 1e-9) / 1e9 if g["ns"] and per >= 300.0 else None
        out["kernels"][k] = {"dispatches": g["dispatches"], "mfma_util_spec": round(us, 4),
                             "held_clock_GHz_info": None if clk is None else round(clk, 3),
                             "us_per_dispatch": round(per, 2), "share_of_conv_time": round(g["ns"] / tot_ns, 4)}
        cs = f"{clk:5.2f} GHz" if clk is not None else "   -    "
        print(f"{us:7.3f}  clk {cs}  {g['ns'] / tot_ns:6.1%} of conv time  x{g['dispatches']:4d}  {per:8.1f} us  {k}")
    out["conv_total"] = {"mfma_util_spec": round(spec(tot_b, tot_ns), 4)}
    print(f"conv kernels: MFMA utilisation at the 2.4 GHz spec clock over the dispatch wall time "
          f"{spec(tot_b, tot_ns):.3f}")
    if a.o:
        with open(a.o, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
