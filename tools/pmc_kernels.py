"""Per-kernel SQ counter summary of one rocprofv3 PMC pass (instruction mix and stall picture).

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \\
        SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU --output-format csv -d DIR -o m -- python3 bench.py ...
    python tools/pmc_kernels.py DIR [--top 20]

Prints, per kernel name (all dispatches summed): dispatches, mean duration, waves, and per wave the
VALU / LDS / SALU instruction counts and wave cycles, the LDS-wait share of the wave cycles and
the LDS bank-conflict cycles per LDS instruction.
"""
import argparse
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--raw", action="store_true", help="every counter per wave (cycle counters as a share of SQ_WAVE_CYCLES)")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = {}
    for r in csv.DictReader(open(f)):
        d = disp.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"],
                                                "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = {}
    for d in disp.values():
        k = re.sub(r"\(.*", "", d["name"]).replace("void ", "").replace("edgedet::", "")
        g = agg.setdefault(k, {"n": 0})
        g["n"] += 1
        for c, v in d.items():
            if c != "name":
                g[c] = g.get(c, 0.0) + v
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])[: a.top]
    if a.raw:
        for k, g in rows:
            w = max(g.get("SQ_WAVES", 0.0), 1.0)
            cyc = max(g.get("SQ_WAVE_CYCLES", 0.0), 1.0)
            parts = [f"{c}={g[c] / cyc:.3f}" if c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) else f"{c}/w={g[c] / w:.1f}"
                     for c in sorted(g) if c.startswith(("SQ_", "GRBM_", "TCC_", "TCP_")) and c != "SQ_WAVES"]
            print(f"{k}: {g['n']} disp, {g['ns'] / g['n'] / 1e3:.1f} us, {w / g['n']:.0f} waves; " + ", ".join(parts))
        return
    print(f"{'us/disp':>8} {'x':>4} {'waves':>7} {'valu/w':>7} {'lds/w':>6} {'salu/w':>6} {'cyc/w':>8} "
          f"{'ldswait':>7} {'conf/lds':>8}  kernel")
    for k, g in rows:
        w = max(g.get("SQ_WAVES", 0.0), 1.0)
        lds = g.get("SQ_INSTS_LDS", 0.0)
        cyc = g.get("SQ_WAVE_CYCLES", 0.0)
        print(f"{g['ns'] / g['n'] / 1e3:8.1f} {g['n']:4d} {w / g['n']:7.0f} {g.get('SQ_INSTS_VALU', 0) / w:7.0f} "
              f"{lds / w:6.0f} {g.get('SQ_INSTS_SALU', 0) / w:6.0f} {cyc / w:8.0f} "
              f"{g.get('SQ_WAIT_INST_LDS', 0) / max(cyc, 1):7.3f} {g.get('SQ_LDS_BANK_CONFLICT', 0) / max(lds, 1):8.2f}  {k}")


if __name__ == "__main__":
    main()
