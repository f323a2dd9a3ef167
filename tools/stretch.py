"""Why a launch runs longer in the pipeline than alone (measurement tool).

    python tools/stretch.py gpurun_out/prof_trace --kernel conv_x6b_group_kernel --grid-wg 822 [-o out.txt]

From a rocprofv3 --kernel-trace CSV of bench.py: every dispatch of the kernel whose name contains
--kernel (and, with --grid-wg, whose grid holds that many workgroups) is one span [start, end].  Per
dispatch: its span, the shortest span of the same launch in the trace (the least-contended dispatch,
close to the solo time), and the time of every OTHER dispatch that overlaps it, summed by kernel:
the co-running work that shares the CUs during the stretched span.  Printed: the mean span, the
stretch over the shortest, the fraction of the span during which at least one other kernel was
running, and the co-runners ranked by overlap (mean microseconds of overlap per dispatch).
"""
import argparse
import collections
import csv
import glob
import os


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("edgedet::", "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--grid-wg", type=int, default=0)
    ap.add_argument("--wg-size", type=int, default=512)
    ap.add_argument("-o", default="")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])

    def wg(r):
        try:
            return int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1) \
                // max(1, int(r["Workgroup_Size_X"]) * int(r.get("Workgroup_Size_Y", 1) or 1))
        except (KeyError, ValueError):
            return -1
    mine = [r for r in rows if a.kernel in r["Kernel_Name"] and (not a.grid_wg or wg(r) == a.grid_wg)]
    if not mine:
        raise SystemExit(f"no dispatch of {a.kernel} with {a.grid_wg} workgroups")
    spans = [r["e"] - r["s"] for r in mine]
    best = min(spans)
    over = collections.Counter()
    busy = 0
    j0 = 0
    piped = []  # spans of the dispatches that ran beside other kernels for most of their span
    for r in mine:
        ivs = []
        while j0 < len(rows) and rows[j0]["e"] < r["s"] - 10 ** 9:
            j0 += 1
        for o in rows[j0:]:
            if o["s"] >= r["e"]:
                break
            if o is r or o["e"] <= r["s"]:
                continue
            lo, hi = max(o["s"], r["s"]), min(o["e"], r["e"])
            over[short(o["Kernel_Name"])] += hi - lo
            ivs.append((lo, hi))
        ivs.sort()
        cov, cur = 0, None
        for lo, hi in ivs:  # union of the other dispatches' overlap intervals
            if cur is None or lo > cur[1]:
                if cur:
                    cov += cur[1] - cur[0]
                cur = [lo, hi]
            else:
                cur[1] = max(cur[1], hi)
        if cur:
            cov += cur[1] - cur[0]
        busy += cov
        if cov > 0.5 * (r["e"] - r["s"]):
            piped.append(r["e"] - r["s"])
    n = len(mine)
    mean = sum(spans) / n
    lines = [f"{a.kernel} ({a.grid_wg or 'any'} workgroups): {n} dispatches, mean span {mean / 1e3:.1f} us, "
             f"shortest {best / 1e3:.1f} us (stretch {mean / best:.2f}x over the least-contended dispatch)",
             f"  another kernel running beside it: {100 * busy / sum(spans):.1f} % of its span",
             f"  pipelined dispatches (another kernel beside it for > 50 % of the span): {len(piped)}, mean span "
             f"{(sum(piped) / max(1, len(piped))) / 1e3:.1f} us (bench.py's in-pipeline probe measures these)",
             "  co-runners (mean overlap per dispatch, us):"]
    for k, v in over.most_common(15):
        lines.append(f"    {v / n / 1e3:8.1f}  {k}")
    print("\n".join(lines))
    if a.o:
        with open(a.o, "w") as fh:
            fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
