"""Device concurrency over the steady state of a rocprofv3 kernel trace.

    python tools/concurrency.py gpurun_out/prof_dir [--skip 0.1] [--last N]

Over the middle of the trace (dropping the first/last `skip` fraction of its time span): the fraction
of time at least one kernel runs, the time-weighted number of kernels in flight, the histogram of
that number, and the kernels that spend the most time alone on the device (the serial tail).
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--skip", type=float, default=0.1)
    ap.add_argument("--last", type=int, default=0, help="only the last N kernels (the timed steps)")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")
             .replace("edgedet::", "")) for r in csv.DictReader(open(f))]
    rows.sort()
    if a.last:
        rows = rows[-a.last:]
    t_lo, t_hi = rows[0][0], max(r[1] for r in rows)
    span = t_hi - t_lo
    w0, w1 = t_lo + a.skip * span, t_hi - a.skip * span
    ev = []
    for s, e, n in rows:
        s, e = max(s, w0), min(e, w1)
        if e > s:
            ev.append((s, 1, n))
            ev.append((e, -1, n))
    ev.sort(key=lambda x: (x[0], x[1]))
    hist, alone = {}, {}
    live = {}
    last = w0
    for t, d, n in ev:
        k = sum(live.values())
        dt = t - last
        hist[k] = hist.get(k, 0) + dt
        if k == 1:
            (only,) = [x for x, c in live.items() if c]
            alone[only] = alone.get(only, 0) + dt
        live[n] = live.get(n, 0) + d
        if live[n] == 0:
            del live[n]
        last = t
    tot = w1 - w0
    busy = tot - hist.get(0, 0)
    avg = sum(k * v for k, v in hist.items()) / tot
    print(f"window {tot / 1e3:.1f} us: busy {busy / tot:.3f}, mean kernels in flight {avg:.2f}")
    for k in sorted(hist):
        print(f"  {k:2d} in flight: {hist[k] / tot:.3f}")
    print("time alone on the device (us over the window):")
    for n, v in sorted(alone.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {v / 1e3:9.1f}  {n}")


if __name__ == "__main__":
    main()
