"""Which hardware queue each kernel of a rocprofv3 kernel trace was dispatched from (measurement tool).

    python tools/queue_map.py gpurun_out/prof_trace [--match ssd_stem_kernel,conv_x6b_group_kernel]

Per queue: the number of dispatches and the kernels most often dispatched from it; then, for each
kernel name in --match, the sequence of queues its dispatches came from.  Streams that share a
hardware queue have their work serialised in submission order, so two batch chains (or two plan
instances) meant to overlap must come from different queues.
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--match", default="ssd_stem_kernel,ssd_postprocess,rpn_level_nms_kernel")
    ap.add_argument("--first", type=int, default=48)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else None
    skey = "Stream_Id" if "Stream_Id" in rows[0] else None
    print("columns:", ", ".join(rows[0].keys()))
    per_q = collections.defaultdict(collections.Counter)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("edgedet::", "")[:48]
        per_q[(r.get(qkey), r.get(skey))][name] += 1
    for q, c in sorted(per_q.items(), key=lambda kv: str(kv[0])):
        print(f"queue {q[0]} stream {q[1]}: {sum(c.values())} dispatches; top: "
              + ", ".join(f"{n} x{k}" for n, k in c.most_common(4)))
    for m in a.match.split(","):
        seq = [(r.get(qkey), r.get(skey)) for r in rows if m in r["Kernel_Name"]]
        if seq:
            print(f"{m}: {len(seq)} dispatches; first {a.first} (queue, stream):",
                  " ".join(f"{q}/{s}" for q, s in seq[:a.first]))


if __name__ == "__main__":
    main()
