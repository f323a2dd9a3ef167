"""End-to-end rate of run_batches (pinned uint8 batches -> rows) at several in-flight counts.
    python tools/e2e_sweep.py [--model ssd|frcnn] [--inflight 2,3,4] [--batches 40]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="ssd")
    ap.add_argument("--inflight", default="2,3,4")
    ap.add_argument("--batches", type=int, default=40)
    a = ap.parse_args()
    from edgeml_amd import fmt, models, synthetic
    m = (models.ssdlite320_mobilenet_v3_large() if a.model == "ssd" else models.fasterrcnn_resnet50_fpn_v2()).to("cuda")
    B = 32 if a.model == "ssd" else 8
    imgs = synthetic.make_batch_u8(B, 640, 640, seed=3).pin_memory()
    work = [(k, imgs) for k in range(a.batches)]
    for n in [int(v) for v in a.inflight.split(",")]:
        for _ in m.run_batches(work[:n + 1], inflight=n, raw=True):
            pass
        torch.cuda.synchronize()
        for fmt_rows in (False, True):
            cnt, t0 = 0, time.perf_counter()
            for _, c, box, score, label in m.run_batches(work, inflight=n, raw=True):
                cnt += len(fmt.format_batch(box, score, label, c, 640, 640)) if fmt_rows else len(c)
            el = time.perf_counter() - t0
            print(f"{a.model} inflight={n} rows={fmt_rows}: {cnt / el:.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
