"""Diagnostic: run_batches with batches in flight against model(images), image by image.

    python tools/race_check.py [--B 16] [--n 24] [--reps 3] [--path stage|pinned] [--kind ssd]

Counts (batch, image) pairs whose detections differ from the one-batch-at-a-time __call__ result of
the same images (the host's float images / 255; the uint8 path equals it bit for bit).  A race
between a batch's input upload and the plan graph's first kernels shows up as differing images at
the end of a batch (the bytes the copy writes last)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="ssd")
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--H", type=int, default=640)
    ap.add_argument("--W", type=int, default=640)
    ap.add_argument("--path", default="stage", choices=["stage", "pinned"])
    ap.add_argument("--inflight", type=int, default=0)
    a = ap.parse_args()
    from edgeml_amd import models, synthetic
    if a.kind == "ssd":
        m = models.SSDLite320(synthetic.synthetic_state_dict("ssd", 91, True, seed=0), 91, True).to("cuda:0")
    else:
        m = models.fasterrcnn_resnet50_fpn_v2().to("cuda:0")
    u8s = [synthetic.make_batch_u8(a.B, a.H, a.W, seed=100 + i) for i in range(a.n)]
    ref = []
    for u in u8s:
        r = m(list(u.float() / 255))
        ref.append([(x["boxes"].cpu().numpy(), x["scores"].cpu().numpy()) for x in r])
    for rep in range(a.reps):
        if a.path == "pinned":
            batches = [(i, u.pin_memory()) for i, u in enumerate(u8s)]
        else:
            batches = [(i, list(u)) for i, u in enumerate(u8s)]
        bad = []
        for tag, dets in m.run_batches(batches, inflight=a.inflight or None):
            for j, (b, s, _) in enumerate(dets):
                rb, rs = ref[tag][j]
                if b.shape != rb.shape or not (np.array_equal(b, rb) and np.array_equal(s, rs)):
                    # stale: the result of an earlier batch's image j (an output copied too early)
                    stale = [t for t in range(max(0, tag - 4), tag)
                             if ref[t][j][0].shape == b.shape and np.array_equal(ref[t][j][0], b)]
                    top = float(np.abs(b[:1] - rb[:1]).max()) if len(b) and len(rb) else -1.0
                    bad.append((tag, j, "stale%s" % stale if stale else "top%.3g" % top))
        print(f"rep {rep} path {a.path} B {a.B}: "
              f"{len(bad)} differing images of {a.n * a.B}: {bad[:12]}", flush=True)


if __name__ == "__main__":
    main()
