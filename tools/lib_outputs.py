"""Detections of fixed synthetic batches under the library EDGEDET_LIB names, for bit-identity checks
between two builds of libedgedet.so (a change meant to keep the arithmetic, e.g. a new epilogue).

    EDGEDET_LIB=.../libedgedet_a.so python tools/lib_outputs.py -o a.npz
    EDGEDET_LIB=.../libedgedet_b.so python tools/lib_outputs.py -o b.npz --compare a.npz

SSDLite at the bench batch (32, two chains) and FRCNN at batch 8, seeded weights and images
(edgeml_amd.synthetic); --compare prints, per model and field, whether every value is bit-identical
and the largest difference, and exits 1 on any difference."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from edgeml_amd import models, synthetic  # noqa: E402


def run():
    out = {}
    dev = "cuda:0"
    cases = [("ssd", lambda sd: models.SSDLite320(sd, 91, True), 32, 11),
             ("faster_rcnn", lambda sd: models.FasterRCNNFPNv2(sd, 91), 8, 23)]
    for kind, make, b, seed in cases:
        sd = synthetic.synthetic_state_dict(kind, 91, True, seed=0)
        model = make(sd).to(dev)
        imgs = synthetic.make_batch_u8(b, 640, 640, seed=seed).to(dev)
        got = model(imgs.float() / 255)
        torch.cuda.synchronize()
        for i, g in enumerate(got):
            for k in ("boxes", "scores", "labels"):
                out[f"{kind}/{i}/{k}"] = g[k].detach().cpu().numpy()
        del model
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--compare", default=None)
    a = ap.parse_args()
    out = run()
    np.savez(a.out, **out)
    if not a.compare:
        return 0
    ref = np.load(a.compare)
    bad = 0
    for kind in ("ssd", "faster_rcnn"):
        keys = [k for k in out if k.startswith(kind + "/")]
        same = all(k in ref and out[k].shape == ref[k].shape and np.array_equal(out[k], ref[k]) for k in keys)
        dmax = max((float(np.abs(out[k].astype(np.float64) - ref[k].astype(np.float64)).max())
                    for k in keys if k in ref and out[k].shape == ref[k].shape and out[k].size), default=0.0)
        print(f"{kind}: {len(keys)} arrays, bit-identical={same}, max |diff| {dmax:.3g}")
        bad += not same
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
