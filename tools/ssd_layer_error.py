"""Feature-map error of the engine's SSDLite against the float64 oracle (measurement tool; needs a GPU).

    python tools/ssd_layer_error.py [--leg 0-1] [--batch 1]

The engine runs bench.py's ORIE-leg images (synthetic.make_batch(1, 640, 640, seed=7000 + i)) in one
batch and its plan buffers are read back: the six feature maps the head reads (backbone.features.0.13,
backbone.features.1.3, backbone.extra.{0..3}.2) and the head outputs.  The CPU oracle computes the
same tensors in float32 and float64 (oracle/ssdlite.py forward_raw).  Printed per tensor: max and RMS
of |value - float64| relative to the tensor's max |float64|, for the engine and for the float32
oracle, and the RMS ratio -- the SSD counterpart of tools/layer_error.py.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FEATS = ["backbone.features.0.13", "backbone.features.1.3"] + [f"backbone.extra.{e}.2" for e in range(4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", default="0-1")
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args()
    from edgeml_amd import models, synthetic
    from edgeml_amd.distributed import usable_cpus
    from oracle.ssdlite import SSDLiteOracle
    from tools.ssd_raw_error import parse
    torch.set_num_threads(usable_cpus())
    sd = synthetic.synthetic_state_dict("ssd", 91, True)
    eng = models.SSDLite320(sd, 91, True).to("cuda")
    orc = {dt: SSDLiteOracle(sd, 91, True, dtype=dt) for dt in (torch.float32, torch.float64)}
    ids = parse(a.leg)
    for s in range(0, len(ids), a.batch):
        c = ids[s:s + a.batch]
        batch = [synthetic.make_batch(1, 640, 640, seed=7000 + i)[0] for i in c]
        eng(batch)
        plan = eng.plan(len(c), 640, 640)
        torch.cuda.synchronize()
        with torch.no_grad():
            ref = {dt: o.forward_raw(batch) for dt, o in orc.items()}
        t64, t32 = ref[torch.float64], ref[torch.float32]
        pairs = [(n, plan.buffers[n].tensor().detach().cpu().double(), t32[2][j].double(), t64[2][j].double())
                 for j, n in enumerate(FEATS)]
        pairs += [("cls_logits", plan.cls_logits.tensor().cpu().double(), t32[0].double(), t64[0].double()),
                  ("bbox_regression", plan.bbox_regression.tensor().cpu().double(), t32[1].double(), t64[1].double())]
        print(f"images {c} (batch {len(c)})")
        print(f"{'tensor':28s} {'engine max':>10s} {'rms':>9s} | {'f32 max':>9s} {'rms':>9s} | rms ratio", flush=True)
        for name, e, f, t in pairs:
            if t.ndim == 4:                       # oracle NCHW -> the engine's NHWC (channels may be padded)
                t, f = t.permute(0, 2, 3, 1), f.permute(0, 2, 3, 1)
                e = e.reshape(e.shape[0], t.shape[1], t.shape[2], -1)[..., :t.shape[3]]
            e = e.reshape(t.shape).numpy()
            t, f = t.numpy(), f.numpy()
            sc = max(np.abs(t).max(), 1e-30)
            de, df = e - t, f - t
            re, rf = np.sqrt((de ** 2).mean()) / sc, np.sqrt((df ** 2).mean()) / sc
            print(f"{name:28s} {np.abs(de).max() / sc:10.2e} {re:9.2e} | {np.abs(df).max() / sc:9.2e} {rf:9.2e} | "
                  f"{re / max(rf, 1e-30):6.2f}", flush=True)


if __name__ == "__main__":
    main()
