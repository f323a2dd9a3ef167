"""SSDLite raw head outputs (class logits, box regression) of the engine and of the float32 CPU oracle
against the float64 oracle (measurement tool; needs a GPU).

    python tools/ssd_raw_error.py [--config4 0-7] [--leg 0-3]

--config4: images of tools/config4_full.py's set (mixed COCO sizes, JPEG q = 90), run in the batch the
detect CLI puts them in; --leg: bench.py's ORIE-leg images (640 x 640, batch 1).  Printed per image:
max |value - float64| and RMS, for the engine and for the float32 oracle.  The parity tests gate the
engine against the float32 oracle (tests/parity_models.py RAW_TOL); this tells which of the two sits
closer to the exact arithmetic when they part.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(s):
    out = []
    for part in filter(None, s.split(",")):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config4", default="0-7")
    ap.add_argument("--leg", default="0-3")
    a = ap.parse_args()
    from edgeml_amd import distributed, models, synthetic
    from edgeml_amd.distributed import usable_cpus
    from oracle.ssdlite import SSDLiteOracle
    from tools.config4_witness import config4_image
    torch.set_num_threads(usable_cpus())
    sd = synthetic.synthetic_state_dict("ssd", 91, True)
    eng = models.SSDLite320(sd, 91, True).to("cuda")
    orc = {dt: SSDLiteOracle(sd, 91, True, dtype=dt) for dt in (torch.float32, torch.float64)}
    jobs = []
    if a.config4:
        rs = np.random.RandomState(1)
        sizes = [synthetic.COCO_SIZES[rs.randint(len(synthetic.COCO_SIZES))] for _ in range(5000)]
        want = set(parse(a.config4))
        for c in distributed.size_batches(sizes, eng.max_batch):
            if set(c) & want:
                jobs.append(("config4", c, [config4_image(i, sizes).float() / 255 for i in c], want))
    for i in parse(a.leg):
        jobs.append(("leg", [i], [synthetic.make_batch(1, 640, 640, seed=7000 + i)[0]], {i}))
    for tag, c, batch, want in jobs:
        eng(batch)
        plan = eng.plan(len(c), *batch[0].shape[-2:])
        torch.cuda.synchronize()
        ec, er = plan.cls_logits.tensor().cpu().double(), plan.bbox_regression.tensor().cpu().double()
        sel = [b for b, i in enumerate(c) if i in want]
        with torch.no_grad():
            ref = {dt: o.forward_raw([batch[b] for b in sel])[:2] for dt, o in orc.items()}
        t_c, t_r = (x.double() for x in ref[torch.float64])
        f_c, f_r = (x.double() for x in ref[torch.float32])
        for k, b in enumerate(sel):
            row = []
            for name, e, f, t in (("cls", ec[b], f_c[k], t_c[k]), ("reg", er[b], f_r[k], t_r[k])):
                de, df = (e - t).abs(), (f - t).abs()
                row.append(f"{name}: engine max {de.max():.2e} rms {de.pow(2).mean().sqrt():.2e} | f32 max "
                           f"{df.max():.2e} rms {df.pow(2).mean().sqrt():.2e} | engine-f32 max {(e - f).abs().max():.2e}")
            print(f"{tag} image {c[b]} ({tuple(batch[b].shape[-2:])}, batch {len(c)}): " + "; ".join(row), flush=True)


if __name__ == "__main__":
    main()
