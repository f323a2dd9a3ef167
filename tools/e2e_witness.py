"""End-to-end FRCNN witness attribution over bench.py's ORIE-leg images (tests/e2e_witness.py).

    python tools/e2e_witness.py --ref f64|f32 --side engine|f32 [--images 0-47] [-o out.json]

--ref    the reference side: the CPU oracle in float32, or with its dense arithmetic in float64 (the
         ground truth of bench.py's `vs_f64`, tests/golden/g5_orie_f64.npz)
--side   the side checked against it: the HIP engine at batch 1 (as the ORIE leg runs it; needs a GPU),
         or the float32 CPU oracle (runs anywhere: the machinery checked on two CPU restatements)
Prints one line per image and the merged report; failures are listed, not raised.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_images(s):
    out = []
    for part in s.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="f32", choices=["f32", "f64"])
    ap.add_argument("--side", default="engine", choices=["engine", "f32"])
    ap.add_argument("--images", default="0-47")
    ap.add_argument("-o", default="")
    args = ap.parse_args()
    from edgeml_amd import synthetic
    from edgeml_amd.distributed import usable_cpus
    from oracle.frcnn import FasterRCNNOracle
    from tests import e2e_witness as W
    torch.set_num_threads(usable_cpus())
    z = np.load(os.path.join(ROOT, "tests", "golden", "g5_orie_f64.npz"))
    sd = synthetic.synthetic_state_dict("faster_rcnn", 91)
    ref = FasterRCNNOracle(sd, 91, dtype=torch.float64 if args.ref == "f64" else torch.float32)
    if args.side == "engine":
        from edgeml_amd import models
        eng = models.FasterRCNNFPNv2(sd, 91).to("cuda")
    else:
        other = FasterRCNNOracle(sd, 91)
    reps, fails = [], []
    for i in parse_images(args.images):
        img = synthetic.make_batch(1, 640, 640, seed=int(z["seeds"][i]))
        assert float(img.double().sum()) == float(z["image_sums"][i]), "regenerated input differs from G5's"
        t0 = time.perf_counter()
        A = W.oracle_side(ref, img[0])
        if args.side == "engine":
            eng(img.cuda())
            plan = eng.plan(1, 640, 640)
            B = W.engine_side(plan, 0, A["anchors"])
        else:
            B = W.oracle_side(other, img[0])
        scale = np.asarray([np.float32(640) / np.float32(A["size"][1]), np.float32(640) / np.float32(A["size"][0])] * 2,
                           np.float32)
        rep, f = W.check_image(A, B, 91, scale, (640, 640))
        reps.append(rep)
        fails += [(i,) + tuple(x) for x in f]
        print(f"image {i}: {time.perf_counter() - t0:.1f}s {json.dumps(rep)}" + (f"  FAIL {f}" if f else ""), flush=True)
    out = {"ref": args.ref, "side": args.side, "images": len(reps), "merged": W.merge(reps),
           "failures": [str(x) for x in fails]}
    print(json.dumps(out, indent=1))
    if args.o:
        with open(args.o, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
