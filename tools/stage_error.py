"""Where the engine's Faster R-CNN deviates from the float64 oracle, stage by stage (measurement tool).

    python tools/stage_error.py [--images 0,1,2] [--batch 1]

For each of bench.py's ORIE-leg images (synthetic.make_batch(1, 640, 640, seed=7000 + i)) the engine
runs at the given batch and its plan buffers are read back: the FPN levels P2..P6, the RPN head outputs
(objectness, deltas), and the box stage's class scores for the engine's own proposals.  The CPU oracle
computes the same tensors in float32 and in float64 (oracle dtype=torch.float64; the box stage cross-fed
the engine's proposals, so that stage compares arithmetic alone).  Printed per stage: the largest
|value - float64| scaled by the stage's largest |float64| value, for the engine and for the float32
oracle, and their ratio.  A float32-grade engine stage reads within a small factor of the float32
oracle; a stage far above it is where precision is lost.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rel(a, ref):
    a, ref = np.asarray(a, np.float64), np.asarray(ref, np.float64)
    return float(np.abs(a - ref).max() / max(np.abs(ref).max(), 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", default="0,1,2")
    ap.add_argument("-o", default="")
    a = ap.parse_args()
    from edgeml_amd import models, synthetic
    from edgeml_amd.distributed import usable_cpus
    from oracle import frcnn as Fr
    from oracle import tv_ops
    from oracle.ssdlite import _SD
    torch.set_num_threads(usable_cpus())
    sd = synthetic.synthetic_state_dict("faster_rcnn", 91)
    eng = models.FasterRCNNFPNv2(sd, 91).to("cuda")
    orc = {dt: Fr.FasterRCNNOracle(sd, 91, dtype=dt) for dt in (torch.float32, torch.float64)}
    report = []
    for i in (int(v) for v in a.images.split(",")):
        img = synthetic.make_batch(1, 640, 640, seed=7000 + i)
        eng(img.cuda())
        plan = eng.plan(1, 640, 640)
        torch.cuda.synchronize()
        feats_e = [f.tensor().cpu().numpy()[0].transpose(2, 0, 1) for f in plan.feats]  # NHWC -> CHW
        heads_e = [(o.tensor().cpu().numpy().reshape(-1), d.tensor().cpu().numpy().reshape(-1)) for o, d in plan.rpn_heads]
        pc = int(plan.proposal_count.tensor().cpu()[0])
        props = torch.from_numpy(plan.proposals.tensor().cpu().numpy()[0, :pc].copy())
        bsc_e = plan.box_scores.tensor().cpu().numpy()[0, :pc]
        out = {}
        with torch.no_grad():
            for dt, o in orc.items():
                osd = _SD(o.sd)
                x, sizes = tv_ops.transform([img[0]], Fr.MEAN, Fr.STD, Fr.MIN_SIZE, Fr.MAX_SIZE, divisible=Fr.DIVISIBLE)
                body = Fr.resnet_body(x.to(dt), osd)
                feats = Fr.fpn(body, osd)
                objs, dels, _ = Fr.rpn_head(feats, osd, tuple(x.shape[-2:]))
                logits, _ = o.box_stage(feats, [props], sizes)
                out[dt] = {"feats": [f[0].double().numpy() for f in feats],
                           "obj": [t[0].double().numpy().reshape(-1) for t in objs],
                           "del": [t[0].double().numpy().reshape(-1) for t in dels],
                           "scores": torch.softmax(logits.double(), -1).numpy()}
        t, f = out[torch.float64], out[torch.float32]
        row = {"image": i}
        for lvl in range(5):
            row[f"P{lvl + 2}"] = (rel(feats_e[lvl], t["feats"][lvl]), rel(f["feats"][lvl], t["feats"][lvl]))
            row[f"rpn_obj{lvl}"] = (rel(heads_e[lvl][0], t["obj"][lvl]), rel(f["obj"][lvl], t["obj"][lvl]))
            row[f"rpn_del{lvl}"] = (rel(heads_e[lvl][1], t["del"][lvl]), rel(f["del"][lvl], t["del"][lvl]))
        row["box_scores"] = (float(np.abs(bsc_e - t["scores"]).max()), float(np.abs(f["scores"] - t["scores"]).max()))
        for k, v in row.items():
            if k != "image":
                e, r = v
                print(f"image {i} {k:10s} engine {e:.3e}  f32 oracle {r:.3e}  ratio {e / max(r, 1e-30):7.2f}", flush=True)
        report.append(row)
    if a.o:
        with open(a.o, "w") as fh:
            json.dump(report, fh, indent=1)


if __name__ == "__main__":
    main()
