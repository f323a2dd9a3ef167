"""Layer-by-layer error of the engine's Faster R-CNN backbone + FPN against the float64 oracle
(measurement tool; needs a GPU).

    python tools/layer_error.py [--image 0]

The engine runs one of bench.py's ORIE-leg images (synthetic.make_batch(1, 640, 640, seed=7000 + i)) at
batch 1 and its plan buffers are read back (named by the conv that writes them: the post-BatchNorm,
post-residual, post-ReLU output); the CPU oracle computes the same tensors in float32 and in float64
(oracle/frcnn.py's arithmetic, layer by layer).  Printed per layer: max and RMS of |value - float64|
relative to the layer's max |float64| for the engine and for the float32 oracle, and the RMS ratio.
Errors propagate, so the place where the ratio rises is where the engine adds error of its own.
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def oracle_layers(x, sd):
    """oracle/frcnn.py resnet_body + fpn, recording each conv's output as the engine's buffer holds it."""
    from oracle import frcnn as Fr
    out = {}
    p = "backbone.body."
    x = F.relu(Fr.bn(Fr.conv(x, sd, p + "conv1", 2), sd, p + "bn1"))
    out[p + "conv1.weight"] = x
    x = F.max_pool2d(x, 3, 2, 1)
    out[p + "maxpool"] = x
    cs = []
    for name, nblk, width, stride in Fr.LAYERS:
        for b in range(nblk):
            q = f"{p}{name}.{b}."
            s = stride if b == 0 else 1
            y = F.relu(Fr.bn(Fr.conv(x, sd, q + "conv1"), sd, q + "bn1"))
            out[q + "conv1.weight"] = y
            y = F.relu(Fr.bn(Fr.conv(y, sd, q + "conv2", s), sd, q + "bn2"))
            out[q + "conv2.weight"] = y
            y = Fr.bn(Fr.conv(y, sd, q + "conv3"), sd, q + "bn3")
            if b == 0:
                idn = Fr.bn(Fr.conv(x, sd, q + "downsample.0", s), sd, q + "downsample.1")
                out[q + "downsample.0.weight"] = idn
            else:
                idn = x
            x = F.relu(y + idn)
            out[q + "conv3.weight"] = x
        cs.append(x)
    f = "backbone.fpn."
    inner = lambda i, t: Fr.bn(Fr.conv(t, sd, f"{f}inner_blocks.{i}.0"), sd, f"{f}inner_blocks.{i}.1")  # noqa: E731
    layer = lambda i, t: Fr.bn(Fr.conv(t, sd, f"{f}layer_blocks.{i}.0"), sd, f"{f}layer_blocks.{i}.1")  # noqa: E731
    last = inner(3, cs[3])
    out[f"{f}inner_blocks.3.0.weight"] = last
    out[f"{f}layer_blocks.3.0.weight"] = layer(3, last)
    for i in (2, 1, 0):
        lat = inner(i, cs[i])
        last = lat + F.interpolate(last, size=lat.shape[-2:], mode="nearest")
        out[f"{f}inner_blocks.{i}.0.weight"] = last
        out[f"{f}layer_blocks.{i}.0.weight"] = layer(i, last)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", type=int, default=0)
    a = ap.parse_args()
    from edgeml_amd import models, synthetic
    from edgeml_amd.distributed import usable_cpus
    from oracle import frcnn as Fr
    from oracle import tv_ops
    from oracle.ssdlite import _SD
    torch.set_num_threads(usable_cpus())
    sd = synthetic.synthetic_state_dict("faster_rcnn", 91)
    eng = models.FasterRCNNFPNv2(sd, 91).to("cuda")
    img = synthetic.make_batch(1, 640, 640, seed=7000 + a.image)
    eng(img.cuda())
    plan = eng.plan(1, 640, 640)
    torch.cuda.synchronize()
    ref = {}
    with torch.no_grad():
        for dt in (torch.float32, torch.float64):
            o = Fr.FasterRCNNOracle(sd, 91, dtype=dt)
            x, _ = tv_ops.transform([img[0]], Fr.MEAN, Fr.STD, Fr.MIN_SIZE, Fr.MAX_SIZE, divisible=Fr.DIVISIBLE)
            ref[dt] = {"pre": x.to(dt)}
            ref[dt].update(oracle_layers(x.to(dt), _SD(o.sd)))
    t64, t32 = ref[torch.float64], ref[torch.float32]
    print(f"{'layer':48s} {'engine max':>10s} {'rms':>9s} | {'f32 max':>9s} {'rms':>9s} | rms ratio", flush=True)
    for name, t in t64.items():
        if name not in plan.buffers:
            continue
        e = plan.buffers[name].tensor().detach().cpu().double().numpy()[0]
        t = t[0].numpy()
        if e.ndim == 3 and e.shape[-1] != t.shape[0]:
            e = e[..., :t.shape[0]]  # NHWC4 padding of the transform output
        e = e.transpose(2, 0, 1) if e.ndim == 3 else e
        e = e[:, :t.shape[1], :t.shape[2]]
        f = t32[name][0].double().numpy()
        s = max(np.abs(t).max(), 1e-30)
        de, df = e - t, f - t
        re, rf = np.sqrt((de ** 2).mean()) / s, np.sqrt((df ** 2).mean()) / s
        print(f"{name:48s} {np.abs(de).max() / s:10.2e} {re:9.2e} | {np.abs(df).max() / s:9.2e} {rf:9.2e} | "
              f"{re / max(rf, 1e-30):6.2f}", flush=True)


if __name__ == "__main__":
    main()
