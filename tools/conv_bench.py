"""Microbenchmark of the conv kernel variants on the FRCNN layer shapes (device time per launch,
HIP events on the current stream).  python tools/conv_bench.py [--tiles 3,23,24] [--reps 20]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (B, H, W, Cin, Cout, k, stride)
    "box_head_3x3": (8000, 7, 7, 256, 256, 3, 1),
    "fpn_p2_3x3": (8, 200, 200, 256, 256, 3, 1),
    "fc6": (8000, 1, 1, 12544, 1024, 1, 1),
    "layer4_3x3": (8, 25, 25, 512, 512, 3, 1),
    "layer1_1x1": (8, 200, 200, 64, 256, 1, 1),
    "layer3_3x3": (8, 50, 50, 256, 256, 3, 1),
    "stem_7x7": (8, 800, 800, 4, 64, 7, 2),
    "ssd_head_cls0": (16, 20, 20, 672, 546, 1, 1),
    "ssd_head_cls1": (16, 10, 10, 480, 546, 1, 1),
    "ssd_f13": (16, 20, 20, 112, 672, 1, 1),
    "ssd_12_3": (16, 20, 20, 672, 112, 1, 1),
    "retina_cls": (8, 100, 100, 256, 819, 3, 1),
    "ssd_head_cls1b": (16, 10, 10, 480, 546, 1, 1),
    "layer1_3x3": (8, 200, 200, 64, 64, 3, 1),
    "layer1_1x1_in": (8, 200, 200, 256, 64, 1, 1),
    "ssd_02_expand": (16, 160, 160, 16, 64, 1, 1),
    "ssd_02_project": (16, 80, 80, 64, 24, 1, 1),
    "ssd_03_expand": (16, 80, 80, 24, 72, 1, 1),
    "ssd_03_project": (16, 80, 80, 72, 24, 1, 1),
    "ssd_04_project": (16, 40, 40, 72, 40, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,3,4,23,24")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    dev = "cuda"
    for name in a.shapes.split(","):
        B, H, W, Cin, Cout, k, s = SHAPES[name]
        pad = (k - 1) // 2
        x = torch.randn(B, H, W, Cin, device=dev)
        w = torch.randn(Cout, Cin, k, k) / (Cin * k * k) ** 0.5
        wp = torch.from_numpy(pack_conv_weight(w.numpy())[0]).to(dev)
        from edgeml_amd.plan import split_bf16x3
        w3 = torch.from_numpy(split_bf16x3(wp.cpu().numpy()).view(np.int16)).to(dev)  # host split: any library
        b = torch.zeros(Cout, device=dev)
        Ho = (H + 2 * pad - k) // s + 1
        Wo = (W + 2 * pad - k) // s + 1
        flops = 2.0 * B * Ho * Wo * Cout * k * k * Cin
        res = []
        for tv in a.tiles.split(","):  # "25p": tile 25 with the input pre-split (x3 scratch)
            t, ps = int(tv.rstrip("p")), tv.endswith("p")
            for use3 in ((False, True) if t == 0 else (t >= 20,)):
                f = lambda: ops.conv2d_nhwc(x, wp, b, Cout, k, s, pad, None if t == 26 else "RE", tile=t, w3=w3 if use3 else None,
                                            presplit=ps)
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    f()
                e1.record()
                e1.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res.append(f"tile{tv}{'x6' if use3 and t == 0 else ''}: {ms:.3f} ms {flops / ms / 1e9:.1f} TF")
        print(f"{name:14s} M={B * Ho * Wo} N={Cout} K={k * k * Cin}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
