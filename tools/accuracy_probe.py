"""Arithmetic accuracy of the conv kernels against float64 (diagnostic; needs a GPU).

    python tools/accuracy_probe.py

1. Error of one FRCNN-shaped conv (3x3 256 -> 256, K = 2304; 1x1 1024 -> 256; 1x1 2048 -> 512; the box
   head's fc6, 1x1 12544 -> 1024 over 1,000 RoIs) against a float64 conv: the bf16x6 tiles, the fp32
   MFMA kernels, the plain fmaf-chain tile (3) and torch's CPU fp32 conv (the oracle's arithmetic).
   Max and RMS error and mean (bias) relative to max |y|.
2. The matrix cores' accumulation: a 1x1 conv whose one output sums 1.0 and 31 (or 63) copies of
   t = 2^-25 (every term exact in bf16 and its products exact): the exact sum is 1 + 31 t =
   1 + 7.75 ulp(1).  Round-to-nearest of the exact sum gives 1 + 8 ulp, truncation 1 + 7, and a
   sequential fp32 chain 1 + 0 (each t is a quarter ulp).  Printed in ulps of 1.0.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def conv_errors():
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    dev = "cuda"
    # tiles: 39 / 25 / 29 / 31 / 38 / 21 the bf16x6 kernels (stage sums since round 6), 3 the exact-fp32
    # MFMA tile with the plain fmaf chain (the accuracy reference), 5 / 14 / 16 the fp32 MFMA kernels
    # with stage sums; the last case is the FRCNN box head's fc6 at 1,000 RoIs (K = 12,544)
    for (B, H, W, Cin, Cout, k, tiles) in ((1, 100, 100, 256, 256, 3, (39, 25, 29, 31, 21, 3, 5)),
                                           (1, 50, 50, 1024, 256, 1, (39, 25, 3, 16)),
                                           (1, 25, 25, 2048, 512, 1, (39, 25, 3, 16)), (2, 56, 56, 64, 64, 3, (38, 3)),
                                           (1000, 1, 1, 12544, 1024, 1, (25, 14, 3))):
        g = torch.Generator().manual_seed(3)
        # post-ReLU activations (non-negative) and zero-mean weights, as in the ResNet body
        x = torch.relu(torch.randn(B, Cin, H, W, generator=g))
        w = torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5
        b = torch.randn(Cout, generator=g) * 0.1
        ref = F.conv2d(x.double(), w.double(), b.double(), 1, (k - 1) // 2)
        scale = ref.abs().max().item()
        res = {}
        cpu = F.conv2d(x, w, b, 1, (k - 1) // 2).double()
        res["cpu_f32"] = cpu - ref
        wp = torch.from_numpy(pack_conv_weight(w.numpy())[0]).to(dev)
        xd = x.permute(0, 2, 3, 1).contiguous().to(dev)
        w3 = ops.split_bf16x3(wp)
        for t in tiles:
            y = ops.conv2d_nhwc(xd, wp, b.to(dev), Cout, k, 1, (k - 1) // 2, None, tile=t,
                                w3=w3 if t >= 21 else None)
            res[f"tile{t}"] = y.permute(0, 3, 1, 2).double().cpu() - ref
        line = " ".join(f"{n}: max {e.abs().max().item() / scale:.2e} rms {e.pow(2).mean().sqrt().item() / scale:.2e} "
                        f"bias {e.mean().item() / scale:+.1e}" for n, e in res.items())
        print(f"conv {Cin}->{Cout} k{k} K={Cin * k * k} |y|max {scale:.2f}: {line}", flush=True)


def accumulation():
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    dev = "cuda"
    t = 2.0 ** -25
    for K in (32, 64, 256):
        x = torch.full((1, 1, 1, K), t)
        x[..., 0] = 1.0
        w = torch.ones(16, K, 1, 1)
        wp = torch.from_numpy(pack_conv_weight(w.numpy())[0]).to(dev)
        w3 = ops.split_bf16x3(wp)
        exact = (1 + (K - 1) * t - 1) / 2.0 ** -23
        out = {}
        for tile in (3, 25, 39, 31):
            y = ops.conv2d_nhwc(x.to(dev), wp, torch.zeros(16, device=dev), 16, 1, 1, 0, None, tile=tile,
                                w3=None if tile == 3 else w3)
            out[tile] = (y[0, 0, 0, 0].item() - 1.0) / 2.0 ** -23
        print(f"K={K}: exact 1 + {exact:.2f} ulp; tiles " + ", ".join(f"{k}: 1 + {v:.2f} ulp" for k, v in out.items()),
              flush=True)
        # the same terms with 1.0 LAST in K order: the small terms accumulate first
        x2 = torch.full((1, 1, 1, K), t)
        x2[..., K - 1] = 1.0
        out = {}
        for tile in (3, 25, 39):
            y = ops.conv2d_nhwc(x2.to(dev), wp, torch.zeros(16, device=dev), 16, 1, 1, 0, None, tile=tile,
                                w3=None if tile == 3 else w3)
            out[tile] = (y[0, 0, 0, 0].item() - 1.0) / 2.0 ** -23
        print(f"K={K} (1.0 last): tiles " + ", ".join(f"{k}: 1 + {v:.2f} ulp" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    accumulation()
    conv_errors()
