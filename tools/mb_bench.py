"""Time the fused MBConv front (ops.mbconv_front_nhwc) against the unfused expand conv + depthwise
pair on the SSDLite shapes (B=16 per chain).  python tools/mb_bench.py"""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from edgeml_amd import ops  # noqa: E402
from edgeml_amd.plan import pack_conv_weight, pack_dw_weight  # noqa: E402

SHAPES = {"b0.2": (16, 160, 160, 16, 64, 3, 2), "b0.3": (16, 80, 80, 24, 72, 3, 1),
          "b0.7": (16, 40, 40, 40, 240, 3, 2), "b0.8": (16, 20, 20, 80, 200, 3, 1)}


def timed(f, reps=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, (B, H, W, Cin, C, k, s) in SHAPES.items():
    x = torch.randn(B, H, W, Cin, device="cuda")
    w1 = torch.from_numpy(pack_conv_weight(torch.randn(C, Cin, 1, 1).numpy())[0]).cuda()
    b1 = torch.randn(C, device="cuda")
    w2 = torch.from_numpy(pack_dw_weight(torch.randn(C, 1, k, k).numpy())).cuda()
    b2 = torch.randn(C, device="cuda")
    fused = timed(lambda: ops.mbconv_front_nhwc(x, w1, b1, "RE", w2, b2, k, s, "RE"))
    e = ops.conv2d_nhwc(x, w1, b1, C, 1, 1, 0, "RE")
    t_exp = timed(lambda: ops.conv2d_nhwc(x, w1, b1, C, 1, 1, 0, "RE"))
    t_dw = timed(lambda: ops.dwconv2d_nhwc(e, w2, b2, k, s, (k - 1) // 2, "RE"))
    print(f"{name}: fused {fused:7.1f} us | expand {t_exp:6.1f} + dw {t_dw:6.1f} = {t_exp + t_dw:6.1f} us", flush=True)
