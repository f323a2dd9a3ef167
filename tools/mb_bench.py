"""Microbench of the fused InvertedResidual kernel (MBCONV record, csrc/layers.hip mbconv_kernel) on the
SSDLite shapes it serves (one 16-image chain): block 0.2 (16 -> 64 -> 24, 3x3 s2 at 160^2) and block
0.3 (24 -> 72 -> 24, 3x3 s1 at 80^2, residual).  Random weights; prints the average launch time and the
algorithmic rates.  Run under rocprofv3 for counters.

    python tools/mb_bench.py [--reps 50] [--shapes b02,b03]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {  # B, H, W, Cin, Cexp, Cout, k, stride, act
    "b02": (16, 160, 160, 16, 64, 24, 3, 2, "RE"),
    "b03": (16, 80, 80, 24, 72, 24, 3, 1, "RE"),
}


def record(B, H, W, Cin, E, Cout, k, s, act):
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight, pack_dw_weight
    g = torch.Generator().manual_seed(1)
    w1 = torch.randn(E, Cin, 1, 1, generator=g) / Cin ** 0.5
    wd = torch.randn(E, 1, k, k, generator=g) / k
    w2 = torch.randn(Cout, E, 1, 1, generator=g) / E ** 0.5
    pad = (k - 1) // 2
    Ho, Wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    p1, _, kp1, _ = pack_conv_weight(w1.numpy())
    p2, _, kp2, _ = pack_conv_weight(w2.numpy())
    keep = [torch.randn(B, H, W, Cin, generator=g).cuda()]
    keep += [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in
             (p1, np.zeros(E, np.float32) + 0.1, pack_dw_weight(wd.numpy()), np.zeros(E, np.float32) + 0.1, p2,
              np.zeros(Cout, np.float32))]
    keep.append(torch.empty(B, Ho, Wo, Cout, device="cuda"))
    rec = np.zeros(1, dtype=ops.OP_DTYPE)
    rec[0]["kind"] = ops.MBCONV
    res = int(s == 1 and Cin == Cout)
    for j, v in enumerate((B, H, W, Cin, E, Cout, Ho, Wo, k, s, pad, ops.ACT[act], kp1, kp2, res)):
        rec[0]["i"][j] = v
    for j, t in enumerate(keep):
        rec[0]["p"][j] = t.data_ptr()
    flops = 2.0 * B * (H * W * Cin * E + Ho * Wo * E * (k * k + Cout))
    byts = 4.0 * (B * H * W * Cin + B * Ho * Wo * Cout)
    return rec, keep, flops, byts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--shapes", default="b02,b03")
    a = ap.parse_args()
    from edgeml_amd import ops
    L = ops.lib()
    for name in a.shapes.split(","):
        rec, keep, flops, byts = record(*SHAPES[name])
        # the launches replayed from one hipGraph, so the host's per-launch cost cannot set the rate
        recs = np.repeat(rec, a.reps)
        stream = torch.cuda.Stream()
        sh = ops.stream_handle(stream)
        ops.check(L.edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, sh))
        g = ctypes.c_void_p()
        ops.check(L.edgedet_graph_create(recs.ctypes.data_as(ctypes.c_void_p), len(recs), sh, ctypes.byref(g)))
        ops.check(L.edgedet_graph_launch(g, sh))
        stream.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ops.check(L.edgedet_graph_launch(g, sh))
        e1.record(stream)
        e1.synchronize()
        L.edgedet_graph_destroy(g)
        ms = e0.elapsed_time(e1) / a.reps
        print(f"{name}: {ms * 1e3:.1f} us  {flops / ms / 1e9:.1f} TFLOP/s  {byts / ms / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
