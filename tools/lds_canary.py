"""LDS canary against the conv tiles (diagnostic, needs a GPU; see tools/lds_canary.hip).

    python tools/lds_canary.py [--iters 40000] [--reps 3]

For each conv variant a canary grid (one 256-thread workgroup per CU slot, 4 KB of LDS each, holding a
known pattern) is launched on one stream and the conv is launched back to back on a second stream, so
the conv's workgroups share CUs with the canaries; the canaries count every LDS word that changed
under them.  Variants: the exact-fp32 MFMA tile 3 (no LDS-DMA), the bf16x6 tile 30 (two register
stages, no LDS-DMA) and the bf16x6 tiles that stage their weight planes by LDS-DMA (29, 31, 25, 39).
A nonzero count with the LDS-DMA tiles and zero without them shows an LDS-DMA write landing outside
its workgroup's allocation.
"""
import argparse
import ctypes
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "tools", "liblds_canary.so")


def build():
    src = os.path.join(ROOT, "tools", "lds_canary.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", SO])
    return SO


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--words", type=int, default=1024)
    ap.add_argument("--convs", type=int, default=400)
    args = ap.parse_args()
    lib = ctypes.CDLL(build())
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    B, H, W, C, k = 2, 50, 50, 256, 3
    x = torch.randn(B, H, W, C, generator=g).to(dev)
    w = torch.randn(C, C, k, k, generator=g) / (9 * C) ** 0.5
    wp = torch.from_numpy(pack_conv_weight(w.numpy())[0]).to(dev)
    w3 = ops.split_bf16x3(wp)
    bias = torch.zeros(C, device=dev)
    bad = torch.zeros(4, dtype=torch.int32, device=dev)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ref = {}
    for tile in (None, 3, 30, 29, 31, 25, 39) * args.reps:
        bad.zero_()
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(sa)
        rc = lib.lds_canary_launch(ctypes.c_void_p(bad.data_ptr()), args.grid, args.iters, args.words,
                                   ctypes.c_void_p(sa.cuda_stream))
        assert rc == 0
        e1.record(sa)
        n = 0
        if tile is not None:
            with torch.cuda.stream(sb):
                for _ in range(args.convs):
                    y = ops.conv2d_nhwc(x, wp, bias, C, k, 1, 1, None, tile=tile, w3=None if tile == 3 else w3)
                    n += 1
                e2.record(sb)
        torch.cuda.synchronize()
        same = None
        if tile is not None:
            if tile not in ref:
                ref[tile] = y.clone()
            same = bool(torch.equal(ref[tile], y))
        b = bad.cpu().tolist()
        print(f"tile {tile}: canary {e0.elapsed_time(e1):.2f} ms, convs "
              f"{(e0.elapsed_time(e2) if tile is not None else 0):.2f} ms; corrupted LDS words {b[0]} "
              f"(first value {b[1]:#x} at word {b[2]}); conv output reproducible: {same}", flush=True)


if __name__ == "__main__":
    main()
