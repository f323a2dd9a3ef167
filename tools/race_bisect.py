"""Diagnostic: which buffer of a plan first differs when a second plan instance runs concurrently.

    python tools/race_bisect.py [--kind frcnn] [--B 6] [--H 427] [--W 640] [--trials 8] [--eager]

Two instances of one (kind, B, H, W, u8) plan on two streams: instance 1 run alone gives the
reference contents of every named buffer; then both run at once (graph replays, or eager runs with
--eager) and instance 1's buffers are compared with the reference, listed in arena order (the
lowering's allocation order, which follows the op order)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="frcnn")
    ap.add_argument("--B", type=int, default=6)
    ap.add_argument("--H", type=int, default=427)
    ap.add_argument("--W", type=int, default=640)
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--n", type=int, default=2, help="instances in flight at once")
    ap.add_argument("--ref-after", type=int, default=0, help="extra solo runs before the reference is taken")
    ap.add_argument("--detail", default="", help="buffer name prefix to describe when it differs (count, max |diff|, where)")
    a = ap.parse_args()
    from edgeml_amd import models, synthetic
    if a.kind == "ssd":
        m = models.SSDLite320(synthetic.synthetic_state_dict("ssd", 91, True, seed=0), 91, True).to("cuda:0")
    else:
        m = models.fasterrcnn_resnet50_fpn_v2().to("cuda:0")
    plans = [m.build_plan(a.B, a.H, a.W, True) for _ in range(a.n)]
    streams = [torch.cuda.Stream() for _ in range(a.n)]
    imgs = [synthetic.make_batch_u8(a.B, a.H, a.W, seed=7 + k).cuda() for k in range(a.n)]
    for p, s in zip(plans, streams):
        if not a.eager:
            p.capture(s)
    torch.cuda.synchronize()

    def go(k):
        plans[k].input.tensor().copy_(imgs[k])
        torch.cuda.synchronize()
        if a.eager:
            plans[k].run(streams[k])
        else:
            plans[k].replay(streams[k])

    bufs = sorted(plans[0].buffers.values(), key=lambda b: b.off)
    go(0)
    torch.cuda.synchronize()
    for _ in range(a.ref_after):
        go(0)
        torch.cuda.synchronize()
    ref = {b.name: b.tensor().clone() for b in bufs}
    ref_host = {b.name: ref[b.name].cpu() for b in bufs}  # to tell a changed reference copy from a changed buffer
    for t in range(a.trials):
        for k in range(a.n):
            plans[k].input.tensor().copy_(imgs[k])
        torch.cuda.synchronize()
        for k in range(a.n) if t % 2 == 0 else reversed(range(a.n)):
            if a.eager:
                plans[k].run(streams[k])
            else:
                plans[k].replay(streams[k])
        torch.cuda.synchronize()
        bad = [b.name for b in bufs if not torch.equal(b.tensor(), ref[b.name])]
        print(f"trial {t}: {len(bad)} of {len(bufs)} buffers differ; first: {bad[:6]}", flush=True)
        moved = [n for n in ref if not torch.equal(ref[n].cpu(), ref_host[n])]
        if moved:
            print(f"  the device reference copies of {len(moved)} buffers changed since they were taken "
                  f"(writes into memory outside the plans): {moved[:6]}", flush=True)
        if "images" in bad:
            x, y = plans[0].input.tensor(), ref["images"]
            d = (x != y).flatten().nonzero().flatten()
            per_img = (x != y).flatten(1).sum(1).tolist() if x.dim() > 1 else []
            print(f"  images: {d.numel()} bytes differ, flat offsets {int(d.min())}..{int(d.max())}, per image "
                  f"{[(i, n) for i, n in enumerate(per_img) if n]}", flush=True)
        if a.detail:
            for b in bufs:
                if b.name.startswith(a.detail) and b.name in bad:
                    x, y = b.tensor(), ref[b.name]
                    if x.dtype != torch.float32 or x.dim() != 4:
                        continue
                    d = (x != y)
                    Bn, Hh, Ww, Cc = x.shape
                    pix = d.any(-1)  # [B, H, W]
                    imgs = pix.flatten(1).any(1).nonzero().flatten().tolist()
                    tiles = sorted({(int(i), int(h) // 16, int(w) // 16) for i, h, w in pix.nonzero().tolist()})
                    print(f"  {b.name}: {int(d.sum())} of {d.numel()} elements differ, max |diff| "
                          f"{float((x - y).abs().max()):.3e}, images {imgs}, {len(tiles)} differing 16x16 output "
                          f"tiles of {Bn * ((Hh + 15) // 16) * ((Ww + 15) // 16)}; first tiles {tiles[:8]}", flush=True)


if __name__ == "__main__":
    main()
