"""Diagnostic: does a replay of the SSD b=32 plan change its own input buffer?  Copies a batch into
'images', checks it, replays (graph) or runs (eager) the plan, checks again; on a change, describes the
new contents (which bytes, and whether they match another batch or another buffer of the plan)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--eager", action="store_true")
    a = ap.parse_args()
    from edgeml_amd import models, synthetic
    m = models.SSDLite320(synthetic.synthetic_state_dict("ssd", 91, True, seed=0), 91, True).to("cuda:0")
    plan = m.build_plan(32, 640, 640, True)
    s = torch.cuda.Stream()
    img = synthetic.make_batch_u8(32, 640, 640, seed=7).cuda()
    alt = synthetic.make_batch_u8(32, 640, 640, seed=8).cuda()
    inp = plan.input.tensor()
    print("input buffer", inp.shape, inp.dtype, "offset", inp.data_ptr() - plan.arena.data_ptr(), flush=True)
    if not a.eager:
        plan.capture(s)
    torch.cuda.synchronize()
    for r in range(a.reps):
        inp.copy_(img)
        torch.cuda.synchronize()
        assert torch.equal(inp, img)
        if a.eager:
            plan.run(s)
        else:
            plan.replay(s)
        torch.cuda.synchronize()
        same = torch.equal(inp, img)
        msg = f"rep {r}: input unchanged after the {'run' if a.eager else 'replay'}: {same}"
        if not same:
            d = (inp != img).flatten()
            nz = d.nonzero().flatten()
            msg += f"; {int(d.sum())} bytes changed, offsets {int(nz.min())}..{int(nz.max())}"
            msg += f"; equals the seed-8 batch: {torch.equal(inp, alt)}; equals zeros: {bool((inp == 0).all())}"
        print(msg, flush=True)


if __name__ == "__main__":
    main()
