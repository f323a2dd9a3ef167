"""No kernel writes outside its buffers (the concurrency non-reproducibility).

The CPU check of tests/test_happens_before.py shows every lowering's records ordered at the record
level; what it cannot see is a kernel that writes past the extent its record declares -- into the
next buffer of the workspace, or past the workspace's end into whatever allocation follows it, which
with several plans in flight is another instance's workspace (its input images and first
activations sit at its start).  Such a write shows up only when it lands after the victim wrote its
own value, i.e. depending on timing.

edgedet_set_redzone(64 KiB) lowers every plan with 64 KiB left unused before, between and after the
workspace buffers.  The gaps are filled with a canary byte, the plan runs eagerly and from its
captured graph (repeatedly, with real inputs: the bench's synthetic images), and every gap must
still hold the canary.  Bytes between a buffer's declared size and its 256-byte round-up are
reported separately (harmless in production, where no buffer lives there).
"""
import pytest
import torch

from edgeml_amd import models, ops, synthetic

pytestmark = pytest.mark.gpu

RZ = 64 * 1024
CANARY = 0xA5


def _gaps(plan):
    """[(lo, hi, kind, preceding buffer name)] of the workspace not covered by a named buffer."""
    bufs = sorted(plan.buffers.values(), key=lambda b: b.off)
    out, end, prev = [], 0, "(workspace start)"
    for b in bufs:
        if b.off > end:
            out.append((end, b.off, "redzone", prev))
        pad_end = b.off + (b.nbytes + 255) // 256 * 256
        if pad_end > b.off + b.nbytes:
            out.append((b.off + b.nbytes, pad_end, "pad", b.name))
        end, prev = max(end, pad_end), b.name
    if plan.arena.numel() > end:
        out.append((end, plan.arena.numel(), "redzone", prev + " (workspace end)"))
    return out


CASES = [("ssd", 32, 640, 640, True), ("ssd", 2, 480, 640, False), ("frcnn", 8, 640, 640, True),
         ("frcnn", 2, 427, 640, False), ("retinanet", 2, 640, 640, True)]


@pytest.mark.parametrize("kind,B,H,W,u8", CASES)
def test_no_kernel_writes_outside_its_buffers(kind, B, H, W, u8):
    L = ops.lib()
    ops.check(L.edgedet_set_redzone(RZ))
    try:
        m = {"ssd": lambda: models.SSDLite320(synthetic.synthetic_state_dict("ssd", 91, True), 91, True),
             "frcnn": lambda: models.FasterRCNNFPNv2(synthetic.synthetic_state_dict("faster_rcnn", 91), 91),
             "retinanet": lambda: models.RetinaNetFPNv2(synthetic.synthetic_state_dict("retinanet", 91), 91)}[kind]()
        m = m.to("cuda")
        plan = m.build_plan(B, H, W, u8).finalize()
        gaps = _gaps(plan)
        assert sum(hi - lo for lo, hi, k, _ in gaps if k == "redzone") >= RZ * len(plan.buffers)
        for lo, hi, _, _ in gaps:   # slices, not a boolean mask (torch's masked ops overflow past 2^31 bytes)
            plan.arena[lo:hi].fill_(CANARY)
        src = synthetic.make_batch_u8(B, H, W, seed=77) if u8 else synthetic.make_batch(B, H, W, seed=77)
        plan.input.tensor().copy_(src.cuda())
        plan.run()
        s = torch.cuda.Stream()
        plan.capture(s)           # runs once more eagerly, then captures and replays twice
        for _ in range(5):
            plan.replay(s)
        torch.cuda.synchronize()
        assert int(plan.out_count.tensor().sum()) > 0
        counts = torch.stack([torch.count_nonzero(plan.arena[lo:hi] != CANARY) for lo, hi, _, _ in gaps]).cpu()
        hit = {}
        for (lo, hi, k, name), n in zip(gaps, counts.tolist()):
            if n:
                first = int(torch.nonzero(plan.arena[lo:hi] != CANARY)[0])
                hit[(k, name)] = (int(n), first)
        red = {k: v for k, v in hit.items() if k[0] == "redzone"}
        if hit:
            print("writes into gaps ((kind, buffer before the gap): (bytes, first offset into the gap)):", hit)
            assert not red, red
    finally:
        ops.check(L.edgedet_set_redzone(0))
