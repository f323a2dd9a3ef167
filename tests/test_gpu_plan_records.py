"""Record-level equivalences of the native executor:

* a GROUP record (EDGEDET_OP_GROUP, csrc/exec.hip run_group) issues its members as ONE grouped launch
  (conv_x6b_group_kernel / dwconv_rb_group_kernel: each member's block range offset by start[k], the
  XCD remap per member); its results must equal the members issued one by one, bit for bit.  Checked
  on every GROUP record of the bench plans: the SSDLite heads (12 depthwise members of six map sizes,
  12 pointwise members with Cout 546 / 24, strided outputs at map offsets, tile 31) and the FRCNN RPN
  head levels (five M sizes, tile 39);
* the chunked RPN top-k (RPN_LEVEL_NMS with the p20..p22 chunk scratch, csrc/detect.hip
  rpn_chunk_select_kernel) must equal the single-pass level selection bit for bit, also when exact
  ties cross the 8,192-anchor chunk and the 4,096-key compaction batch boundaries, and on a level with
  fewer anchors than the top-k (P6: 507 < 1,000); the chunk union's selection from registers (the
  default when the union fits 32 keys per thread) against the radix selection of the single pass;
* the split NMS (p23 scratch: selection / IoU mask over many workgroups / scan) equal to the one-
  workgroup-per-segment kernel, chunked or not.
"""
import ctypes

import numpy as np
import pytest
import torch

from edgeml_amd import models, ops, synthetic

pytestmark = pytest.mark.gpu


def _run(recs):
    ops.check(ops.lib().edgedet_plan_run(recs.ctypes.data_as(ctypes.c_void_p), len(recs), ops.stream_handle()))
    torch.cuda.synchronize()


def _region(plan, ptr, nbytes):
    off = int(ptr) - plan.arena.data_ptr()
    assert 0 <= off and off + nbytes <= plan.arena.numel(), (off, nbytes)
    return plan.arena[off:off + nbytes]


def _out_extent(rec):
    """(first byte, byte count) a CONV / DWCONV record writes (csrc/exec.hip conv_params / dw_params)."""
    i = rec["i"]
    if rec["kind"] == ops.CONV:
        B, Ho, Wo, Cout, yp, yb, yoff = (int(i[j]) for j in (0, 4, 5, 6, 15, 18, 20))
        return int(rec["p"][3]) + 4 * yoff, 4 * ((B - 1) * yb + (Ho * Wo - 1) * yp + Cout)
    B, Ho, Wo, C = (int(i[j]) for j in (0, 4, 5, 3))
    return int(rec["p"][3]), 4 * B * Ho * Wo * C


def _plans():
    sd_ssd = synthetic.synthetic_state_dict("ssd", 91, True)
    ssd = models.SSDLite320(sd_ssd, 91, True).to("cuda")
    frc = models.FasterRCNNFPNv2(synthetic.synthetic_state_dict("faster_rcnn", 91), 91).to("cuda")
    return [("ssd b=32", ssd, 32), ("frcnn b=1", frc, 1)]


@pytest.mark.parametrize("which", [0, 1])
def test_group_launch_equals_members_one_by_one(which):
    name, m, B = _plans()[which]
    imgs = synthetic.make_batch(B, 640, 640, seed=41 + which)
    m(imgs.cuda())                       # every buffer of the plan holds a real forward's values
    plan = m.plan(B, 640, 640)
    groups = [k for k, op in enumerate(plan.ops) if op.kind == ops.GROUP]
    assert groups, name
    kinds = set()
    for k in groups:
        n = int(plan.records[k]["i"][0])
        recs = plan.records[k:k + 1 + n].copy()
        recs["i"][:, ops.LANE_FIELD] = 0
        outs = [_region(plan, *_out_extent(r)) for r in recs[1:]]
        got = []
        for sub in (recs, recs[1:]):     # the grouped launch, then the members one by one
            for o in outs:
                o.fill_(0xFF)
            _run(sub)
            got.append([o.clone() for o in outs])
        for j, (a, b) in enumerate(zip(*got)):
            assert torch.equal(a, b), (name, plan.ops[k + 1 + j].name)
        kinds.add(int(recs[1]["kind"]))
        if recs[1]["kind"] == ops.CONV:  # members of different M, Cout and output strides in one launch
            assert len({(int(r["i"][4]), int(r["i"][6]), int(r["i"][15])) for r in recs[1:]}) > 1 or n == 1
    assert kinds == ({ops.CONV, ops.DWCONV} if which == 0 else {ops.CONV}), (name, kinds)


@pytest.mark.parametrize("size", [(640, 640), (427, 640)])
@pytest.mark.parametrize("pattern", ["quantized", "all_equal", "continuous", "two_values"])
def test_rpn_chunked_split_equal_single_pass(pattern, size):
    """The four RPN selection forms write the same records.  640 x 640 (resized 800 x 800): P2's 15
    chunks take the split selection's register bisection; 427 x 640 (a COCO size, resized 800 x 1199,
    padded 800 x 1216): P2's 23 chunks exceed its 16 and take the radix select + compact fallback."""
    B = 2
    m = models.FasterRCNNFPNv2(synthetic.synthetic_state_dict("faster_rcnn", 91), 91).to("cuda")
    plan = m.plan(B, *size)
    k = next(j for j, op in enumerate(plan.ops) if op.kind == ops.RPN_LEVEL_NMS)
    rec = plan.records[k:k + 1].copy()
    rec["i"][0, ops.LANE_FIELD] = 0
    L, KM = int(rec["i"][0, 1]), int(rec["i"][0, 5])
    ns = [int(rec["i"][0, 6 + l]) for l in range(L)]
    assert max(ns) > 8192 * 4 and min(ns) < 1000, ns  # several chunks at P2, n < topk at P6
    nch = (max(ns) + 8191) // 8192
    assert (nch <= 16) == (size == (640, 640)), (ns, nch)  # the register path's limit: 16 chunks
    assert rec["p"][0, 20] and rec["i"][0, 16] == 8192
    g = torch.Generator().manual_seed(hash(pattern) % 1000)
    for l, n in enumerate(ns):
        obj = _region(plan, rec["p"][0, l], B * n * 4).view(torch.float32)
        if pattern == "quantized":     # a handful of distinct values: ties everywhere, at every cut
            v = torch.round(torch.randn(B * n, generator=g) * 2) / 4
        elif pattern == "all_equal":   # the top-k is the first 1,000 indices of the level
            v = torch.full((B * n,), 0.5)
        elif pattern == "two_values":  # a high tie group straddling chunk and batch boundaries
            v = torch.where(torch.rand(B * n, generator=g) < 0.02, torch.tensor(1.0), torch.tensor(-1.0))
        else:
            v = torch.randn(B * n, generator=g)
        obj.copy_(v.cuda())
        d = _region(plan, rec["p"][0, 15 + l], B * n * 16).view(torch.float32)
        d.copy_((torch.randn(B * n * 4, generator=g) * 0.2).cuda())
    sizes = [B * L * KM * 16, B * L * KM * 4, B * L * KM * 4, B * L * KM * 4, B * L * 4]
    outs = [_region(plan, rec["p"][0, 10 + j], sizes[j]) for j in range(5)]
    assert rec["p"][0, 23], "the lowering's record carries the split-NMS scratch"
    got = []
    variants = [(True, True), (True, False), (False, True), (False, False)]  # (chunked, split)
    for chunked, split in variants:
        r = rec.copy()
        if not chunked:
            r["p"][0, 20:23] = 0
        if not split:
            r["p"][0, 23] = 0
        for o in outs:
            o.fill_(0xFF)
        _run(r)
        got.append([o.clone() for o in outs])
    cnt = got[0][4].view(torch.int32)
    assert (cnt > 0).all(), cnt
    for v in range(1, len(variants)):
        for j, (a, b) in enumerate(zip(got[0], got[v])):
            assert torch.equal(a, b), (pattern, variants[v], ["box", "score", "tb", "level", "count"][j])
