"""Model-level parity checks shared by the GPU tests (test infrastructure).

Each ``*_check`` takes a plan the engine has just run on `imgs` (plain run or graph replay), runs
the CPU oracle on the same images, and asserts the protocol of tests/flips.py:
  * raw head outputs agree to fp32 tolerance (RAW_TOL);
  * the decision replay of the engine's pre-decision values reproduces the engine's output rows
    (exactly where those values are read back from the device, to 1 ulp where they are recomputed
    on the host), and the replay of the oracle's values reproduces the oracle's own postprocess;
  * candidates are paired by identity: paired rows agree within north_star's 1e-3;
  * every candidate whose fate differs is a boundary flip: the deciding quantity on the oracle side
    lies within EPS_* of its boundary, directly or by cascade from such a flip.
FRCNN is checked stage by stage (RPN proposals from each side's own features, then the box stage
with the oracle's box head fed the engine's proposals), so a proposal flip cannot hide an error of
the box stage.  Returns a summary dict (printed by the tests).
"""
import numpy as np
import torch

from tests import chains
from tests.flips import check_replay_reproduces, classify, max_margin, paired_deltas, replay

RAW_TOL = 2e-3       # max |engine - oracle| of raw head outputs (logits / deltas)
EPS_SCORE = 1e-5     # class probability / sigmoid score: thresholds and order inversions
EPS_LOGIT = 1e-4     # RPN pre-NMS top-k key (objectness logit)
EPS_IOU = 1e-5       # NMS IoU straddles
TOL = 1e-3           # north_star: paired rows agree within 1e-3 (score absolute, box rel. to its size)


class _Acc:
    def __init__(self, what):
        self.what = what
        self.flips, self.paired, self.rows = 0, 0, 0
        self.margin = [0.0, 0.0, 0.0]   # score, key (logit), iou
        self.delta = [0.0, 0.0]         # paired |dscore|, box rel
        self.by = {}

    def add(self, rep, tA, tB, sA, sB, tag, key_stages=()):
        assert not rep["unexplained"], (self.what, tag, rep["unexplained"][:5])
        other = [k for k in ("filter", "topk", "nms", "cut") if k not in key_stages]
        ms = max_margin(rep, kinds=("straddle", "inversion"), stages=other)
        mk = max_margin(rep, kinds=("straddle", "inversion"), stages=key_stages) if key_stages else 0.0
        mi = max_margin(rep, kinds=("iou_straddle",))
        assert ms <= EPS_SCORE and mk <= EPS_LOGIT and mi <= EPS_IOU, (self.what, tag, ms, mk, mi, rep["by_stage"])
        npair, ds, db = paired_deltas(sA, tA, sB, tB)
        assert ds <= TOL and db <= TOL, (self.what, tag, ds, db)
        self.margin = [max(a, b) for a, b in zip(self.margin, (ms, mk, mi))]
        self.delta = [max(a, b) for a, b in zip(self.delta, (ds, db))]
        self.flips += len(rep["flips"])
        self.paired += npair
        self.rows += max(len(tA.out), len(tB.out))
        for k, v in rep["by_stage"].items():
            self.by[k] = self.by.get(k, 0) + v

    def summary(self):
        return {"what": self.what, "flips": self.flips, "paired": self.paired, "rows": self.rows, "by": self.by,
                "max_margin_score": self.margin[0], "max_margin_logit": self.margin[1],
                "max_margin_iou": self.margin[2], "max_paired_dscore": self.delta[0], "max_paired_box_rel": self.delta[1]}


def _np(t):
    return t.tensor().detach().cpu().numpy()


def _ratio(H, W, h, w):
    """transform.postprocess scale (orig / resized, float32) as [rw, rh, rw, rh]."""
    rw, rh = np.float32(W) / np.float32(w), np.float32(H) / np.float32(h)
    return np.asarray([rw, rh, rw, rh], np.float32)


# ------------------------------------------------------------------------------ SSDLite
def ssd_check(plan, sd, num_classes, reduced_tail, imgs, what="ssd", own_check=2, only=None, f64_arbiter=False):
    """only: the batch slots to check (default all).  f64_arbiter: when the raw heads part from the
    float32 oracle's by RAW_TOL or more, the float64 oracle decides: the engine must sit no further
    from it than twice the float32 oracle does (two float32 evaluations of one network, summed in
    different orders, part by more than RAW_TOL on some real-looking images: tools/ssd_raw_error.py)."""
    from oracle.ssdlite import SSDLiteOracle, postprocess
    B, _, H, W = imgs.shape
    idx = list(range(B)) if only is None else list(only)
    cls, reg = plan.cls_logits.tensor().cpu()[idx], plan.bbox_regression.tensor().cpu()[idx]
    st, bx = _np(plan.scores_t), _np(plan.boxes)
    cnt = _np(plan.out_count)
    ob, osc, ol = _np(plan.out_box), _np(plan.out_score), _np(plan.out_label)
    o = SSDLiteOracle(sd, num_classes, reduced_tail)
    cls_ref, reg_ref, _ = o.forward_raw([imgs[b] for b in idx])
    ec, er = (cls - cls_ref).abs().max().item(), (reg - reg_ref).abs().max().item()
    arb = None
    if f64_arbiter and not (ec < RAW_TOL and er < RAW_TOL):
        c64, r64, _ = SSDLiteOracle(sd, num_classes, reduced_tail, dtype=torch.float64).forward_raw(
            [imgs[b] for b in idx])
        e_eng = max((cls.double() - c64).abs().max().item(), (reg.double() - r64).abs().max().item())
        e_f32 = max((cls_ref.double() - c64).abs().max().item(), (reg_ref.double() - r64).abs().max().item())
        arb = {"engine_vs_f64": e_eng, "f32_vs_f64": e_f32}
        assert e_eng <= max(RAW_TOL, 2 * e_f32), (what, ec, er, arb)
    else:
        assert ec < RAW_TOL and er < RAW_TOL, (what, ec, er)
    A = st.shape[2]
    label_of = chains.ssd_label_of(A)
    scale = _ratio(H, W, 320, 320)
    acc = _Acc(what)
    for k, b in enumerate(idx):
        sB = chains.ssd_side(st[b], bx[b])
        tB = replay(sB, chains.SSD_STAGES)
        n = int(cnt[b])
        check_replay_reproduces(tB, sB, ob[b, :n], osc[b, :n], ol[b, :n], label_of, scale=scale)
        sA = chains.ssd_side(*chains.ssd_oracle_inputs(cls_ref[k], reg_ref[k], o.anchors))
        tA = replay(sA, chains.SSD_STAGES)
        if k < own_check:  # the replay is the oracle's own postprocess
            ref = postprocess(cls_ref[k:k + 1], reg_ref[k:k + 1], o.anchors, num_classes)[0]
            check_replay_reproduces(tA, sA, ref["boxes"].numpy(), ref["scores"].numpy(), ref["labels"].numpy(),
                                    label_of)
        acc.add(classify(sA, tA, sB, tB, chains.SSD_STAGES), tA, tB, sA, sB, f"image {b}")
    out = acc.summary()
    out.update(raw_dcls=ec, raw_dreg=er)
    if arb:
        out.update(arb)
    return out


# ------------------------------------------------------------------------------ Faster R-CNN
def frcnn_check(plan, sd, num_classes, imgs, what="frcnn", own_check=2):
    from oracle import frcnn as Fr
    from oracle import tv_ops
    from oracle.ssdlite import _SD
    B, _, H, W = imgs.shape
    NC = num_classes
    Ho, Wo, Hp, Wp = plan.resized
    pc = _np(plan.proposal_count)
    props = _np(plan.proposals)
    heads = [(o.tensor().cpu().reshape(B, -1), d.tensor().cpu().reshape(B, -1, 4)) for o, d in plan.rpn_heads]
    bsc, bdec = _np(plan.box_scores), _np(plan.box_decoded)
    cnt = _np(plan.out_count)
    ob, osc, ol = _np(plan.out_box), _np(plan.out_score), _np(plan.out_label)
    o = Fr.FasterRCNNOracle(sd, NC)
    osd = _SD(o.sd)
    with torch.no_grad():
        x, sizes = tv_ops.transform(list(imgs), Fr.MEAN, Fr.STD, Fr.MIN_SIZE, Fr.MAX_SIZE, divisible=Fr.DIVISIBLE)
        assert tuple(x.shape[-2:]) == (Hp, Wp) and sizes[0] == (Ho, Wo)
        feats = Fr.fpn(Fr.resnet_body(x, osd), osd)
        objs, dels, anchors = Fr.rpn_head(feats, osd, (Hp, Wp))
        k = min(own_check, B)
        ref_props = Fr.rpn_filter([t[:k] for t in objs], [t[:k] for t in dels], anchors, sizes[:k])
    eo = max((h[0] - r).abs().max().item() for h, r in zip(heads, objs))
    ed = max((h[1] - r).abs().max().item() for h, r in zip(heads, dels))
    assert eo < RAW_TOL and ed < RAW_TOL, (what, eo, ed)

    # stage 1: RPN proposals, each side from its own features
    rpn = _Acc(what + ".rpn")
    for b in range(B):
        sB = chains.rpn_side([h[0][b] for h in heads], [h[1][b] for h in heads], anchors, (Ho, Wo))
        tB = replay(sB, chains.RPN_STAGES)
        n = int(pc[b])
        assert len(tB.out) == n, (what, b, len(tB.out), n)  # decode + sigmoid recomputed on the host: 1-ulp tolerance
        # (two proposals whose recomputed scores tie within an ulp may come out swapped: matched in
        # the engine's order within a 16-place window, e2e_witness._engine_order)
        from tests.e2e_witness import _engine_order
        tB.out = _engine_order(sB, tB.out, props[b, :n])
        np.testing.assert_allclose(sB.box[tB.out], props[b, :n], rtol=2e-6, atol=1e-4)
        sA = chains.rpn_side([t[b] for t in objs], [t[b] for t in dels], anchors, sizes[b])
        tA = replay(sA, chains.RPN_STAGES)
        if b < k:
            np.testing.assert_array_equal(sA.box[tA.out], ref_props[b].numpy())
        rpn.add(classify(sA, tA, sB, tB, chains.RPN_STAGES), tA, tB, sA, sB, f"image {b}", key_stages=("topk",))

    # stage 2: box head + postprocess on the engine's proposals (the oracle's box head cross-fed)
    eprops = [torch.from_numpy(props[b, :int(pc[b])].copy()) for b in range(B)]
    with torch.no_grad():
        logits, deltas = o.box_stage(feats, eprops, sizes)
    off = np.concatenate([[0], np.cumsum(pc)]).astype(np.int64)
    box = _Acc(what + ".box")
    scale = _ratio(H, W, Ho, Wo)
    for b in range(B):
        lo, hi, n, kk = int(off[b]), int(off[b + 1]), int(pc[b]), int(cnt[b])
        sB = chains.box_side_from_values(bsc[b, :n], bdec[b, :n])
        tB = replay(sB, chains.BOX_STAGES)
        check_replay_reproduces(tB, sB, ob[b, :kk], osc[b, :kk], ol[b, :kk], chains.box_label_of(NC), scale=scale)
        sA = chains.box_side(logits[lo:hi], deltas[lo:hi], eprops[b], sizes[b])
        tA = replay(sA, chains.BOX_STAGES)
        if b < own_check:
            ref = Fr.box_postprocess(logits[lo:hi], deltas[lo:hi], [eprops[b]], [sizes[b]])[0]
            check_replay_reproduces(tA, sA, ref["boxes"].numpy(), ref["scores"].numpy(), ref["labels"].numpy(),
                                    chains.box_label_of(NC))
        box.add(classify(sA, tA, sB, tB, chains.BOX_STAGES), tA, tB, sA, sB, f"image {b}")
    return {"raw_dobj": eo, "raw_ddelta": ed, "rpn": rpn.summary(), "box": box.summary()}


# ------------------------------------------------------------------------------ RetinaNet
def retina_check(plan, sd, num_classes, imgs, what="retinanet", own_check=1):
    from oracle import retinanet as R
    B, _, H, W = imgs.shape
    Ho, Wo, _, _ = plan.resized
    cls, reg = plan.cls_logits.tensor().cpu(), plan.bbox_regression.tensor().cpu()
    na = list(plan.level_anchors)
    cnt = _np(plan.out_count)
    ob, osc, ol = _np(plan.out_box), _np(plan.out_score), _np(plan.out_label)
    o = R.RetinaNetOracle(sd, num_classes)
    cls_ref, reg_ref, anchors, sizes, _ = o.forward_raw(list(imgs))
    ec = (cls - torch.cat(cls_ref, 1)).abs().max().item()
    er = (reg - torch.cat(reg_ref, 1)).abs().max().item()
    assert ec < RAW_TOL and er < RAW_TOL, (what, ec, er)
    cls_l, reg_l = torch.split(cls, na, 1), torch.split(reg, na, 1)
    acc = _Acc(what)
    scale = _ratio(H, W, Ho, Wo)
    for b in range(B):
        sA, sB, label_of = chains.retina_sides([c[b] for c in cls_ref], [r[b] for r in reg_ref],
                                               [c[b] for c in cls_l], [r[b] for r in reg_l], anchors, sizes[b])
        tA, tB = replay(sA, chains.RETINA_STAGES), replay(sB, chains.RETINA_STAGES)
        n = int(cnt[b])
        # sigmoid / decode recomputed on the host from the engine's logits: 1-ulp tolerance
        check_replay_reproduces(tB, sB, ob[b, :n], osc[b, :n], ol[b, :n], label_of, scale=scale, rtol=2e-6)
        if b < own_check:
            ref = R.postprocess([c[b:b + 1] for c in cls_ref], [r[b:b + 1] for r in reg_ref], anchors, sizes[b:b + 1])[0]
            check_replay_reproduces(tA, sA, ref["boxes"].numpy(), ref["scores"].numpy(), ref["labels"].numpy(),
                                    label_of)
        acc.add(classify(sA, tA, sB, tB, chains.RETINA_STAGES), tA, tB, sA, sB, f"image {b}")
    out = acc.summary()
    out.update(raw_dcls=ec, raw_dreg=er)
    return out
