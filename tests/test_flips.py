"""CPU tests of the decision-replay parity classifier (tests/flips.py, tests/chains.py).

* the replay of the oracle's own pre-decision values reproduces the oracle's detections exactly
  (SSDLite, and the FRCNN box stage on seeded inputs), so candidate identities are trustworthy;
* each flip kind is attributed to the right stage with the right witness on hand-made cases;
* a run perturbed by rounding-sized noise leaves only boundary flips (margins bounded by the noise).
"""
import numpy as np
import pytest
import torch

from tests import chains
from tests.flips import Side, classify, compare, max_margin, replay, check_replay_reproduces


def _side(scores, boxes, groups=None):
    scores = np.asarray(scores, np.float32)
    n = len(scores)
    g = np.zeros(n, np.int64) if groups is None else np.asarray(groups)
    ids = np.arange(n)
    return Side(scores, np.asarray(boxes, np.float32), {"g": g}, q={"score": scores}, ties=(ids,),
                tkties={"id": ids})


STAGES = [("filter", "score", 0.5, ">"), ("topk", 2, "g", "score", "id"), ("nms", 0.5, "g"), ("cut", 2)]
FAR = [[0, 0, 10, 10], [100, 100, 110, 110], [200, 200, 210, 210], [300, 300, 310, 310]]


def _kinds(rep):
    return sorted((r["id"], r["kind"], r["reason"]) for r in rep["flips"])


def test_filter_straddle():
    a = _side([0.9, 0.5000001, 0.1, 0.1], FAR)
    b = _side([0.9, 0.4999999, 0.1, 0.1], FAR)
    rep = compare(a, b, STAGES)
    assert _kinds(rep) == [(1, "filter", "straddle")] and not rep["unexplained"]
    assert max_margin(rep) < 1e-6


def test_topk_inversion_and_cut():
    a = _side([0.9, 0.80001, 0.8, 0.6], FAR)
    b = _side([0.9, 0.79999, 0.8, 0.6], FAR)
    rep = compare(a, b, STAGES)
    assert _kinds(rep) == [(1, "topk", "inversion"), (2, "topk", "inversion")]
    assert max_margin(rep) < 2e-5


def test_nms_iou_straddle_and_cascade():
    # box 1 overlaps box 0 at IoU just around 0.5; box 2 overlaps box 1 heavily (suppressed by 1 when 1 is kept)
    b0 = [0, 0, 10, 10]
    a1 = [0, 0, 10, 20.0001]   # IoU(0,1) = 100 / 200.001 < 0.5 on A: kept
    b1 = [0, 0, 10, 19.9999]   # > 0.5 on B: suppressed
    box2 = [0, 10, 10, 20]     # IoU(1,2) ~ 0.5 vs box 1 ... make it clearly > 0.5
    box2 = [0, 1, 10, 21]
    sa = Side(np.float32([0.9, 0.8, 0.7]), np.float32([b0, a1, box2]), {"g": np.zeros(3, int)},
              q={"score": np.float32([0.9, 0.8, 0.7])}, ties=(np.arange(3),), tkties={"id": np.arange(3)})
    sb = Side(np.float32([0.9, 0.8, 0.7]), np.float32([b0, b1, box2]), {"g": np.zeros(3, int)},
              q={"score": np.float32([0.9, 0.8, 0.7])}, ties=(np.arange(3),), tkties={"id": np.arange(3)})
    st = [("nms", 0.5, "g"), ("cut", 10)]
    rep = compare(sa, sb, st)
    assert _kinds(rep) == [(1, "nms", "iou_straddle"), (2, "nms", "cascade")], _kinds(rep)
    assert max_margin(rep) < 1e-5


def test_nms_order_inversion():
    box = [[0, 0, 10, 10], [0, 0, 10, 10.5]]  # heavy overlap: whichever ranks first survives
    sa = _side([0.70001, 0.7], box)
    sb = _side([0.69999, 0.7], box)
    rep = compare(sa, sb, [("nms", 0.5, "g"), ("cut", 10)])
    assert _kinds(rep) == [(0, "nms", "inversion"), (1, "nms", "inversion")]


def test_replay_reproduces_ssd_oracle_and_perturbation_flips_are_boundary():
    from edgeml_amd import synthetic
    from oracle.ssdlite import SSDLiteOracle
    sd = synthetic.synthetic_state_dict("ssd", 91, True, seed=0)
    o = SSDLiteOracle(sd, 91, True)
    imgs = synthetic.make_batch(1, 480, 640, seed=7)
    ref = o(list(imgs))[0]
    cls, reg, _ = o.forward_raw(list(imgs))
    st, bx = chains.ssd_oracle_inputs(cls[0], reg[0], o.anchors)
    sa = chains.ssd_side(st, bx)
    ta = replay(sa, chains.SSD_STAGES)
    A = st.shape[1]
    check_replay_reproduces(ta, sa, ref["boxes"].numpy(), ref["scores"].numpy(), ref["labels"].numpy(),
                            chains.ssd_label_of(A), scale=[640 / 320, 480 / 320] * 2)
    # rounding-sized noise on the logits (the engine's fp32 reorder noise is ~1e-5 relative)
    g = torch.Generator().manual_seed(1)
    noisy = cls[0] * (1 + 2e-6 * torch.randn(cls[0].shape, generator=g))
    st2, bx2 = chains.ssd_oracle_inputs(noisy, reg[0], o.anchors)
    sb = chains.ssd_side(st2, bx2)
    rep = compare(sa, sb, chains.SSD_STAGES)
    print({k: rep[k] for k in ("n_oracle", "n_engine", "paired", "by_stage", "max_score_diff")}, max_margin(rep))
    assert not rep["unexplained"]
    assert rep["paired"] >= 295 and rep["max_score_diff"] < 1e-5
    assert max_margin(rep) <= rep["max_score_diff"] * 2 + 1e-9


def test_replay_reproduces_frcnn_box_postprocess():
    from oracle import frcnn
    rs = np.random.RandomState(3)
    R, NC = 300, 91
    c = rs.uniform(0, 700, (R, 2))
    wh = rs.uniform(2, 200, (R, 2))
    props = torch.from_numpy(np.concatenate([c - wh / 2, c + wh / 2], 1).clip(0, 800).astype(np.float32))
    logits = torch.from_numpy(rs.normal(0, 2.5, (R, NC)).astype(np.float32))
    deltas = torch.from_numpy(rs.normal(0, 0.3, (R, 4 * NC)).astype(np.float32))
    ref = frcnn.box_postprocess(logits, deltas, [props], [(800, 800)])[0]
    s = chains.box_side(logits, deltas, props, (800, 800))
    t = replay(s, chains.BOX_STAGES)
    check_replay_reproduces(t, s, ref["boxes"].numpy(), ref["scores"].numpy(), ref["labels"].numpy(),
                            chains.box_label_of(NC))
    assert len(t.out) == 100
