"""End-to-end FRCNN witness attribution (test infrastructure).

tests/parity_models.frcnn_check checks Faster R-CNN stage by stage: the box stage of the oracle is fed
the ENGINE's proposals, so a final-row difference that comes from the two sides' own proposals never
reaches an assertion.  Here each side runs end to end on its own values, as bench.py's ORIE leg does:

  RPN        each side's proposal filter over its own head outputs (flips.replay of RPN_STAGES); every
             candidate whose fate differs must carry a boundary witness (tests/flips.classify).
  box stage  candidates are (anchor, class) over the UNION of both sides' proposals, identified by the
             anchor that produced the proposal (level offset + anchor index, the RPN candidate id), so
             a proposal the other side's RPN did not emit is a candidate that side does not have
             ("proposal_flip", explained by the RPN flip of that anchor); every other divergence needs
             its own box-stage witness (threshold straddle, order inversion, IoU straddle, cascade).
  rows       candidates output by both sides (identity-paired) must agree within north_star's 1e-3 in
             score and box, unless the RoI level of their proposals differs between the sides
             (MultiScaleRoIAlign's LevelMapper floor, a discontinuity: "level_straddle").  The rows as
             bench.py pairs them (tools/rowpair.py: class + IoU >= 0.99 on the detect.py files) are
             then mapped back to candidate ids: every such pair with |dconf| > 1e-3 and every row
             rowpair leaves unpaired must be an identity pair within tolerance or a witnessed flip.

Side values for one image (dict):
  objs, dels   per-level RPN objectness logits [A_l] and deltas [A_l, 4] (float32)
  anchors      per-level anchors (the oracle's generator; the engine's plan constants are pinned to it)
  size         (h, w) of the resized image
  props        [R, 4] the side's proposals in its own order (checked against the replay)
  scores       [R, NC] box-head class probabilities, boxes [R, NC, 4] decoded + clipped (resized space)
  out          (boxes [K, 4] in resized space, scores [K], labels [K]) the side's own output rows
"""
import numpy as np
import torch

from tests import chains
from tests.flips import Side, box_rel_err, check_replay_reproduces, classify, max_margin, replay

# Witness margins (the reference side's distance of the deciding quantity from its boundary).  End to end
# the two sides' RPN boxes differ by the RPN head's float32 error through BoxCoder.decode (~1e-4 of a
# box's size), so IoUs and clipped box sizes carry that noise; box-stage scores are compared end to end
# (each side on its own proposals), so their threshold straddles are bounded by north_star's 1e-3.
EPS_SCORE = 1e-5    # RPN sigmoid scores (same-stage arithmetic)
EPS_LOGIT = 1e-4    # RPN top-k keys
EPS_IOU = 1e-4      # NMS IoU straddles (RPN and box stage)
EPS_SIZE = 1e-4     # remove_small straddles: |min side - threshold| / max(1, |coords|, w, h) of the box
TOL = 1e-3          # north_star: paired rows within 1e-3; box-stage score straddles within it


def box_values(logits, deltas, proposals, image_size):
    """The oracle's softmax / decode / clip of the box stage (oracle/frcnn.py box_postprocess) as
    arrays: scores [R, NC], boxes [R, NC, 4]."""
    from oracle import tv_ops
    scores = torch.softmax(torch.as_tensor(logits), -1)
    boxes = tv_ops.clip_boxes(tv_ops.decode_boxes(torch.as_tensor(deltas), torch.as_tensor(proposals),
                                                  (10.0, 10.0, 5.0, 5.0)), image_size)
    return scores.numpy().astype(np.float32), boxes.numpy().astype(np.float32)


def _union_side(U, ids, scores, boxes, NC):
    """A flips.Side over (anchor in U, class 1..NC-1); candidates whose anchor is not among this
    side's proposals get score -1 (dropped by the first filter) and are reported absent."""
    nu, C = len(U), NC - 1
    pos = np.full(nu, -1, np.int64)
    pos[np.searchsorted(U, ids)] = np.arange(len(ids))
    n = nu * C
    u = np.repeat(np.arange(nu), C)
    c = np.tile(np.arange(1, NC), nu)
    p = pos[u]
    ok = p >= 0
    score = np.full(n, -1.0, np.float32)
    box = np.zeros((n, 4), np.float32)
    score[ok] = scores[p[ok], c[ok]]
    box[ok] = boxes[p[ok], c[ok]]
    # the side's own flattened candidate order (proposal-major, class-minor) breaks score ties, as in
    # box_postprocess / the engine's box NMS; absent candidates sort last (never reach a tie anyway)
    tie = np.where(ok, p * C + (c - 1), n + np.arange(n))
    side = Side(score, box, {"cls": c}, q={"score": score, "minsize": chains._minsize(box)}, ties=(tie,))
    return side, ~ok, pos


def _engine_order(side, ids, props, window=16):
    """The anchor ids of the engine's proposals in the ENGINE's order.  The host replay recomputes the
    sigmoid of the engine's logits (the device's expf is not the host's), so two proposals whose
    scores tie within an ulp can come out of the replay in swapped order; each engine proposal is
    matched to the replay output within `window` places holding its box (decode is recomputed too:
    1-ulp tolerance).  The kept set itself must be the replay's."""
    box = side.box[ids]
    close = lambda j, q: np.allclose(box[q], props[j], rtol=2e-6, atol=1e-4)  # noqa: E731
    out, used = np.empty_like(ids), np.zeros(len(ids), bool)
    for j in range(len(ids)):
        if not used[j] and close(j, j):
            used[j] = True
            out[j] = ids[j]
            continue
        cand = [q for q in range(max(0, j - window), min(len(ids), j + window + 1)) if not used[q] and close(j, q)]
        assert cand, ("engine proposal not in the host replay's output", j, props[j])
        q = min(cand, key=lambda q: abs(q - j))
        used[q] = True
        out[j] = ids[q]
    return out


PROPOSAL_TOL = 2e-3  # a proposal shift inside the RPN's float32 band: |dcoord| / box size (RAW_TOL on deltas)


def _proposal_shift(A, B, ja, jb, c, tol):
    """Witness for an identity-paired row whose score or box differs by more than tol: the two sides'
    proposals for its anchor differ (the RPN head's float32 error through BoxCoder.decode), and the
    box head is steep in the proposal's coordinates.  The difference splits in two:
      s_B(P_B) - s_A(P_A) = [s_B(P_B) - s_A(P_B)] + [s_A(P_B) - s_A(P_A)]
    the box stage's own arithmetic on the SAME proposal (the reference's box head fed the engine's
    proposal: must agree within tol, as the stage-by-stage parity of tests/parity_models.py asserts)
    and the reference's response to the proposal shift.  The witness holds when the first term is
    within tol and the shift itself is inside PROPOSAL_TOL.  None when it does not hold (or side A
    cannot evaluate its box stage at another proposal)."""
    if "box_at" not in A:
        return None
    pa = np.asarray(A["props"][ja], np.float32)
    pb = np.asarray(B["props"][jb], np.float32)
    shift = float(box_rel_err(pa[None], pb[None])[0])
    sc, bx = A["box_at"](pb[None])
    s_ab, b_ab = float(sc[0, c]), bx[0, c]
    s_bb, b_bb = float(B["scores"][jb, c]), np.asarray(B["boxes"][jb, c], np.float32)
    arith = abs(s_bb - s_ab)
    arith_box = float(box_rel_err(b_ab[None], b_bb[None])[0])
    if shift > PROPOSAL_TOL or arith > tol or arith_box > tol:
        return None
    return {"proposal_shift": shift, "box_stage_dscore": arith, "box_stage_dbox": arith_box,
            "response": abs(s_ab - float(A["scores"][ja, c]))}


def _beyond_band(r, sA, tol):
    """A base-explained witness whose reference-side margin lies outside its noise band."""
    m = r.get("margin")
    if m is None:
        return False
    if r["kind"] == "filter" and r.get("quantity") == "minsize":
        b = sA.box[r["id"]].astype(np.float64)
        return m / max(1.0, float(np.abs(b).max()), float(b[2] - b[0]), float(b[3] - b[1])) > EPS_SIZE
    if r["reason"] == "iou_straddle":
        return m > EPS_IOU
    return m > tol


def _filter_margins(rep, sA):
    """(largest score-filter margin, largest remove_small margin relative to the box's scale) over the
    base-explained filter straddles of a classify report."""
    ms, mz = 0.0, 0.0
    for r in rep["flips"]:
        if r["kind"] != "filter" or r["reason"] != "straddle":
            continue
        if r.get("quantity") == "minsize":
            b = sA.box[r["id"]].astype(np.float64)
            scale = max(1.0, float(np.abs(b).max()), float(b[2] - b[0]), float(b[3] - b[1]))
            mz = max(mz, r["margin"] / scale)
        else:
            ms = max(ms, r["margin"])
    return ms, mz


def _levels(props):
    from oracle import tv_ops
    return tv_ops.level_mapper(torch.as_tensor(np.asarray(props, np.float32).reshape(-1, 4))).numpy()


def _rows(side, q, NC, scale, orig_hw):
    """detect.py rows of a side's output (fmt.format_detections of the replayed output, which
    reproduces the side's own rows exactly) and, per row, the candidate id it came from (rows of the
    11 dropped COCO ids are removed by the formatter)."""
    from edgeml_amd import fmt
    from edgeml_amd.labelmap import coco_to_yolov5
    labels = chains.box_label_of(NC)(q.out)
    H, W = orig_hw
    rows = fmt.format_detections(side.box[q.out] * np.asarray(scale, np.float32), side.score[q.out], labels, H, W)
    kept = np.array([coco_to_yolov5[int(l)] != -1 for l in labels], bool)
    return rows, q.out[kept]


def check_image(A, B, NC, scale, orig_hw, own_check_A=True, tol=TOL):
    """Attribute every end-to-end difference of one image between side A (the reference: the CPU
    oracle, float32 or float64) and side B (the engine).  Returns (report dict, list of failures)."""
    from tools import rowpair
    fails = []
    # ---------------------------------------------------------------- RPN, each side on its own values
    sA = chains.rpn_side(A["objs"], A["dels"], A["anchors"], A["size"])
    sB = chains.rpn_side(B["objs"], B["dels"], B["anchors"], B["size"])
    tA, tB = replay(sA, chains.RPN_STAGES), replay(sB, chains.RPN_STAGES)
    np.testing.assert_array_equal(sA.box[tA.out], np.asarray(A["props"], np.float32))
    assert len(tB.out) == len(B["props"]), ("engine proposals", len(tB.out), len(B["props"]))
    tB.out = _engine_order(sB, tB.out, np.asarray(B["props"], np.float32))
    rrep = classify(sA, tA, sB, tB, chains.RPN_STAGES)
    if rrep["unexplained"]:
        fails.append(("rpn unexplained", rrep["unexplained"][:5]))
    m_s, m_z = _filter_margins(rrep, sA)
    m_s = max(m_s, max_margin(rrep, kinds=("inversion",), stages=("nms", "cut")))
    m_k = max_margin(rrep, kinds=("straddle", "inversion"), stages=("topk",))
    m_i = max_margin(rrep, kinds=("iou_straddle",))
    if m_s > EPS_SCORE or m_k > EPS_LOGIT or m_i > EPS_IOU or m_z > EPS_SIZE:
        fails.append(("rpn margins", m_s, m_k, m_i, m_z))
    rpn_div = {int(r["id"]) for r in rrep["flips"] if r["reason"] is not None}

    # ---------------------------------------------------------------- box stage over the union of proposals
    U = np.union1d(tA.out, tB.out)
    bA, absA, posA = _union_side(U, tA.out, A["scores"], A["boxes"], NC)
    bB, absB, posB = _union_side(U, tB.out, B["scores"], B["boxes"], NC)
    qA, qB = replay(bA, chains.BOX_STAGES), replay(bB, chains.BOX_STAGES)
    label_of = chains.box_label_of(NC)
    for side, q, X, own in ((bA, qA, A, own_check_A), (bB, qB, B, True)):
        if own and "out_scaled" in X:  # the engine's rows, rescaled to the original size on the device
            check_replay_reproduces(q, side, *X["out_scaled"], label_of, scale=scale)
        elif own:
            check_replay_reproduces(q, side, *X["out"], label_of)
    brep = classify(bA, qA, bB, qB, chains.BOX_STAGES, absent=(absA, absB))
    if brep["unexplained"]:
        fails.append(("box unexplained", brep["unexplained"][:5]))
    C = NC - 1
    for r in brep["flips"]:
        if r["reason"] == "proposal_flip" and int(U[r["id"] // C]) not in rpn_div:
            fails.append(("proposal flip without an RPN witness", r))
    # a box-stage witness whose reference margin lies outside its band is re-examined at the engine's
    # proposal: the reference's box stage fed the engine's proposal must land within tol of the engine
    # for every class that flipped on that anchor (the divergence is the proposal shift, see
    # _proposal_shift); otherwise the flip fails
    shifted = {}
    for r in brep["flips"]:
        if r["reason"] in (None, "proposal_flip", "cascade") or not _beyond_band(r, bA, tol):
            continue
        x = int(r["id"])
        w = _proposal_shift(A, B, posA[x // C], posB[x // C], x % C + 1, tol)
        if w is None:
            fails.append(("box flip beyond its band without a witness", {k: r.get(k) for k in
                                                                           ("id", "kind", "reason", "margin")}))
        else:
            r["reason"] = "proposal_shift"
            shifted[x] = w
    b_s, b_z = _filter_margins(brep, bA)
    b_s = max(b_s, max_margin(brep, kinds=("inversion",)))
    b_i = max_margin(brep, kinds=("iou_straddle",))
    box_div = {int(r["id"]) for r in brep["flips"] if r["reason"] is not None}

    # ---------------------------------------------------------------- identity-paired rows
    both = np.intersect1d(qA.out, qB.out)
    ds = np.abs(bA.score[both] - bB.score[both]) if len(both) else np.zeros(0)
    db = box_rel_err(bA.box[both], bB.box[both]) if len(both) else np.zeros(0)
    anc = U[both // C]
    lvA = _levels(np.asarray(A["props"])[posA[both // C]]) if len(both) else np.zeros(0, np.int64)
    lvB = _levels(np.asarray(B["props"])[posB[both // C]]) if len(both) else np.zeros(0, np.int64)
    level_straddle = lvA != lvB
    big = (ds > tol) | (db > tol)
    shift_ids, shifts = set(), []
    for k in np.nonzero(big & ~level_straddle)[0]:
        x = int(both[k])
        rec = {"id": x, "anchor": int(anc[k]), "dscore": float(ds[k]), "dbox": float(db[k]),
               "score_ref": float(bA.score[x])}
        w = _proposal_shift(A, B, posA[x // C], posB[x // C], x % C + 1, tol)
        if w is None:
            fails.append(("identity pair beyond 1e-3 without a witness", rec))
        else:
            rec.update(w)
            shifts.append(rec)
            shift_ids.add(x)
    ok_pair = {int(x) for x, b in zip(both, big) if not b}

    # ---------------------------------------------------------------- the rows as bench.py pairs them
    rA, idA = _rows(bA, qA, NC, scale, orig_hw)
    rB, idB = _rows(bB, qB, NC, scale, orig_hw)
    pairs, ua, ub = rowpair.pair_rows(rA, rB)
    rp = {"pairs": len(pairs), "gt_1e-3": 0, "gt_1e-3_identity": 0, "gt_1e-3_flip": 0, "gt_1e-3_level": 0,
          "gt_1e-3_proposal_shift": 0,
          "unpaired": len(ua) + len(ub), "unpaired_flip": 0, "max_dconf": 0.0}
    lvl_ids = {int(x) for x, s in zip(both, level_straddle) if s}
    for i, j in pairs:
        d = abs(rA[i, 5] - rB[j, 5])
        rp["max_dconf"] = max(rp["max_dconf"], float(d))
        if d <= tol:
            continue
        rp["gt_1e-3"] += 1
        a, b = int(idA[i]), int(idB[j])
        if a == b and a in lvl_ids:
            rp["gt_1e-3_level"] += 1
        elif a == b and a in shift_ids:
            rp["gt_1e-3_proposal_shift"] += 1
        elif a == b and a in ok_pair:
            rp["gt_1e-3_identity"] += 1   # float32 -> float64 of the same row: cannot exceed tol (guard)
        elif a != b and a in box_div and b in box_div:
            rp["gt_1e-3_flip"] += 1
        else:
            fails.append(("rowpair pair beyond 1e-3 not attributed", {"ref_id": a, "eng_id": b, "dconf": float(d)}))
    un_ids = [int(idA[k]) for k in range(len(rA)) if not any(k == i for i, _ in pairs)] + \
             [int(idB[k]) for k in range(len(rB)) if not any(k == j for _, j in pairs)]
    rp["unpaired_identity"] = []
    for x in un_ids:
        if x in box_div:
            rp["unpaired_flip"] += 1
        elif x in ok_pair:
            # the same detection on both sides within tolerance that the IoU >= 0.99 pairing misses: a
            # thin box, where a coordinate difference well inside 1e-3 of its size moves the IoU under 0.99
            a, b = bA.box[x].astype(np.float64), bB.box[x].astype(np.float64)
            iw = max(0.0, min(a[2], b[2]) - max(a[0], b[0]))
            ih = max(0.0, min(a[3], b[3]) - max(a[1], b[1]))
            ar = lambda q: (q[2] - q[0]) * (q[3] - q[1])  # noqa: E731
            iou = iw * ih / (ar(a) + ar(b) - iw * ih) if ar(a) + ar(b) > 0 else 0.0
            rp["unpaired_identity"].append({"id": x, "score": float(bA.score[x]), "iou": round(float(iou), 5),
                                            "w": round(float(a[2] - a[0]), 3), "h": round(float(a[3] - a[1]), 3),
                                            "dbox": float(box_rel_err(a[None], b[None])[0])})
        elif x not in lvl_ids and x not in shift_ids:
            fails.append(("rowpair-unpaired row without a witness", x))
    rep = {"rpn_flips": len(rrep["flips"]), "rpn_by": rrep["by_stage"], "box_flips": len(brep["flips"]),
           "box_by": brep["by_stage"], "proposals_only_ref": int(len(np.setdiff1d(tA.out, tB.out))),
           "proposals_only_eng": int(len(np.setdiff1d(tB.out, tA.out))), "identity_paired": int(len(both)),
           "max_identity_dscore": float(ds.max()) if len(ds) else 0.0,
           "max_identity_dbox": float(db.max()) if len(db) else 0.0,
           "level_straddles": int(level_straddle.sum()), "proposal_shifts": len(shifts),
           "box_flips_proposal_shift": len(shifted),
           "max_shift_response": max([r["response"] for r in shifts], default=0.0),
           "max_shift_box_arith": max([r["box_stage_dscore"] for r in shifts], default=0.0),
           "max_margin": {"rpn_score": m_s, "rpn_logit": m_k, "rpn_iou": m_i, "rpn_size": m_z, "box_score": b_s,
                          "box_iou": b_i, "box_size": b_z},
           "rowpair": rp}
    return rep, fails


def merge(reports):
    """Sum / max of per-image reports (printed by the tests and tools/e2e_witness.py)."""
    out = {}
    for r in reports:
        for k, v in r.items():
            if isinstance(v, dict):
                d = out.setdefault(k, {})
                for kk, vv in v.items():
                    if isinstance(vv, float):
                        d[kk] = max(d.get(kk, 0.0), vv)
                    elif isinstance(vv, list):
                        d[kk] = d.get(kk, []) + vv
                    else:
                        d[kk] = d.get(kk, 0) + vv
            elif isinstance(v, float):
                out[k] = max(out.get(k, 0.0), v)
            else:
                out[k] = out.get(k, 0) + v
    return out


# ------------------------------------------------------------------------------ the two sides' values
def oracle_side(o, img):
    """One image through the CPU oracle (float32 or float64 FasterRCNNOracle), end to end."""
    from oracle import frcnn as Fr
    logits, deltas, props, sizes, feats = o.forward_raw([img])
    objs, dels, anchors = o.last_rpn
    scores, boxes = box_values(logits, deltas, props[0], sizes[0])
    ref = Fr.box_postprocess(logits, deltas, props, sizes)[0]

    def box_at(p):  # the reference's box stage at other proposals (the proposal-shift witness)
        pt = torch.as_tensor(np.asarray(p, np.float32).reshape(-1, 4))
        lg, dl = o.box_stage(feats, [pt], sizes)
        return box_values(lg, dl, pt, sizes[0])
    return {"objs": [t[0] for t in objs], "dels": [t[0] for t in dels], "anchors": anchors, "size": sizes[0],
            "props": props[0].numpy(), "scores": scores, "boxes": boxes, "box_at": box_at,
            "out": (ref["boxes"].numpy(), ref["scores"].numpy(), ref["labels"].numpy())}


def engine_side(plan, b, anchors):
    """Image b of a plan the engine has just run: its own RPN heads, proposals and box-stage values
    read back from the device (the named buffers of edgedet_model_buffers)."""
    B = plan.B
    Ho, Wo, _, _ = plan.resized
    np_ = lambda t: t.tensor().detach().cpu().numpy()  # noqa: E731
    n = int(np_(plan.proposal_count)[b])
    heads = [(o.tensor().cpu().reshape(B, -1)[b], d.tensor().cpu().reshape(B, -1, 4)[b]) for o, d in plan.rpn_heads]
    k = int(np_(plan.out_count)[b])
    return {"objs": [h[0] for h in heads], "dels": [h[1] for h in heads], "anchors": anchors, "size": (Ho, Wo),
            "props": np_(plan.proposals)[b, :n], "scores": np_(plan.box_scores)[b, :n],
            "boxes": np_(plan.box_decoded)[b, :n],
            # the engine's rows are rescaled to the original size; the replay compares in resized space
            "out_scaled": (np_(plan.out_box)[b, :k], np_(plan.out_score)[b, :k], np_(plan.out_label)[b, :k])}
