"""Decision-replay parity classifier (test infrastructure).

The post-processing tails of the three detectors are chains of discrete decisions over a fixed set
of candidates:
  SSDLite  (anchor, class):  score > 0.001 -> per-class top-300 -> per-class NMS 0.55 -> [:300]
  RPN      (level, anchor):  per-level top-1000 logits -> min size 1e-3 -> per-level NMS 0.7 -> [:1000]
  FRCNN    (proposal, class): score > 0.05 -> min size 1e-2 -> per-class NMS 0.5 -> [:100]
  RetinaNet (level, anchor, class): score > 0.05 -> per-level top-1000 -> per-class NMS 0.5 -> [:300]
Two runs of the same fp32 network with different summation orders (the CPU oracle = side A, the
HIP engine = side B) feed these chains values that differ by rounding noise, so a candidate whose
decisive quantity sits within that noise of a boundary can take a different fate on the two sides
(SURVEY.md §7 hard part 1).

``replay`` runs a chain over one side's candidate values and records, per candidate, the stage that
dropped it (its fate), the candidate that suppressed it in NMS, and the final output order.  The
replay of the engine's own inputs must reproduce the engine's output rows exactly, and the replay
of the oracle's inputs the oracle's rows, so candidate identities (anchor, class, proposal ...)
are known on both sides and rows are paired by identity, not by value.

``classify`` then attributes every candidate whose fate differs to the first stage where the sides
part, and requires a concrete witness there:
  filter  the quantity straddles the threshold (q_A and q_B on opposite sides);
  topk    a candidate y kept by the dropping side's top-k either ranks behind x on the other side
          (an order inversion of two near-equal keys) or did not reach the top-k there (cascade);
  nms     x's suppressor y on the dropping side either was not kept on the other side (cascade),
          or ranks behind x there (order inversion), or IoU(x, y) straddles the NMS threshold;
  cut     a candidate y ahead of x in the dropping side's output either did not survive NMS on the
          other side (cascade) or ranks behind x there (order inversion).
A cascade counts only if y's own divergence is explained (fixed point).  Every witness carries a
margin: the reference side's distance of the decisive quantity from its boundary (|q_A - t|,
|IoU_A - t|, |key_A(x) - key_A(y)|).  Tests assert zero unexplained divergences and bound the
margins by explicit tolerances.
"""
import numpy as np

# ------------------------------------------------------------------------------ one side
class Side:
    """Candidate values of one side.

    score   float32 [n]: the NMS / final order key (descending)
    box     float32 [n, 4] xyxy (the NMS boxes)
    groups  {name: int [n]}: grouping keys of top-k / NMS stages
    q       {name: float [n]}: filter quantities
    keys    {name: float32 [n]}: top-k keys (descending)
    ties    tuple of int [n]: tie-breakers of the global order after -score (lexicographic)
    tkties  {name: int [n]}: tie-breaker of a top-k stage after -key
    """

    def __init__(self, score, box, groups, q=None, keys=None, ties=(), tkties=None):
        self.score = np.ascontiguousarray(score, np.float32)
        self.box = np.ascontiguousarray(box, np.float32).reshape(-1, 4)
        self.groups = {k: np.asarray(v) for k, v in groups.items()}
        self.q = {k: np.asarray(v) for k, v in (q or {}).items()}
        self.keys = {k: np.asarray(v, np.float32) for k, v in (keys or {}).items()}
        self.keys.setdefault("score", self.score)
        self.ties = tuple(np.asarray(t) for t in ties)
        self.tkties = {k: np.asarray(v) for k, v in (tkties or {}).items()}
        n = self.score.shape[0]
        order = np.lexsort(tuple(reversed(self.ties)) + (-self.score,)) if n else np.zeros(0, np.int64)
        self.pos = np.empty(n, np.int64)
        self.pos[order] = np.arange(n)

    def __len__(self):
        return self.score.shape[0]


def iou_rows(box, i, js):
    """IoU of box i with boxes js in torchvision's CPU nms op order (float32; nms_kernel.cpp)."""
    x1, y1, x2, y2 = box[:, 0], box[:, 1], box[:, 2], box[:, 3]
    area = (x2 - x1) * (y2 - y1)
    xx1 = np.maximum(x1[i], x1[js])
    yy1 = np.maximum(y1[i], y1[js])
    xx2 = np.minimum(x2[i], x2[js])
    yy2 = np.minimum(y2[i], y2[js])
    w = np.maximum(np.float32(0), xx2 - xx1)
    h = np.maximum(np.float32(0), yy2 - yy1)
    inter = w * h
    return inter / ((area[i] + area[js]) - inter)


def _greedy_nms(box, ids, thr, block=2048):
    """Greedy NMS over ids (already in processing order): per position, the position of the first
    kept candidate that suppresses it, or -1 when kept.  IoUs in torchvision's op order; the IoU of
    a pair is symmetric bit for bit ((a + b) == (b + a), max / min commute), so rows of a block
    matrix equal the reference's per-kept-box rows."""
    m = len(ids)
    sup = np.full(m, -1, np.int64)
    b = box[ids]
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    area = (x2 - x1) * (y2 - y1)
    supp = np.zeros(m, bool)
    for r0 in range(0, m, block):
        r1 = min(m, r0 + block)
        xx1 = np.maximum(x1[r0:r1, None], x1[None, :])
        yy1 = np.maximum(y1[r0:r1, None], y1[None, :])
        xx2 = np.minimum(x2[r0:r1, None], x2[None, :])
        yy2 = np.minimum(y2[r0:r1, None], y2[None, :])
        inter = np.maximum(np.float32(0), xx2 - xx1) * np.maximum(np.float32(0), yy2 - yy1)
        hit = (inter / ((area[r0:r1, None] + area[None, :]) - inter)).astype(np.float64) > thr
        a = r0
        while a < r1:
            free = np.flatnonzero(~supp[a:r1])
            if not len(free):
                break
            a += int(free[0])
            row = hit[a - r0].copy()
            row[:a + 1] = False
            row &= ~supp
            sup[row] = a
            supp |= row
            a += 1
    return sup


class Trace:
    def __init__(self, n, nstages):
        self.fate = np.full(n, nstages, np.int32)   # stage index that dropped it; nstages = output
        self.sup = np.full(n, -1, np.int64)         # NMS suppressor
        self.trank = {}                             # top-k stage -> rank within group (-1 = not ranked)
        self.out = np.zeros(0, np.int64)            # output ids in output order


def replay(side, stages):
    """Run the decision chain `stages` over `side`; see the module docstring for the stage kinds:
    ("filter", qname, thr, ">" | ">="), ("topk", k, group, keyname, tiename), ("nms", thr, group),
    ("cut", n)."""
    n = len(side)
    tr = Trace(n, len(stages))
    alive = np.ones(n, bool)
    for si, st in enumerate(stages):
        kind = st[0]
        drop = np.zeros(n, bool)
        if kind == "filter":
            _, name, thr, op = st
            q = side.q[name]
            ok = (q > thr) if op == ">" else (q >= thr)
            drop = alive & ~ok
        elif kind == "topk":
            _, k, g, key, tie = st
            idx = np.nonzero(alive)[0]
            gv = side.groups[g][idx]
            o = idx[np.lexsort((side.tkties[tie][idx], -side.keys[key][idx], gv))]
            gs = side.groups[g][o]
            start = np.searchsorted(gs, gs, side="left")
            r = np.arange(len(o)) - start
            rank = np.full(n, -1, np.int64)
            rank[o] = r
            tr.trank[si] = rank
            drop[o[r >= k]] = True
        elif kind == "nms":
            _, thr, g = st
            idx = np.nonzero(alive)[0]
            idx = idx[np.argsort(side.pos[idx], kind="stable")]
            gv = side.groups[g][idx]
            for gval in np.unique(gv):
                ids = idx[gv == gval]
                sup = _greedy_nms(side.box, ids, thr)
                tr.sup[ids[sup >= 0]] = ids[sup[sup >= 0]]
                drop[ids[sup >= 0]] = True
        elif kind == "cut":
            _, N = st
            idx = np.nonzero(alive)[0]
            idx = idx[np.argsort(side.pos[idx], kind="stable")]
            drop[idx[N:]] = True
        else:
            raise ValueError(kind)
        tr.fate[drop] = si
        alive &= ~drop
    idx = np.nonzero(alive)[0]
    tr.out = idx[np.argsort(side.pos[idx], kind="stable")]
    return tr


# ------------------------------------------------------------------------------ classification
def _topk_before(side, st, x, y):
    """x ahead of y in the top-k order of stage st on `side` (same group)."""
    _, _, _, key, tie = st
    kx, ky = side.keys[key][x], side.keys[key][y]
    if kx != ky:
        return kx > ky
    return side.tkties[tie][x] < side.tkties[tie][y]


def classify(sA, tA, sB, tB, stages, absent=None):
    """Attribute every candidate whose fate differs between side A (oracle) and side B (engine).
    absent = (bool [n] for A, bool [n] for B): candidates that do not exist on that side (an
    end-to-end box stage over the union of both sides' proposals: a proposal one side's RPN did not
    emit).  Such a candidate is dropped by the first stage (a filter) on that side, and the divergence
    is attributed to the upstream flip ("proposal_flip"), which the caller must explain at its own
    stage.  Returns {"flips": [dict per divergent candidate], "unexplained": [ids], "by_stage": {...}}."""
    fa, fb = tA.fate, tB.fate
    div = np.nonzero(fa != fb)[0]
    base, deps, info = {}, {}, {}
    for x in div:
        x = int(x)
        s = int(min(fa[x], fb[x]))
        st = stages[s]
        kind = st[0]
        A_passes = fa[x] > s
        P, D, tP, tD = (sA, sB, tA, tB) if A_passes else (sB, sA, tB, tA)
        rec = {"id": x, "stage": s, "kind": kind, "dropped_by": "engine" if A_passes else "oracle"}
        if absent is not None and absent[1 if A_passes else 0][x]:
            rec.update(margin=None)
            base[x] = "proposal_flip"
        elif kind == "filter":
            _, name, thr, op = st
            qa, qb = float(sA.q[name][x]), float(sB.q[name][x])
            okP = (P.q[name][x] > thr) if op == ">" else (P.q[name][x] >= thr)
            okD = (D.q[name][x] > thr) if op == ">" else (D.q[name][x] >= thr)
            rec.update(quantity=name, margin=abs(qa - thr), delta=abs(qa - qb))
            if okP and not okD:
                base[x] = "straddle"
        elif kind == "topk":
            _, k, g, key, tie = st
            grp = D.groups[g][x]
            rank = tD.trank[s]
            members = np.nonzero((rank >= 0) & (rank < k) & (D.groups[g] == grp))[0]
            best = None
            for y in members:
                y = int(y)
                if y == x:
                    continue
                if tP.fate[y] < s:
                    deps.setdefault(x, []).append(y)
                elif not _topk_before(P, st, y, x):
                    m = abs(float(sA.keys[key][x]) - float(sA.keys[key][y]))
                    best = m if best is None else min(best, m)
            rec.update(margin=best)
            if best is not None:
                base[x] = "inversion"
        elif kind == "nms":
            thr = st[1]
            y = int(tD.sup[x])
            rec["suppressor"] = y
            if y < 0:
                pass
            elif tP.fate[y] >= s and P.pos[y] > P.pos[x]:
                rec["margin"] = abs(float(sA.score[x]) - float(sA.score[y]))
                base[x] = "inversion"
            elif tP.fate[y] <= s:
                deps.setdefault(x, []).append(y)
                rec["margin"] = 0.0
            else:
                ia = float(iou_rows(sA.box, y, np.asarray([x]))[0])
                ib = float(iou_rows(sB.box, y, np.asarray([x]))[0])
                iP, iD = (ia, ib) if A_passes else (ib, ia)
                rec.update(iou_oracle=ia, iou_engine=ib, margin=abs(ia - thr), delta=abs(ia - ib))
                if iP <= thr < iD:
                    base[x] = "iou_straddle"
        elif kind == "cut":
            ahead = tD.out[:st[1]]
            best = None
            for y in ahead:
                y = int(y)
                if tP.fate[y] < s:
                    deps.setdefault(x, []).append(y)
                elif P.pos[y] > P.pos[x]:
                    m = abs(float(sA.score[x]) - float(sA.score[y]))
                    best = m if best is None else min(best, m)
            rec.update(margin=best)
            if best is not None:
                base[x] = "inversion"
        info[x] = rec
    explained = dict(base)
    changed = True
    while changed:
        changed = False
        for x, ys in deps.items():
            if x not in explained and any(y in explained for y in ys):
                explained[x] = "cascade"
                changed = True
    flips = []
    for x in div:
        x = int(x)
        r = info[x]
        r["reason"] = explained.get(x)
        flips.append(r)
    unexplained = [r for r in flips if r["reason"] is None]
    by = {}
    for r in flips:
        key = f"{r['kind']}:{r['reason']}"
        by[key] = by.get(key, 0) + 1
    return {"flips": flips, "unexplained": unexplained, "by_stage": by}


def max_margin(report, kinds=("straddle", "inversion", "iou_straddle"), stages=None):
    """Largest reference-side boundary distance over the base-explained flips of `report` (optionally
    only those attributed to stage kinds `stages`, e.g. ("topk",) whose key may be a logit)."""
    ms = [r["margin"] for r in report["flips"] if r["reason"] in kinds and r.get("margin") is not None
          and (stages is None or r["kind"] in stages)]
    return max(ms) if ms else 0.0


def box_rel_err(ref, got):
    """Per-row max coordinate difference relative to the row's scale max(1, |coord|, w, h): a decoded
    coordinate's rounding error is proportional to its box's size (BoxCoder.decode multiplies the
    deltas by the anchor / proposal width and height), not to its distance from the image origin."""
    ref, got = np.asarray(ref, np.float64).reshape(-1, 4), np.asarray(got, np.float64).reshape(-1, 4)
    size = np.maximum(ref[:, 2] - ref[:, 0], ref[:, 3] - ref[:, 1])[:, None]
    return (np.abs(ref - got) / np.maximum(np.maximum(1.0, np.abs(ref)), size)).max(1) if len(ref) else np.zeros(0)


def paired_deltas(sA, tA, sB, tB):
    """Rows output by both sides, paired by candidate identity: (count, max |score diff|, max
    box_rel_err)."""
    both = np.intersect1d(tA.out, tB.out)
    if not len(both):
        return 0, 0.0, 0.0
    ds = float(np.abs(sA.score[both] - sB.score[both]).max())
    db = float(box_rel_err(sA.box[both], sB.box[both]).max())
    return int(len(both)), ds, db


def compare(sA, sB, stages):
    """Replay both sides and classify: the dict the parity tests assert on."""
    tA, tB = replay(sA, stages), replay(sB, stages)
    rep = classify(sA, tA, sB, tB, stages)
    n, ds, db = paired_deltas(sA, tA, sB, tB)
    rep.update(traces=(tA, tB), paired=n, n_oracle=int(len(tA.out)), n_engine=int(len(tB.out)),
               max_score_diff=ds, max_box_rel=db)
    return rep


def summary(rep):
    return {k: rep[k] for k in ("n_oracle", "n_engine", "paired", "max_score_diff", "max_box_rel", "by_stage")} | {
        "unexplained": len(rep["unexplained"]), "max_margin": max_margin(rep)}


def check_replay_reproduces(trace, side, boxes, scores, labels, label_of, scale=None, rtol=0.0):
    """The replay's output ids reproduce a model's actual output rows (boxes / scores / labels) in
    order: exactly (rtol 0) or to within rtol (values recomputed on the host from device inputs)."""
    ids = trace.out
    assert len(ids) == len(scores), ("row count", len(ids), len(scores))
    if label_of is not None:
        np.testing.assert_array_equal(label_of(ids), np.asarray(labels))
    bx = side.box[ids]
    if scale is not None:
        bx = bx * np.asarray(scale, np.float32)
    if rtol == 0.0:
        np.testing.assert_array_equal(side.score[ids], np.asarray(scores, np.float32))
        np.testing.assert_array_equal(bx, np.asarray(boxes, np.float32))
    else:
        np.testing.assert_allclose(side.score[ids], scores, rtol=rtol, atol=1e-7)
        np.testing.assert_allclose(bx, boxes, rtol=rtol, atol=1e-4)
