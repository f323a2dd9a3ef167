"""Parity protocol shared by the GPU tests, smoke() and the parity report (test infrastructure).

Detections are compared in the reference's output space.  Two runs of the same fp32 algorithm with
different summation orders agree on every continuous value to ~1e-6 relative, but the discrete
decisions (score thresholds, top-k cut-offs, NMS IoU > t, ties in score order) can flip for
candidates that sit within that noise of a boundary (SURVEY.md §7 hard part 1).  The protocol:
  * `match_report` pairs every reference row with an unused engine row of the same label whose box
    (relative to max(1, |coord|)) and score agree within `tol` (north_star: 1e-3);
  * unmatched rows on either side are the decision flips; tests bound them.
"""
import numpy as np


def _a(x):
    return x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)


def match_report(ref, got, tol=1e-3):
    rb, rs, rl = _a(ref["boxes"]).reshape(-1, 4), _a(ref["scores"]).reshape(-1), _a(ref["labels"]).reshape(-1)
    gb, gs, gl = _a(got["boxes"]).reshape(-1, 4), _a(got["scores"]).reshape(-1), _a(got["labels"]).reshape(-1)
    used = np.zeros(len(gs), bool)
    matched, max_box, max_score = 0, 0.0, 0.0
    for i in range(len(rs)):
        ok = (gl == rl[i]) & ~used & (np.abs(gs - rs[i]) <= tol)
        if not ok.any():
            continue
        rel = (np.abs(gb - rb[i]) / np.maximum(1.0, np.abs(rb[i]))).max(1)
        ok &= rel <= tol
        cand = np.nonzero(ok)[0]
        if len(cand):
            j = cand[np.argmin(rel[cand])]
            used[j] = True
            matched += 1
            max_box = max(max_box, float(rel[j]))
            max_score = max(max_score, float(abs(gs[j] - rs[i])))
    sorted_ok = bool(np.all(gs[:-1] >= gs[1:])) if len(gs) > 1 else True
    return {"n_ref": int(len(rs)), "n_got": int(len(gs)), "matched": matched,
            "ref_unmatched": int(len(rs) - matched), "got_unmatched": int(len(gs) - matched),
            "max_box_rel": max_box, "max_score_abs": max_score, "scores_sorted": sorted_ok,
            "match_frac": 1.0 if len(rs) == 0 and len(gs) == 0 else matched / max(len(rs), len(gs), 1)}


def set_match(ref, got, tol=1e-3):
    return match_report(ref, got, tol)["match_frac"]
