"""Parity helpers shared by the GPU tests, smoke() and bench.py (test infrastructure)."""
import numpy as np


def compare_detections(ref, got, box_tol=1e-3, score_tol=1e-3):
    """Compare two detection dicts (boxes/scores/labels, numpy or torch) of one image.

    Rows are compared in order (both are score-sorted with the same tie rule).  Returns a report
    dict; `exact_set` is True when counts and labels agree row by row and every box/score is within
    tolerance (relative to max(1, |ref|) for boxes).
    """
    def a(x):
        return x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)

    rb, rs, rl = a(ref["boxes"]), a(ref["scores"]), a(ref["labels"])
    gb, gs, gl = a(got["boxes"]), a(got["scores"]), a(got["labels"])
    rep = {"n_ref": len(rs), "n_got": len(gs)}
    n = min(len(rs), len(gs))
    rep["label_mismatch"] = int((rl[:n] != gl[:n]).sum())
    if n:
        bd = np.abs(rb[:n] - gb[:n]) / np.maximum(1.0, np.abs(rb[:n]))
        rep["max_box_rel"] = float(bd.max())
        rep["max_score_abs"] = float(np.abs(rs[:n] - gs[:n]).max())
        rep["first_bad_row"] = int(np.argmax((bd.max(1) > box_tol) | (np.abs(rs[:n] - gs[:n]) > score_tol)
                                             | (rl[:n] != gl[:n]))) if (
            (bd.max(1) > box_tol) | (np.abs(rs[:n] - gs[:n]) > score_tol) | (rl[:n] != gl[:n])).any() else -1
    else:
        rep["max_box_rel"] = rep["max_score_abs"] = 0.0
        rep["first_bad_row"] = -1
    rep["exact_set"] = (rep["n_ref"] == rep["n_got"] and rep["label_mismatch"] == 0
                        and rep["max_box_rel"] <= box_tol and rep["max_score_abs"] <= score_tol)
    return rep


def set_match(ref, got, box_tol=1e-3, score_tol=1e-3):
    """Order-insensitive match: fraction of reference rows with a same-label row within tolerance."""
    def a(x):
        return x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)

    rb, rs, rl = a(ref["boxes"]), a(ref["scores"]), a(ref["labels"])
    gb, gs, gl = a(got["boxes"]), a(got["scores"]), a(got["labels"])
    if len(rs) == 0:
        return 1.0 if len(gs) == 0 else 0.0
    used = np.zeros(len(gs), bool)
    hit = 0
    for i in range(len(rs)):
        cand = np.nonzero((gl == rl[i]) & ~used & (np.abs(gs - rs[i]) <= score_tol)
                          & (np.abs(gb - rb[i]).max(1) <= box_tol * np.maximum(1, np.abs(rb[i]).max())))[0]
        if len(cand):
            used[cand[0]] = True
            hit += 1
    return hit / len(rs)
