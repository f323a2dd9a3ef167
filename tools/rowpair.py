"""Identity pairing of two detect.py output files (measurement helper for bench.py's ORIE leg and
tools/config4_full.py; not product code).

A file is the (N, 6) float64 array detect.py writes (detect.py:83-105): [cls, xc, yc, w, h, conf],
normalised.  Two implementations of the same detector give files that differ in a few rows (a
detection on one side only, where a score or an IoU sits at a threshold) and in the low bits of the
others, and rows of equal class and near-equal score can trade places.  Comparing by row position
mixes those cases up.  Here rows are paired by identity instead: same class and IoU >= 0.99 (greedy
over the highest IoUs first, each row used once).  Paired rows give the value differences; the rest
are the unpaired detections of each side.
"""
import numpy as np

IOU_PAIR = 0.99


def _xyxy(r):
    xc, yc, w, h = r[:, 1], r[:, 2], r[:, 3], r[:, 4]
    return np.stack([xc - w / 2, yc - h / 2, xc + w / 2, yc + h / 2], 1)


def pair_rows(a, b, iou=IOU_PAIR):
    """Pair the rows of two files.  -> (pairs [(i, j)], unpaired rows of a, unpaired rows of b)."""
    a = np.asarray(a, np.float64).reshape(-1, 6)
    b = np.asarray(b, np.float64).reshape(-1, 6)
    pairs = []
    used_a, used_b = np.zeros(len(a), bool), np.zeros(len(b), bool)
    for c in np.intersect1d(a[:, 0], b[:, 0]):
        ia, ib = np.where(a[:, 0] == c)[0], np.where(b[:, 0] == c)[0]
        ba, bb = _xyxy(a[ia]), _xyxy(b[ib])
        lt = np.maximum(ba[:, None, :2], bb[None, :, :2])
        rb = np.minimum(ba[:, None, 2:], bb[None, :, 2:])
        inter = np.clip(rb - lt, 0, None).prod(2)
        area = lambda x: (x[:, 2] - x[:, 0]) * (x[:, 3] - x[:, 1])  # noqa: E731
        union = area(ba)[:, None] + area(bb)[None, :] - inter
        m = np.where(union > 0, inter / np.where(union > 0, union, 1), 0.0)
        cand = np.argwhere(m >= iou)
        for k in np.argsort(-m[cand[:, 0], cand[:, 1]], kind="stable"):
            i, j = ia[cand[k, 0]], ib[cand[k, 1]]
            if not used_a[i] and not used_b[j]:
                used_a[i] = used_b[j] = True
                pairs.append((int(i), int(j)))
    return pairs, a[~used_a], b[~used_b]


def compare_dirs(names, load_a, load_b):
    """Aggregate identity-paired differences over images.  load_a / load_b: name -> rows."""
    out = {"images": len(names), "files_identical": 0, "paired": 0, "unpaired_a": 0, "unpaired_b": 0,
           "images_with_unpaired": 0, "max_paired_dconf": 0.0, "max_paired_dbox": 0.0,
           "max_unpaired_conf": 0.0, "order_differs": 0, "paired_dconf_gt_1e-4": 0, "paired_dconf_gt_1e-3": 0}
    for n in names:
        a, b = load_a(n), load_b(n)
        if a.shape == b.shape and np.array_equal(a, b):
            out["files_identical"] += 1
        pairs, ua, ub = pair_rows(a, b)
        out["paired"] += len(pairs)
        out["unpaired_a"] += len(ua)
        out["unpaired_b"] += len(ub)
        out["images_with_unpaired"] += bool(len(ua) or len(ub))
        if pairs:
            i, j = np.array(pairs).T
            dc = np.abs(a[i, 5] - b[j, 5])
            out["max_paired_dconf"] = max(out["max_paired_dconf"], float(dc.max()))
            out["paired_dconf_gt_1e-4"] += int(np.count_nonzero(dc > 1e-4))
            out["paired_dconf_gt_1e-3"] += int(np.count_nonzero(dc > 1e-3))
            out["max_paired_dbox"] = max(out["max_paired_dbox"], float(np.abs(a[i, 1:5] - b[j, 1:5]).max()))
            # the same detections in a different row order (two near-equal scores traded places)
            out["order_differs"] += bool(not np.array_equal(np.argsort(i, kind="stable"), np.argsort(j, kind="stable")))
        for u in (ua, ub):
            if len(u):
                out["max_unpaired_conf"] = max(out["max_unpaired_conf"], float(u[:, 5].max()))
    return out
