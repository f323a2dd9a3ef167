"""Happens-before check of a plan's records (test infrastructure).

The native executor (csrc/exec.hip run_ops) issues each record on lane 0 (the caller's stream) or a
side lane; FORK makes side lanes 1..n wait for everything issued so far on lane 0, JOIN makes lane 0
wait for lanes 1..n, WAIT(a, b) makes lane a wait for everything issued so far on lane b, and a GROUP's
members run as one launch on the GROUP's lane.  check_topology validates that structure only.  This
module checks the DATA: for every byte range a record reads, the last record that wrote it must be
ordered before the reader (same lane earlier, or through FORK / JOIN / WAIT), and for every range a
record writes, every earlier reader and writer of it must be ordered before the writer.  A range that
two unordered records touch, one of them writing, is a race whose outcome depends on timing.

Ordering is tracked with vector clocks (one per lane).  A plan is replayed many times on one stream:
the check also requires every record to be ordered before the end of the plan (joined into lane 0),
so a replay never overlaps the previous one.

Byte ranges come from the record fields (csrc/exec.hip's record layouts): the exact strided extents of
CONV inputs / outputs / residuals (the SSDLite heads write map slices of the concatenated outputs,
and the batch chains write batch slices of shared buffers), the dense extents of the depthwise /
pooling records, and otherwise the named buffer holding the pointer (edgedet_model_buffers), cut to
the record's batch when the buffer's leading dimension is the plan's batch.  Pointers outside the
workspace (the packed weights) are never written and are ignored.
"""
import numpy as np

from edgeml_amd import ops

R, W, RW = "r", "w", "rw"

# (kind) -> {pointer field: role}; the record layouts of csrc/exec.hip
ROLES = {
    ops.MEMSET: {0: W},
    ops.PREPROCESS: {0: R, 2: R, 1: W},
    ops.CONV: {0: R, 2: R, 4: R, 5: R, 7: R, 3: W, 8: RW},
    ops.SSD_STEM: {0: R, 8: R, 9: R, 7: W},
    ops.DWCONV: {0: R, 3: W, 4: W},
    ops.MBCONV: {0: R, 7: W},
    ops.CHANNEL_MEAN: {0: R, 1: W},
    ops.SE_FC: {0: R, 5: W, 6: W},
    ops.MAXPOOL: {0: R, 1: W},
    ops.SSD_SCORES: {0: R, 1: R, 2: R, 3: W, 4: W},
    ops.SSD_CLASS_NMS: {0: R, 1: R, 2: W, 3: W, 4: W, 5: W, 6: W},
    ops.MERGE_TOPK: {0: R, 1: R, 2: R, 3: R, 4: R, 5: R, 6: W, 7: W, 8: W, 9: W},
    ops.RPN_LEVEL_NMS: dict([(j, R) for j in range(10)] + [(j, R) for j in range(15, 20)] +
                            [(j, W) for j in range(10, 15)] + [(j, RW) for j in (20, 21, 22, 23)]),
    ops.ROI_ALIGN: {0: R, 1: R, 2: R, 3: R, 4: R, 5: R, 6: W},
    ops.BOX_SCORES: {0: R, 1: R, 2: R, 3: W, 4: W},
    ops.BOX_CLASS_NMS: {0: R, 1: R, 2: R, 3: W, 4: W, 5: W, 6: W, 7: W},
    ops.SSD_POSTPROCESS: {0: R, 1: R, 4: R, 2: RW, 3: RW, 5: W, 6: W, 7: W, 8: W},
    ops.GN_STATS: {0: R, 3: W, 4: W},
    ops.RETINA_SELECT: {0: R, 1: R, 2: R, 3: W, 4: W, 5: W, 6: W, 7: W, 8: RW, 9: RW, 10: RW},
    ops.RETINA_CLASS_NMS: {0: R, 1: R, 2: R, 3: R, 4: R, 5: W, 6: W, 7: W, 8: W, 9: W},
}


def op_batch(kind, i):
    """The images a record covers (its batch field)."""
    if kind == ops.BOX_SCORES:
        return int(i[1])
    if kind == ops.ROI_ALIGN:
        return int(i[3])
    return int(i[0])


def _per_image(off, B, bstride, extent):
    """The element ranges of a strided batch: one per image when an image's extent leaves a gap to
    the next image (a map slice of the SSDLite heads' concatenated outputs), else one."""
    if B > 1 and extent < bstride:
        return [(off + 4 * b * bstride, 4 * extent) for b in range(B)]
    return off, 4 * ((B - 1) * bstride + extent)


def _exact(kind, i, f):
    """Exact (offset from the pointer, bytes) of the strided / dense fields -- a list of them for a
    batch with gaps -- or None."""
    i = [int(v) for v in i]
    if kind == ops.CONV:
        B, H, W_, Cin, Ho, Wo, Cout = i[0:7]
        xp, yp, rp, xb, yb, rb, yoff, rH, rW = i[14], i[15], i[16], i[17], i[18], i[19], i[20], i[21], i[22]
        if f == 0:
            return _per_image(0, B, xb, (H * W_ - 1) * xp + Cin)
        if f == 3:
            return _per_image(4 * yoff, B, yb, (Ho * Wo - 1) * yp + Cout)
        if f == 4:
            return _per_image(0, B, rb, (rH * rW - 1) * rp + Cout)
        if f == 8:
            return 0, 2 * 3 * B * H * W_ * Cin + 64
    if kind == ops.DWCONV:
        B, H, W_, C, Ho, Wo = i[0:6]
        if f == 0:
            return 0, 4 * B * H * W_ * C
        if f == 3:
            return 0, 4 * B * Ho * Wo * C
        if f == 4:
            return 0, 4 * B * (i[10] or ops.SE_PARTS) * C
    if kind == ops.MBCONV:
        B, H, W_, Cin, Cexp, Cout, Ho, Wo = i[0:8]
        if f == 0:
            return 0, 4 * B * H * W_ * Cin
        if f == 7:
            return 0, 4 * B * Ho * Wo * Cout
    if kind == ops.MAXPOOL:
        B, H, W_, C, Ho, Wo = i[0:6]
        return (0, 4 * B * H * W_ * C) if f == 0 else (0, 4 * B * Ho * Wo * C)
    if kind == ops.MEMSET:
        return 0, i[0]
    if kind == ops.SSD_STEM:
        B, H, W_, Ho, Wo, _, _, H0, W0 = i[0:9]
        if f == 7:
            return 0, 4 * B * Ho * Wo * 16
        if f == 0:
            return 0, 4 * B * H * W_ * 4
        if f == 8:
            return 0, 4 * B * 3 * H0 * W0
        if f == 9:
            return 0, B * 3 * H0 * W0
    if kind == ops.BOX_SCORES and f == 0:  # predictor rows of LD floats, 5 * NC of them written / read
        LD, B, R, NC = i[0:4]
        return [(4 * r * LD, 4 * 5 * NC) for r in range(B * R)]
    if kind == ops.PREPROCESS:
        B, H, W_, Ho, Wo, Hp, Wp = i[0:7]
        return {0: (0, 4 * B * 3 * H * W_), 2: (0, B * 3 * H * W_), 1: (0, 16 * B * Hp * Wp)}[f]
    return None


class Accesses:
    def __init__(self, plan):
        self.base = plan.arena.data_ptr()
        self.size = plan.arena.numel()
        self.B = plan.B
        bufs = sorted(plan.buffers.values(), key=lambda b: b.off)
        self.starts = np.array([b.off for b in bufs], np.int64)
        self.bufs = bufs

    def buffer_of(self, off):
        k = int(np.searchsorted(self.starts, off, side="right")) - 1
        if k < 0:
            return None
        b = self.bufs[k]
        return b if off < b.off + b.nbytes else None

    def ranges(self, rec):
        """[(lo, hi, role, field)] arena byte ranges of one record."""
        kind = int(rec["kind"])
        out = []
        for f, role in ROLES.get(kind, {}).items():
            ptr = int(rec["p"][f])
            if not ptr:
                continue
            off = ptr - self.base
            if not 0 <= off < self.size:
                continue  # packed weights / caller memory outside the workspace: never written by a record
            ex = _exact(kind, rec["i"], f)
            if isinstance(ex, list):
                for o_, n in ex:
                    assert n > 0 and off + o_ + n <= self.size, (kind, f, off + o_, n)
                    out.append((off + o_, off + o_ + n, role, f))
                continue
            if ex is not None:
                lo, n = off + ex[0], ex[1]
            else:
                b = self.buffer_of(off)
                if b is None:
                    raise AssertionError(f"record kind {kind} field {f}: pointer outside every named buffer")
                lo, hi = off, b.off + b.nbytes
                if b.shape and b.shape[0] == self.B and op_batch(kind, rec["i"]) < self.B:
                    hi = min(hi, lo + b.nbytes // self.B * op_batch(kind, rec["i"]))
                n = hi - lo
            assert n > 0 and lo + n <= self.size, (kind, f, lo, n)
            out.append((lo, lo + n, role, f))
        return out


def check(plan, names=None):
    """Races between the records of `plan` (NativePlan): a list of strings, empty when every
    conflicting pair of accesses is ordered."""
    recs = plan.records
    names = names or [op.name for op in plan.ops]
    acc = Accesses(plan)
    L = ops.MAX_LANES
    vc = np.zeros((L, L), np.int64)          # vc[lane] = that lane's vector clock
    hist = []                                  # (lo, hi, role, op index, lane, clock copy)
    races = []

    def ordered(lane_a, clock_a, lane_b):      # a (issued earlier) happens before the lane_b's next op
        return clock_a[lane_a] <= vc[lane_b][lane_a]

    k = 0
    while k < len(recs):
        kind, lane = int(recs[k]["kind"]), int(recs[k]["i"][ops.LANE_FIELD])
        if kind == ops.FORK:
            for l in range(1, int(recs[k]["i"][0]) + 1):
                vc[l] = np.maximum(vc[l], vc[0])
            k += 1
            continue
        if kind == ops.JOIN:
            for l in range(1, int(recs[k]["i"][0]) + 1):
                vc[0] = np.maximum(vc[0], vc[l])
            k += 1
            continue
        if kind == ops.WAIT:
            a, b = int(recs[k]["i"][0]), int(recs[k]["i"][1])
            vc[a] = np.maximum(vc[a], vc[b])
            k += 1
            continue
        members = [k]
        if kind == ops.GROUP:
            members = list(range(k + 1, k + 1 + int(recs[k]["i"][0])))
        vc[lane][lane] += 1
        clock = vc[lane].copy()
        per = [acc.ranges(recs[m]) for m in members]
        mine = [r for rs in per for r in rs]
        for a in range(len(per)):          # a grouped launch's members run concurrently
            for b in range(a + 1, len(per)):
                for lo, hi, role, f in per[a]:
                    for plo, phi, prole, pf in per[b]:
                        if lo < phi and plo < hi and (role != R or prole != R):
                            races.append(f"group members {names[members[a]]} / {names[members[b]]} overlap "
                                         f"(p{f} {role} / p{pf} {prole})")
        for lo, hi, role, f in mine:
            for (plo, phi, prole, pk, plane, pclock) in hist:
                if phi <= lo or hi <= plo:
                    continue
                if role == R and prole == R:
                    continue
                if not ordered(plane, pclock, lane):
                    races.append(f"{names[pk]} ({prole}) -> {names[members[0]]} ({role}, p{f}): "
                                 f"bytes [{max(lo, plo)}, {min(hi, phi)}) unordered (lanes {plane} -> {lane})")
        for lo, hi, role, f in mine:
            hist.append((lo, hi, role, members[0], lane, clock))
        k = members[-1] + 1
    # the next replay starts on lane 0: every record must be joined into it
    for (_, _, _, pk, plane, pclock) in hist:
        if not pclock[plane] <= vc[0][plane]:
            races.append(f"{names[pk]} on lane {plane} is not joined into lane 0 by the end of the plan")
            break
    return races


def _subtract(lo, hi, covered):
    """[lo, hi) minus the union of the sorted, merged intervals `covered` -> list of intervals."""
    out, cur = [], lo
    for a, b in covered:
        if b <= cur:
            continue
        if a >= hi:
            break
        if a > cur:
            out.append((cur, min(a, hi)))
        cur = max(cur, b)
        if cur >= hi:
            break
    if cur < hi:
        out.append((cur, hi))
    return out


def _add(covered, lo, hi):
    """Insert [lo, hi) into the sorted, merged interval list."""
    res, placed = [], False
    for a, b in covered:
        if b < lo or a > hi:
            res.append((a, b))
        else:
            lo, hi = min(lo, a), max(hi, b)
    res.append((lo, hi))
    res.sort()
    return res


def stale_reads(plan, names=None):
    """Reads of bytes no earlier record of the same pass wrote (in issue order), classified: bytes that a
    LATER record writes are read from the previous pass (a replayed plan would see the last pass's
    values there, its first pass the zeroed workspace) -- reported; bytes no record writes must be the
    constants edgedet_model_prepare wrote or the input images -- others are reported too.  Empty when
    every read sees this pass's data or a constant."""
    recs = plan.records
    names = names or [op.name for op in plan.ops]
    acc = Accesses(plan)
    order = []  # (record index, lo, hi, role)
    k = 0
    while k < len(recs):
        kind = int(recs[k]["kind"])
        if kind in (ops.FORK, ops.JOIN, ops.WAIT):
            k += 1
            continue
        members = list(range(k + 1, k + 1 + int(recs[k]["i"][0]))) if kind == ops.GROUP else [k]
        for m in members:
            for lo, hi, role, f in acc.ranges(recs[m]):
                order.append((m, lo, hi, role, f))
        k = members[-1] + 1
    # bytes of a buffer that no record writes at all are constants (edgedet_model_prepare's anchors,
    # the packed tables) or the caller's input images
    written_ever = []
    for _, lo, hi, role, _ in order:
        if role != R:
            written_ever = _add(written_ever, lo, hi)
    never = []
    for b in plan.buffers.values():
        if not any(lo < b.off + b.nbytes and b.off < hi for lo, hi in written_ever):
            never = _add(never, b.off, b.off + b.nbytes)
    issues = []
    written = []
    for pos, (m, lo, hi, role, f) in enumerate(order):
        if role == R:
            for a, b in _subtract(lo, hi, written):
                later = [(m2, max(a, l2), min(b, h2)) for (m2, l2, h2, r2, _) in order[pos + 1:]
                         if r2 != R and l2 < b and a < h2]
                if later:
                    issues.append(f"{names[m]} (p{f}) reads bytes [{a}, {b}) that {names[later[0][0]]} writes later "
                                  f"in the pass: the previous pass's values")
                elif _subtract(a, b, never):
                    issues.append(f"{names[m]} (p{f}) reads bytes [{a}, {b}) that no record writes, inside a "
                                  f"buffer that records do write: uninitialised")
        else:
            written = _add(written, lo, hi)
    return issues
