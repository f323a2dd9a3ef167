"""Every lowering's records are race-free at the record level (tests/happens_before.py, on the CPU):
each byte range a record reads was last written by a record ordered before it (same lane, or through
FORK / JOIN / WAIT), each range it writes was last read and written by records ordered before it, the
members of a grouped launch touch disjoint outputs, and every record is joined into lane 0 by the end
of the plan.  The checker itself is shown to catch a moved lane, a dropped WAIT /
JOIN edge and overlapping group members."""
import numpy as np
import pytest

from edgeml_amd import models, ops
from tests import happens_before as hb

CASES = [
    ("ssd", 32, 640, 640, True), ("ssd", 16, 640, 640, True), ("ssd", 2, 480, 640, False),
    ("ssd_full", 32, 640, 640, True),
    ("frcnn", 8, 640, 640, True), ("frcnn", 6, 427, 640, True), ("frcnn", 1, 375, 500, False),
    ("retinanet", 8, 640, 640, True), ("retinanet", 2, 427, 640, False),
]
_MODELS = {}


def _model(kind):
    if kind not in _MODELS:
        _MODELS[kind] = {"ssd": lambda: models.ssdlite320_mobilenet_v3_large(),
                         "ssd_full": lambda: models.ssdlite320_mobilenet_v3_large(reduced_tail=False),
                         "frcnn": lambda: models.fasterrcnn_resnet50_fpn_v2(),
                         "retinanet": lambda: models.retinanet_resnet50_fpn_v2()}[kind]()
    return _MODELS[kind]


@pytest.mark.parametrize("kind,B,H,W,u8", CASES)
def test_plan_records_are_race_free(kind, B, H, W, u8):
    plan = _model(kind).build_plan(B, H, W, u8)
    races = hb.check(plan)
    assert not races, races[:10]


class _Mut:
    """A plan with its records replaced (the checker reads records, arena, buffers, ops, B)."""

    def __init__(self, plan, recs, names=None):
        self.records, self.arena, self.buffers, self.B = recs, plan.arena, plan.buffers, plan.B
        self.ops = plan.ops if names is None else [type("O", (), {"name": n}) for n in names]


def _ssd32():
    return _model("ssd").build_plan(32, 640, 640, True)


def test_checker_catches_an_op_moved_to_another_lane():
    plan = _ssd32()
    recs = plan.records.copy()
    lanes = recs["i"][:, ops.LANE_FIELD]
    k = int(np.nonzero(lanes == 1)[0][1])  # chain 1's second record reads what its first wrote on lane 1
    recs["i"][k, ops.LANE_FIELD] = 0
    assert hb.check(_Mut(plan, recs))


def test_checker_catches_a_missing_join_edge():
    plan = _ssd32()
    keep = [k for k, r in enumerate(plan.records) if r["kind"] != ops.JOIN]
    recs = plan.records[keep]
    names = [plan.ops[k].name for k in keep]
    races = hb.check(_Mut(plan, recs, names))
    assert any("not joined" in r for r in races), races[:3]


def test_checker_catches_overlapping_group_members():
    plan = _ssd32()
    recs = plan.records.copy()
    k = next(j for j, r in enumerate(recs) if r["kind"] == ops.GROUP)
    recs[k + 2]["p"][3] = recs[k + 1]["p"][3]  # two members write the same output
    recs[k + 2]["i"][20] = recs[k + 1]["i"][20]
    assert any("group members" in r for r in hb.check(_Mut(plan, recs)))


def test_checker_catches_a_dropped_wait():
    plan = _model("retinanet").build_plan(2, 640, 640, False)
    waits = [k for k, r in enumerate(plan.records) if r["kind"] == ops.WAIT]
    joins = [k for k, r in enumerate(plan.records) if r["kind"] == ops.JOIN]
    if not waits:
        pytest.skip("no WAIT record in this lowering")
    keep = [k for k in range(len(plan.records)) if k != waits[0]]
    recs = plan.records[keep]
    names = [plan.ops[k].name for k in keep]
    assert joins and hb.check(_Mut(plan, recs, names))


@pytest.mark.parametrize("kind,B,H,W,u8", CASES)
def test_every_read_sees_this_pass_or_a_constant(kind, B, H, W, u8):
    """No record reads bytes that only a later record of the pass writes (a replayed graph would hand
    it the previous pass's values -- a cross-pass dependence that timing cannot disturb but that makes
    the first pass differ from the rest), nor bytes of a written buffer that nothing writes."""
    plan = _model(kind).build_plan(B, H, W, u8)
    stale = hb.stale_reads(plan)
    assert not stale, stale[:10]


def test_stale_read_check_catches_a_consumer_moved_before_its_producer():
    plan = _ssd32()
    recs = plan.records
    k = next(j for j, r in enumerate(recs) if r["kind"] == ops.CONV and j > 0 and recs[j - 1]["kind"] == ops.CONV
             and recs[j - 1]["p"][3] == recs[j]["p"][0])
    order = list(range(len(recs)))
    order[k - 1], order[k] = k, k - 1
    mut = _Mut(plan, recs[order], [plan.ops[j].name for j in order])
    stale = hb.stale_reads(mut)
    assert any("writes later" in s for s in stale), stale[:3]
