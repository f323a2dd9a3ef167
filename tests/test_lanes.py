"""Lane topology of plan records (csrc/exec.hip check_topology), on the CPU: FORK / JOIN / WAIT and
every record's lane are checked before anything is issued, so a refused plan returns an error code
without touching a stream or a capture (the side-lane -> side-lane wait)."""
import ctypes

import numpy as np
import pytest

from edgeml_amd import ops


def _recs(spec):
    """spec: list of (kind, i0, i1, lane)."""
    r = np.zeros(len(spec), dtype=ops.OP_DTYPE)
    for k, (kind, a, b, lane) in enumerate(spec):
        r[k]["kind"] = kind
        r[k]["i"][0], r[k]["i"][1] = a, b
        r[k]["i"][ops.LANE_FIELD] = lane
    return r


def _check(r):
    L = ops.lib()
    return L.edgedet_plan_check(r.ctypes.data_as(ctypes.c_void_p), len(r))


M = ops.MEMSET
GOOD = [
    [(ops.FORK, 3, 0, 0), (M, 0, 0, 1), (ops.WAIT, 2, 1, 0), (M, 0, 0, 2), (ops.WAIT, 3, 2, 0), (M, 0, 0, 3),
     (ops.JOIN, 3, 0, 0)],                                             # chain lane 1 -> 2 -> 3
    [(ops.FORK, 2, 0, 0), (ops.WAIT, 0, 2, 0), (ops.WAIT, 1, 0, 0), (ops.JOIN, 2, 0, 0)],  # lane 0 both ways
    [(M, 0, 0, 0)],
    [(ops.GROUP, 2, 0, 0), (ops.CONV, 0, 0, 0), (ops.CONV, 0, 0, 0), (M, 0, 0, 0)],          # grouped launch
    [(ops.FORK, 1, 0, 0), (ops.GROUP, 1, 0, 1), (ops.DWCONV, 0, 0, 1), (ops.JOIN, 1, 0, 0)],  # on a side lane
]
BAD = {
    "op on a lane that is not forked": [(M, 0, 0, 1)],
    "wait: two distinct forked lanes": [(ops.FORK, 1, 0, 0), (ops.WAIT, 2, 1, 0), (ops.JOIN, 1, 0, 0)],
    "wait: two distinct forked lanes ": [(ops.FORK, 2, 0, 0), (ops.WAIT, 1, 1, 0), (ops.JOIN, 2, 0, 0)],
    "fork while side lanes are open": [(ops.FORK, 1, 0, 0), (ops.FORK, 1, 0, 0), (ops.JOIN, 1, 0, 0)],
    "join: the forked side lanes": [(ops.FORK, 2, 0, 0), (ops.JOIN, 1, 0, 0)],
    "missing JOIN": [(ops.FORK, 2, 0, 0), (M, 0, 0, 2)],
    "fork: 1..3 side lanes": [(ops.FORK, 4, 0, 0), (ops.JOIN, 4, 0, 0)],
    "group: 1..12 following records": [(ops.GROUP, 3, 0, 0), (ops.CONV, 0, 0, 0), (ops.CONV, 0, 0, 0)],
    "group: 1..12 following records ": [(ops.GROUP, 13, 0, 0)] + [(ops.CONV, 0, 0, 0)] * 13,
    "group: CONV or DWCONV members": [(ops.GROUP, 1, 0, 0), (M, 0, 0, 0)],
    "group: members of one kind on the group's lane": [(ops.GROUP, 2, 0, 0), (ops.CONV, 0, 0, 0), (ops.DWCONV, 0, 0, 0)],
    "group on a lane that is not forked": [(ops.GROUP, 1, 0, 2), (ops.CONV, 0, 0, 2)],
}


@pytest.mark.parametrize("spec", GOOD)
def test_good_topologies_pass(spec):
    assert _check(_recs(spec)) == 0, ops.lib().edgedet_last_error()


@pytest.mark.parametrize("msg", sorted(BAD))
def test_bad_topologies_refused_before_issue(msg):
    r = _recs(BAD[msg])
    assert _check(r) < 0
    assert msg.strip() in ops.lib().edgedet_last_error().decode()
    # the run entry refuses it the same way before any stream or device is touched (no GPU here)
    L = ops.lib()
    assert L.edgedet_plan_run(r.ctypes.data_as(ctypes.c_void_p), len(r), None) < 0
    assert msg.strip() in L.edgedet_last_error().decode()


def test_group_members_requesting_different_tiles_refused():
    """run_group launches every CONV member with member 0's tile, so check_topology refuses a GROUP
    whose CONV members request different tiles (i23) instead of silently running one of them."""
    r = _recs([(ops.GROUP, 2, 0, 0), (ops.CONV, 0, 0, 0), (ops.CONV, 0, 0, 0)])
    r[1]["i"][23], r[2]["i"][23] = 31, 31
    assert _check(r) == 0
    r[2]["i"][23] = 39
    assert _check(r) < 0
    assert "different tiles" in ops.lib().edgedet_last_error().decode()
