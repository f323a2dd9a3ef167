"""CPU checks of the ORIE-leg machinery: the G5 float64 ground-truth fixture (tests/golden/
make_orie_f64.py) and the identity pairing of detection files (tools/rowpair.py)."""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _rows(z, tag, i):
    cnt = z[tag + "_count"]
    off = np.concatenate([[0], np.cumsum(cnt)])
    return z[tag + "_rows"][off[i]:off[i + 1]]


def test_g5_inputs_and_a_float64_forward_reproduce():
    """The fixture's inputs are the seeded images the ORIE leg regenerates (checksums), and the
    float64 SSDLite oracle reproduces its first image's file exactly on this host."""
    from edgeml_amd import fmt, synthetic
    from oracle.ssdlite import SSDLiteOracle
    z = np.load(os.path.join(HERE, "golden", "g5_orie_f64.npz"))
    assert len(z["seeds"]) == 48 and int(z["seeds"][0]) == 7000
    for i in (0, 1, 47):
        img = synthetic.make_batch(1, 640, 640, seed=int(z["seeds"][i]))
        assert float(img.double().sum()) == float(z["image_sums"][i])
    img = synthetic.make_batch(1, 640, 640, seed=int(z["seeds"][0]))
    o = SSDLiteOracle(synthetic.synthetic_state_dict("ssd", 91, True), 91, True, dtype=torch.float64)
    p = o([img[0]])[0]
    rows = fmt.format_detections(p["boxes"].numpy(), p["scores"].numpy(), p["labels"].numpy(), 640, 640)
    want = _rows(z, "weak_f64", 0)
    assert rows.shape == want.shape
    # float64 arithmetic, float32 heads: equal up to last-bit float32 rounding of the head outputs
    np.testing.assert_allclose(rows, want, rtol=0, atol=1e-6)


def test_rowpair_pairs_by_identity_not_position():
    from tools import rowpair
    rs = np.random.RandomState(0)
    a = np.zeros((6, 6))
    a[:, 0] = [1, 1, 2, 3, 3, 5]
    a[:, 1:3] = rs.uniform(0.2, 0.8, (6, 2))
    a[:, 3:5] = rs.uniform(0.05, 0.2, (6, 2))
    a[:, 5] = np.linspace(0.9, 0.4, 6)
    b = a.copy()
    b[[0, 1]] = b[[1, 0]]            # two same-class rows traded places
    b[3, 5] += 1e-4                  # a value difference
    b = np.concatenate([b[:5], [[7, 0.5, 0.5, 0.1, 0.1, 0.01]]])  # a's last row unpaired, b has a new one
    pairs, ua, ub = rowpair.pair_rows(a, b)
    assert sorted(pairs) == [(0, 1), (1, 0), (2, 2), (3, 3), (4, 4)]
    assert len(ua) == 1 and ua[0, 0] == 5 and len(ub) == 1 and ub[0, 0] == 7
    r = rowpair.compare_dirs(["x"], lambda n: a, lambda n: b)
    assert r["paired"] == 5 and r["unpaired_a"] == 1 and r["unpaired_b"] == 1 and r["order_differs"] == 1
    assert abs(r["max_paired_dconf"] - 1e-4) < 1e-9 and r["max_paired_dbox"] == 0.0
    # empty files
    e = np.zeros((0, 6))
    assert rowpair.compare_dirs(["x"], lambda n: e, lambda n: e)["files_identical"] == 1
