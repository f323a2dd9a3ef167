"""Faster R-CNN end to end against the CPU oracle, every difference attributed.

bench.py's ORIE leg writes the engine's FRCNN files from the engine's OWN proposals; the stage-by-stage
parity of tests/parity_models.py feeds the oracle's box head the engine's proposals, so a row that
differs because the two sides' proposals differ never reached an assertion there.  Here both sides
run end to end on the 48 seeded images of that leg (tests/golden/g5_orie_f64.npz, input checksums
pinned), the engine at batch 1 as the leg runs it, against
  * the float32 oracle (the reference CPU path's restatement), and
  * the float64 oracle (the ground truth of the leg's `vs_f64`; dense arithmetic in float64, heads
    rounded to float32, float32 post-processing),
and tests/e2e_witness.check_image must attribute every difference: each RPN flip and each box-stage
flip carries a boundary witness (margins in tests/e2e_witness.py: RPN score 1e-5 and logit 1e-4, IoU
and remove_small 1e-4 of the box's scale, box-stage scores 1e-3) or cascades from one, a proposal only
one side emitted explains the candidates of that proposal, identity-paired rows agree within
north_star's 1e-3 -- or their RoIs straddle a LevelMapper boundary, or (proposal shift) the reference's
box head fed the engine's proposal agrees with the engine within 1e-3 while the two proposals differ
inside the RPN's float32 band --, and every pair of rows that bench.py's identity pairing (class +
IoU >= 0.99) matches with |dconf| > 1e-3, and every row it leaves unpaired, maps to such a witness.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
_CACHE = {}


def _setup():
    if not _CACHE:
        from edgeml_amd import models, synthetic
        from edgeml_amd.distributed import usable_cpus
        torch.set_num_threads(usable_cpus())
        sd = synthetic.synthetic_state_dict("faster_rcnn", 91)
        _CACHE.update(z=np.load(os.path.join(HERE, "golden", "g5_orie_f64.npz")), sd=sd,
                      eng=models.FasterRCNNFPNv2(sd, 91).to("cuda"))
    return _CACHE


@pytest.mark.parametrize("ref,images", [("f32", range(0, 24)), ("f32", range(24, 48)),
                                        ("f64", range(0, 12)), ("f64", range(12, 24)),
                                        ("f64", range(24, 36)), ("f64", range(36, 48))])
def test_frcnn_end_to_end_differences_are_witnessed(ref, images):
    from edgeml_amd import synthetic
    from oracle.frcnn import FasterRCNNOracle
    from tests import e2e_witness as W
    c = _setup()
    z, eng = c["z"], c["eng"]
    o = FasterRCNNOracle(c["sd"], 91, dtype=torch.float64 if ref == "f64" else torch.float32)
    reps, fails = [], []
    for i in images:
        img = synthetic.make_batch(1, 640, 640, seed=int(z["seeds"][i]))
        assert float(img.double().sum()) == float(z["image_sums"][i]), "regenerated input differs from G5's"
        A = W.oracle_side(o, img[0])
        eng(img.cuda())
        B = W.engine_side(eng.plan(1, 640, 640), 0, A["anchors"])
        h, w = A["size"]
        scale = np.asarray([np.float32(640) / np.float32(w), np.float32(640) / np.float32(h)] * 2, np.float32)
        rep, f = W.check_image(A, B, 91, scale, (640, 640))
        reps.append(rep)
        fails += [(i,) + tuple(x) for x in f]
    merged = W.merge(reps)
    print(ref, list(images)[0], "..", list(images)[-1], merged)
    assert not fails, fails[:5]
    assert merged["identity_paired"] > 50 * len(reps)  # the comparison is not vacuous
