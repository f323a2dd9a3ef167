"""Oracle parity at the benchmarked configurations, every flip accounted for.

BASELINE configs[1] (SSDLite320 b=32 640x640) and configs[2] (FRCNN-R50-FPN-v2 b=8 640x640) run
through exactly what bench.py times: the same seeded weights and inputs, the same plan (SSD: two
16-image chains on stream lanes with the tuned tiles of those shapes; FRCNN: the b=8 tiles
including split-K and the 392,000-row box head), captured into a hipGraph and replayed on a
stream.  Protocol: tests/parity_models.py (decision replay, identity pairing, every divergent
candidate a boundary flip within EPS of its threshold / cut / NMS IoU).
"""
import pytest
import torch

from tests import parity_models as PM

pytestmark = pytest.mark.gpu


def _run_graph(plan):
    s = torch.cuda.Stream()
    plan.capture(s)
    plan.replay(s)
    s.synchronize()


def test_ssd_b32_bench_plan_matches_oracle():
    from edgeml_amd import models, synthetic
    sd = synthetic.synthetic_state_dict("ssd", 91, True, seed=0)  # bench.py's weights
    m = models.SSDLite320(sd, 91, True).to("cuda")
    plan = m.plan(32, 640, 640)
    assert plan.chains == 2
    imgs = synthetic.make_batch(32, 640, 640, seed=0)  # bench.py's rank-0 input
    plan.input.tensor().copy_(imgs.cuda())
    _run_graph(plan)
    rep = PM.ssd_check(plan, sd, 91, True, imgs, "ssd b=32")
    print(rep)
    assert rep["rows"] == 32 * 300


def test_frcnn_b8_bench_plan_matches_oracle():
    from edgeml_amd import models, synthetic
    sd = synthetic.synthetic_state_dict("faster_rcnn", 91, seed=0)
    m = models.FasterRCNNFPNv2(sd, 91).to("cuda")
    plan = m.plan(8, 640, 640)
    imgs = synthetic.make_batch(8, 640, 640, seed=50)  # bench.py's rank-0 FRCNN input
    plan.input.tensor().copy_(imgs.cuda())
    _run_graph(plan)
    rep = PM.frcnn_check(plan, sd, 91, imgs, "frcnn b=8")
    print(rep)
    assert rep["rpn"]["rows"] == 8 * 1000 and rep["box"]["rows"] == 8 * 100
