"""GeneralizedRCNNTransform's resize size for FRCNN / RetinaNet (reached from
torch_models/detect.py:30,78).

torchvision's `_resize_image_and_masks` computes the scale on float32 tensors,
    scale = torch.min(800. / min_f32, 1333. / max_f32)
where `float / Tensor` is `Tensor.__rtruediv__` = `reciprocal(t) * x`, then resizes with
`scale_factor=scale.item(), recompute_scale_factor=True`, i.e. size = floor(side * scale) in double.
The restatement below runs exactly those torch tensor ops; the engine's Python host
(models.FasterRCNNFPNv2.resized_size), the oracle (oracle/tv_ops.resize_output_size) and the native
lowering (csrc/lower.hip, checked through the PREPROCESS record) must all agree with it.  A double
scale gives 800 rows instead of 799 on 427x640, 375x500 and 333x500 (missing #1).
"""
import math

import pytest
import torch

from edgeml_amd import models, native, synthetic
from oracle import tv_ops

FIXED = {(427, 640): (799, 1199), (375, 500): (799, 1066), (333, 500): (799, 1201),
         (640, 640): (800, 800), (480, 640): (800, 1066), (640, 480): (1066, 800), (612, 612): (800, 800)}


def torch_rule(h, w, min_size=800.0, max_size=1333.0):
    im_shape = torch.tensor([h, w])
    mn = torch.min(im_shape).to(dtype=torch.float32)
    mx = torch.max(im_shape).to(dtype=torch.float32)
    scale = torch.min(min_size / mn, max_size / mx).item()
    return int(math.floor(float(h) * scale)), int(math.floor(float(w) * scale))


def double_rule(h, w):
    s = min(800.0 / min(h, w), 1333.0 / max(h, w))
    return int(math.floor(h * s)), int(math.floor(w * s))


@pytest.fixture(scope="module")
def frcnn():
    return models.FasterRCNNFPNv2(synthetic.synthetic_state_dict("faster_rcnn", 91, seed=3, calibrated=False), 91)


def test_fixed_cases(frcnn):
    for (h, w), want in FIXED.items():
        assert torch_rule(h, w) == want, (h, w)
        assert frcnn.resized_size(h, w) == want, (h, w)
        assert tv_ops.resize_output_size(h, w, 800, 1333) == want, (h, w)


def test_enumerated_sizes_match_torch_rule(frcnn):
    """Every (H, W) on a grid covering COCO's image sizes (and the >1333/800 aspect regime)."""
    differ_from_double = 0
    for h in range(64, 1300, 7):
        for w in range(64, 1300, 11):
            want = torch_rule(h, w)
            assert frcnn.resized_size(h, w) == want, (h, w)
            assert tv_ops.resize_output_size(h, w, 800, 1333) == want, (h, w)
            differ_from_double += want != double_rule(h, w)
    assert differ_from_double > 0  # the grid does exercise the sizes where the two rules part


@pytest.mark.parametrize("h,w", [(427, 640), (375, 500), (333, 500), (640, 427), (500, 333), (1080, 1920)])
def test_native_lowering_uses_the_same_rule(h, w):
    """csrc/lower.hip's FasterRCNN::resized_size, read back from its PREPROCESS record (i[3], i[4])."""
    rec = native.records("faster_rcnn", 1, h, w, 0, 0, 91, True, False)
    pre = rec[0]
    assert int(pre["kind"]) == 2  # EDGEDET_OP_PREPROCESS
    assert (int(pre["i"][3]), int(pre["i"][4])) == torch_rule(h, w)
