"""Seeded synthetic inputs and weights (there is no network: no COCO images, no checkpoints).

* ``synthetic_state_dict`` stands in for ``weights="DEFAULT"`` (detect.py:24,30), which would
  download COCO weights.  Conv/linear weights are He-normal from a seeded CPU generator; BatchNorm
  running statistics come from a committed calibration table (``data/calib_*.npz``, produced by
  tests/golden/make_calibration.py) so every layer's activations stay in a healthy range and the
  detectors emit realistic, well-separated scores.  This is weight synthesis, never inference.
* ``make_scene`` / ``make_dataset`` write COCO-like synthetic images and YOLO-format labels
  (SURVEY.md §8d config C1).
"""
import math
import os
import re

import numpy as np
import torch

from . import arch

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def _variant(kind, num_classes, reduced_tail):
    if kind == "ssd":
        return f"ssd_{'reduced' if reduced_tail else 'full'}_{num_classes}"
    # RetinaNet's only BatchNorms are the ResNet-50 body's, drawn first from the same seeded stream as
    # Faster R-CNN's body and fed the same transform: its calibration is FRCNN's body statistics.
    return f"frcnn_{num_classes}"


def calib_path(kind, num_classes=91, reduced_tail=True):
    return os.path.join(_DATA, f"calib_{_variant(kind, num_classes, reduced_tail)}.npz")


def table_for(kind, num_classes=91, reduced_tail=True):
    if kind == "ssd":
        return arch.ssdlite_table(num_classes, reduced_tail)
    if kind == "faster_rcnn":
        return arch.frcnn_table(num_classes)
    if kind == "retinanet":
        return arch.retinanet_table(num_classes)
    raise ValueError(kind)


def _head_gain(kind, name):
    """(weight std multiplier over 1/sqrt(fan_in), background-logit bias) for output layers."""
    if kind == "ssd":
        if name.startswith("head.classification_head") and name.endswith(".1.weight"):
            return 1.5, None
        if name.startswith("head.regression_head") and name.endswith(".1.weight"):
            return 0.7, None
    elif kind == "retinanet":
        if name == "head.classification_head.cls_logits.weight":
            return 0.7, None  # logits ~ prior bias +- 0.7: a few thousand (anchor, class) scores > 0.05
        if name == "head.regression_head.bbox_reg.weight":
            return 0.15, None
    else:
        if name == "rpn.head.cls_logits.weight":
            return 1.5, None
        if name == "rpn.head.bbox_pred.weight":
            return 0.5, None
        if name == "roi_heads.box_predictor.cls_score.weight":
            return 2.0, None
        if name == "roi_heads.box_predictor.bbox_pred.weight":
            return 0.5, None
    return None, None


def _is_residual_bn(kind, name):
    """Last BN of a residual branch (zero-init-residual style small gamma keeps random nets stable)."""
    if kind in ("faster_rcnn", "retinanet"):
        return bool(re.search(r"layer\d\.\d+\.bn3\.weight$", name))
    return False


def synthetic_state_dict(kind, num_classes=91, reduced_tail=True, seed=0, calibrated=True):
    """Deterministic torchvision-keyed state_dict for ``kind`` in {"ssd", "faster_rcnn", "retinanet"}.

    The committed BN calibration tables were measured on the seed-0 weight draws: with another seed
    the running statistics do not match the weights and activations grow by orders of magnitude
    (an ill-conditioned network on which fp32 summation-order noise reaches 1e-2), so calibrated
    weights exist for seed 0 only."""
    if calibrated and seed != 0:
        raise ValueError("calibrated synthetic weights exist for seed=0 only (data/calib_*.npz); "
                         "pass calibrated=False for other seeds")
    table = table_for(kind, num_classes, reduced_tail)
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, shape in table.items():
        if name.endswith("num_batches_tracked"):
            sd[name] = torch.tensor(0, dtype=torch.int64)
            continue
        if name.endswith("running_mean"):
            sd[name] = torch.zeros(shape)
            continue
        if name.endswith("running_var"):
            sd[name] = torch.ones(shape)
            continue
        is_bn = name.endswith(".weight") and (name[:-len(".weight")] + ".running_mean") in table
        is_bn_bias = name.endswith(".bias") and (name[:-len(".bias")] + ".running_mean") in table
        if len(shape) == 1 and name.endswith(".weight") and ".conv." in name and kind == "retinanet":
            is_bn = True  # GroupNorm affine
        if len(shape) == 1 and name.endswith(".bias") and ".conv." in name and kind == "retinanet":
            is_bn_bias = True
        if is_bn:
            lo, hi = (0.2, 0.4) if _is_residual_bn(kind, name) else (0.8, 1.2)
            sd[name] = torch.empty(shape).uniform_(lo, hi, generator=g)
        elif is_bn_bias:
            sd[name] = torch.randn(shape, generator=g) * 0.1
        elif name.endswith(".bias"):
            b = torch.randn(shape, generator=g) * 0.05
            if kind == "ssd" and name.startswith("head.classification_head"):
                b.view(6, num_classes)[:, 0] += 2.0     # background logit per anchor
            if kind == "faster_rcnn" and name == "roi_heads.box_predictor.cls_score.bias":
                b[0] += 2.0
            if kind == "retinanet" and name == "head.classification_head.cls_logits.bias":
                b += -math.log((1 - 0.01) / 0.01)  # torchvision's prior-probability init
            sd[name] = b
        else:
            fan_in = 1
            for d in shape[1:]:
                fan_in *= d
            gain, _ = _head_gain(kind, name)
            std = (gain if gain is not None else math.sqrt(2.0)) / math.sqrt(fan_in)
            sd[name] = torch.randn(shape, generator=g) * std
    if calibrated:
        path = calib_path(kind, num_classes, reduced_tail)
        if not os.path.exists(path):  # other class counts: the class-independent BN layers of the 91
            path = calib_path(kind, 91, reduced_tail)
        if not os.path.exists(path):
            raise FileNotFoundError(f"BN calibration table missing: {path} "
                                    f"(regenerate with tests/golden/make_calibration.py)")
        with np.load(path, allow_pickle=False) as z:
            for k in z.files:
                if k in table and tuple(z[k].shape) == tuple(table[k]):
                    sd[k] = torch.from_numpy(z[k].astype(np.float32))
    return sd


# ------------------------------------------------------------------------------------------ scenes
COCO_SIZES = ((480, 640), (640, 480), (427, 640), (612, 612))


def make_scene(seed, h=640, w=640, return_boxes=False):
    """uint8 [3,h,w]: smooth gradient + 3-8 filled rectangles/ellipses + noise (seeded)."""
    rs = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    ang = rs.uniform(0, 2 * np.pi)
    t = (np.cos(ang) * xx / w + np.sin(ang) * yy / h)
    t = (t - t.min()) / max(t.max() - t.min(), 1e-6)
    c0, c1 = rs.uniform(0, 255, 3), rs.uniform(0, 255, 3)
    img = c0[:, None, None] * (1 - t)[None] + c1[:, None, None] * t[None]
    boxes = []
    for _ in range(rs.randint(3, 9)):
        bw, bh = rs.uniform(0.08, 0.5) * w, rs.uniform(0.08, 0.5) * h
        x0, y0 = rs.uniform(0, w - bw), rs.uniform(0, h - bh)
        col = rs.uniform(0, 255, 3)
        if rs.rand() < 0.6:
            m = (xx >= x0) & (xx < x0 + bw) & (yy >= y0) & (yy < y0 + bh)
        else:
            m = ((xx - x0 - bw / 2) / (bw / 2)) ** 2 + ((yy - y0 - bh / 2) / (bh / 2)) ** 2 <= 1
        img[:, m] = col[:, None]
        boxes.append((rs.randint(0, 80), (x0 + bw / 2) / w, (y0 + bh / 2) / h, bw / w, bh / h))
    img = img + rs.normal(0, 8, img.shape)
    img = np.clip(np.rint(img), 0, 255).astype(np.uint8)
    return (img, boxes) if return_boxes else img


def make_batch_u8(n, h=640, w=640, seed=0):
    """uint8 [n,3,h,w]: the decoded images (detect.py:57) of make_batch."""
    return torch.from_numpy(np.stack([make_scene(seed + i, h, w) for i in range(n)]))


def make_batch(n, h=640, w=640, seed=0):
    """float32 [n,3,h,w] in [0,1] (the detect.py:58 input contract)."""
    return make_batch_u8(n, h, w, seed).float() / 255


def make_dataset(img_dir, n, seed=0, label_dir=None, sizes=COCO_SIZES, ext=".png"):
    """Write n images named %012d<ext> (sizes cycled from a seeded draw) and YOLO labels."""
    from PIL import Image
    os.makedirs(img_dir, exist_ok=True)
    if label_dir:
        os.makedirs(label_dir, exist_ok=True)
    rs = np.random.RandomState(seed)
    names = []
    for i in range(n):
        h, w = sizes[rs.randint(len(sizes))]
        img, boxes = make_scene(seed * 100003 + i, h, w, return_boxes=True)
        name = f"{i:012d}"
        Image.fromarray(img.transpose(1, 2, 0)).save(os.path.join(img_dir, name + ext))
        if label_dir:
            with open(os.path.join(label_dir, name + ".txt"), "w") as f:
                for b in boxes:
                    f.write(" ".join(str(v) for v in b) + "\n")
        names.append(name)
    return names
