"""Anchor tables (host constants, computed once per plan and uploaded into the plan arena).

Float32 restatements of torchvision's generators, bit-for-bit (checked against the oracle in
tests/test_host.py):
  * SSD ``DefaultBoxGenerator([[2, 3]] * 6, min_ratio=0.2, max_ratio=0.95)`` for
    ``ssdlite320_mobilenet_v3_large`` (detect.py:24,26);
  * RPN ``AnchorGenerator(sizes=((32,), (64,), (128,), (256,), (512,)), ratios=(0.5, 1.0, 2.0))``
    for ``fasterrcnn_resnet50_fpn_v2`` (detect.py:30,32; App. A.2 step 4).
"""
import math

import numpy as np

f32 = np.float32


def ssd_default_boxes(grid_sizes, image_size=(320, 320), aspect_ratios=((2, 3),) * 6, min_ratio=0.2,
                      max_ratio=0.95):
    """[A, 4] xyxy pixels, order (map, i, j, a)."""
    n = len(aspect_ratios)
    scales = [min_ratio + (max_ratio - min_ratio) * k / (n - 1.0) for k in range(n)] + [1.0]
    out = []
    for k, (fh, fw) in enumerate(grid_sizes):
        sk = scales[k]
        spk = math.sqrt(scales[k] * scales[k + 1])
        wh = [[sk, sk], [spk, spk]]
        for ar in aspect_ratios[k]:
            sq = math.sqrt(ar)
            wh.extend([[sk * sq, sk / sq], [sk / sq, sk * sq]])
        wh = np.clip(np.asarray(wh, dtype=f32), f32(0), f32(1))
        sx = (np.arange(fw, dtype=f32) + f32(0.5)) / f32(fw)
        sy = (np.arange(fh, dtype=f32) + f32(0.5)) / f32(fh)
        yy, xx = np.meshgrid(sy, sx, indexing="ij")
        xy = np.stack([xx.reshape(-1), yy.reshape(-1)], 1)          # [HW, 2]
        cxy = np.repeat(xy, len(wh), axis=0)                          # [HW*A, 2]
        whr = np.tile(wh, (fh * fw, 1))
        out.append(np.concatenate([cxy, whr], 1))
    d = np.concatenate(out, 0).astype(f32)
    size = np.asarray([image_size[1], image_size[0]], dtype=f32)
    half = f32(0.5) * d[:, 2:]
    return np.concatenate([(d[:, :2] - half) * size, (d[:, :2] + half) * size], 1).astype(f32)


def rpn_cell_anchors(size, ratios=(0.5, 1.0, 2.0)):
    """AnchorGenerator.generate_anchors: one scale, or a tuple of scales (ratio-major order)."""
    scales = np.asarray(size if isinstance(size, (tuple, list)) else [size], dtype=f32)
    ar = np.asarray(ratios, dtype=f32)
    hr = np.sqrt(ar).astype(f32)
    wr = (f32(1) / hr).astype(f32)
    ws = (wr[:, None] * scales[None, :]).reshape(-1).astype(f32)
    hs = (hr[:, None] * scales[None, :]).reshape(-1).astype(f32)
    base = np.stack([-ws, -hs, ws, hs], 1) / f32(2)
    return np.round(base).astype(f32)  # round-half-even, as torch.round


def rpn_anchors(grid_sizes, image_size, sizes=(32, 64, 128, 256, 512)):
    """Per level [gh*gw*3, 4] anchors, order (y, x, a); strides = image_size // grid."""
    out = []
    for (gh, gw), sz in zip(grid_sizes, sizes):
        sh, sw = image_size[0] // gh, image_size[1] // gw
        base = rpn_cell_anchors(sz)
        shx = np.arange(gw, dtype=np.int64) * sw
        shy = np.arange(gh, dtype=np.int64) * sh
        yy, xx = np.meshgrid(shy, shx, indexing="ij")
        xx, yy = xx.reshape(-1), yy.reshape(-1)
        shifts = np.stack([xx, yy, xx, yy], 1).astype(f32)
        out.append((shifts[:, None, :] + base[None, :, :]).reshape(-1, 4).astype(f32))
    return out


# retinanet _default_anchorgen(): sizes (x, int(x * 2^(1/3)), int(x * 2^(2/3))) per level, 3 ratios
RETINA_SIZES = tuple((x, int(x * 2 ** (1.0 / 3)), int(x * 2 ** (2.0 / 3))) for x in (32, 64, 128, 256, 512))


def retina_anchors(grid_sizes, image_size):
    """Per level [gh*gw*9, 4] anchors of retinanet_resnet50_fpn_v2 (P3..P7), order (y, x, a)."""
    return rpn_anchors(grid_sizes, image_size, sizes=RETINA_SIZES)
