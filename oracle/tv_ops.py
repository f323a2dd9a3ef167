"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the torchvision detection ops used on the eval path of the models that
torch_models/detect.py:24,26,30,32 constructs.  torchvision itself is absent;
every function cites the SURVEY appendix line that restates the torchvision behaviour it follows.

Tie rules (implementation-defined in torchvision, fixed here and in the HIP kernels alike):
  * top-k and every score sort: descending score, ties -> lower index first (torchvision's CPU nms
    already sorts with ``stable=True``);
  * batched_nms: exact per-group NMS (torchvision's ``_batched_nms_vanilla`` semantics).  The
    coordinate-offset trick torchvision uses for <= 1000 CPU boxes is mathematically identical but
    rounds IoUs of offset coordinates; decisions can differ only for IoU within ~1e-5 of the threshold.
"""
import ctypes
import math
import os
import subprocess

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build_c(force=False):
    """Compile oracle/c/tvops_ref.c -> oracle/c/libtvops_ref.so (gcc, -ffp-contract=off)."""
    src = os.path.join(_HERE, "c", "tvops_ref.c")
    out = os.path.join(_HERE, "c", "libtvops_ref.so")
    if force or not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared", src, "-o", out, "-lm"])
    return out


def _lib():
    global _LIB
    if _LIB is None:
        lib = ctypes.CDLL(build_c())
        lib.nms_ref.restype = ctypes.c_int64
        lib.nms_ref.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
        lib.roi_align_ref.restype = None
        lib.roi_align_ref.argtypes = [ctypes.c_void_p] + [ctypes.c_int64] * 4 + [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _LIB = lib
    return _LIB


# ---------------------------------------------------------------- NMS (SURVEY A.0 "nms", "batched_nms")
def nms(boxes, scores, iou_threshold):
    """torchvision::nms CPU semantics.  boxes [n,4] float32 xyxy, scores [n]. Returns int64 indices."""
    b = np.ascontiguousarray(np.asarray(boxes, dtype=np.float32))
    s = np.ascontiguousarray(np.asarray(scores, dtype=np.float32))
    n = s.shape[0]
    keep = np.empty(max(n, 1), dtype=np.int64)
    k = _lib().nms_ref(b.ctypes.data, s.ctypes.data, n, float(iou_threshold), keep.ctypes.data)
    return keep[:k].copy()


def nms_numpy(boxes, scores, iou_threshold):
    """Pure-numpy greedy NMS (identical semantics); used to cross-check nms() on small cases."""
    b = np.asarray(boxes, dtype=np.float32)
    s = np.asarray(scores, dtype=np.float32)
    order = np.argsort(-s, kind="stable")
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    areas = (x2 - x1) * (y2 - y1)
    sup = np.zeros(len(s), dtype=bool)
    keep = []
    for ii in range(len(order)):
        i = order[ii]
        if sup[i]:
            continue
        keep.append(i)
        rest = order[ii + 1:]
        xx1 = np.maximum(x1[i], x1[rest])
        yy1 = np.maximum(y1[i], y1[rest])
        xx2 = np.minimum(x2[i], x2[rest])
        yy2 = np.minimum(y2[i], y2[rest])
        w = np.maximum(np.float32(0), xx2 - xx1)
        h = np.maximum(np.float32(0), yy2 - yy1)
        inter = w * h
        ovr = inter / ((areas[i] + areas[rest]) - inter)
        sup[rest[ovr.astype(np.float64) > iou_threshold]] = True
    return np.asarray(keep, dtype=np.int64)


def batched_nms(boxes, scores, idxs, iou_threshold):
    """Per-group NMS; result sorted by score descending, ties by lower index."""
    boxes = np.asarray(boxes, dtype=np.float32)
    scores = np.asarray(scores, dtype=np.float32)
    idxs = np.asarray(idxs)
    if scores.shape[0] == 0:
        return np.zeros((0,), dtype=np.int64)
    keep_mask = np.zeros(scores.shape[0], dtype=bool)
    for g in np.unique(idxs):
        cur = np.nonzero(idxs == g)[0]
        k = nms(boxes[cur], scores[cur], iou_threshold)
        keep_mask[cur[k]] = True
    keep = np.nonzero(keep_mask)[0]
    return keep[np.argsort(-scores[keep], kind="stable")]


def topk_stable(scores, k):
    """Top-k indices, descending, ties -> lower index (SURVEY A.0 "topk tie order")."""
    s = np.asarray(scores, dtype=np.float32)
    return np.argsort(-s, kind="stable")[:k]


# ---------------------------------------------------------------- boxes
def decode_boxes(rel_codes, boxes, weights, clip=math.log(1000.0 / 16)):
    """BoxCoder.decode_single.  rel_codes [n, 4*k], boxes [n,4] -> [n, k, 4] (torch float32 CPU)."""
    rel_codes = torch.as_tensor(rel_codes, dtype=torch.float32)
    boxes = torch.as_tensor(boxes, dtype=torch.float32)
    widths = boxes[:, 2] - boxes[:, 0]
    heights = boxes[:, 3] - boxes[:, 1]
    ctr_x = boxes[:, 0] + 0.5 * widths
    ctr_y = boxes[:, 1] + 0.5 * heights
    wx, wy, ww, wh = weights
    dx = rel_codes[:, 0::4] / wx
    dy = rel_codes[:, 1::4] / wy
    dw = rel_codes[:, 2::4] / ww
    dh = rel_codes[:, 3::4] / wh
    dw = torch.clamp(dw, max=clip)
    dh = torch.clamp(dh, max=clip)
    pcx = dx * widths[:, None] + ctr_x[:, None]
    pcy = dy * heights[:, None] + ctr_y[:, None]
    pw = torch.exp(dw) * widths[:, None]
    ph = torch.exp(dh) * heights[:, None]
    hh = torch.tensor(0.5, dtype=torch.float32) * ph
    hw = torch.tensor(0.5, dtype=torch.float32) * pw
    return torch.stack((pcx - hw, pcy - hh, pcx + hw, pcy + hh), dim=2)


def clip_boxes(boxes, size):
    h, w = size
    b = boxes.clone()
    b[..., 0::2] = b[..., 0::2].clamp(min=0, max=w)
    b[..., 1::2] = b[..., 1::2].clamp(min=0, max=h)
    return b


def remove_small(boxes, min_size):
    ws = boxes[:, 2] - boxes[:, 0]
    hs = boxes[:, 3] - boxes[:, 1]
    return torch.where((ws >= min_size) & (hs >= min_size))[0]


# ---------------------------------------------------------------- transform (SURVEY A.0 "Transform resize")
def resize_scale_f32(h, w, min_size, max_size):
    """[TV] `_resize_image_and_masks`: `scale = torch.min(800. / min_f32, 1333. / max_f32)` on float32
    tensors. `float / Tensor` is `Tensor.__rtruediv__` = `reciprocal(t) * other`, so
    each ratio is fp32(fp32(1/side) * size); `.item()` widens the smaller one to a Python double."""
    mn, mx = np.float32(min(h, w)), np.float32(max(h, w))
    a = np.float32(np.float32(1.0) / mn) * np.float32(min_size)
    b = np.float32(np.float32(1.0) / mx) * np.float32(max_size)
    return float(min(a, b))


def resize_output_size(h, w, min_size, max_size, fixed=None):
    """F.interpolate(scale_factor=s, recompute_scale_factor=True): size = floor(float(side) * s) in
    double, s the fp32 scale above."""
    if fixed is not None:
        return fixed
    scale = resize_scale_f32(h, w, min_size, max_size)
    return int(math.floor(h * scale)), int(math.floor(w * scale))


def transform(images, mean, std, min_size, max_size, fixed=None, divisible=1):
    """GeneralizedRCNNTransform eval: normalize -> bilinear resize -> zero-pad batch (NCHW torch)."""
    out, sizes = [], []
    for img in images:
        m = torch.as_tensor(mean, dtype=torch.float32)[:, None, None]
        s = torch.as_tensor(std, dtype=torch.float32)[:, None, None]
        x = (img - m) / s
        oh, ow = resize_output_size(x.shape[-2], x.shape[-1], min_size, max_size, fixed)
        x = F.interpolate(x[None], size=(oh, ow), mode="bilinear", align_corners=False)[0]
        out.append(x)
        sizes.append((oh, ow))
    mh = max(o.shape[-2] for o in out)
    mw = max(o.shape[-1] for o in out)
    mh = int(math.ceil(mh / divisible) * divisible)
    mw = int(math.ceil(mw / divisible) * divisible)
    batch = torch.zeros((len(out), out[0].shape[0], mh, mw), dtype=torch.float32)
    for i, o in enumerate(out):
        batch[i, :, :o.shape[-2], :o.shape[-1]] = o
    return batch, sizes


def rescale_boxes(boxes, resized, original):
    """transform.postprocess -> resize_boxes: ratios original/resized in float32."""
    rh = torch.tensor(original[0], dtype=torch.float32) / torch.tensor(resized[0], dtype=torch.float32)
    rw = torch.tensor(original[1], dtype=torch.float32) / torch.tensor(resized[1], dtype=torch.float32)
    return torch.stack((boxes[:, 0] * rw, boxes[:, 1] * rh, boxes[:, 2] * rw, boxes[:, 3] * rh), dim=1)


# ---------------------------------------------------------------- anchors
def ssd_default_boxes(grid_sizes, image_size=(320, 320), aspect_ratios=((2, 3),) * 6,
                      min_ratio=0.2, max_ratio=0.95):
    """DefaultBoxGenerator -> [A, 4] xyxy pixels, order (i, j, a)."""
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
        wh = torch.as_tensor(wh, dtype=torch.float32).clamp(min=0, max=1)
        sx = ((torch.arange(0, fw) + 0.5) / fw).to(torch.float32)
        sy = ((torch.arange(0, fh) + 0.5) / fh).to(torch.float32)
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        xx, yy = xx.reshape(-1), yy.reshape(-1)
        shifts = torch.stack((xx, yy) * len(wh), dim=-1).reshape(-1, 2)
        whr = wh.repeat(fh * fw, 1)
        out.append(torch.cat((shifts, whr), dim=1))
    d = torch.cat(out, 0)
    xy = torch.tensor([image_size[1], image_size[0]])
    return torch.cat([(d[:, :2] - 0.5 * d[:, 2:]) * xy, (d[:, :2] + 0.5 * d[:, 2:]) * xy], -1)


def rpn_cell_anchors(size, ratios=(0.5, 1.0, 2.0)):
    """AnchorGenerator.generate_anchors for one level; size = one scale or a
    tuple of scales (ratio-major, scale-minor order)."""
    scales = torch.as_tensor(size if isinstance(size, (tuple, list)) else [size], dtype=torch.float32)
    ar = torch.as_tensor(ratios, dtype=torch.float32)
    hr = torch.sqrt(ar)
    wr = 1 / hr
    ws = (wr[:, None] * scales[None, :]).view(-1)
    hs = (hr[:, None] * scales[None, :]).view(-1)
    return (torch.stack([-ws, -hs, ws, hs], dim=1) / 2).round()


def rpn_anchors(grid_sizes, image_size, sizes=(32, 64, 128, 256, 512)):
    out = []
    for (gh, gw), sz in zip(grid_sizes, sizes):
        sh, sw = image_size[0] // gh, image_size[1] // gw
        base = rpn_cell_anchors(sz)
        shx = torch.arange(0, gw, dtype=torch.int32) * sw
        shy = torch.arange(0, gh, dtype=torch.int32) * sh
        yy, xx = torch.meshgrid(shy, shx, indexing="ij")
        xx, yy = xx.reshape(-1), yy.reshape(-1)
        shifts = torch.stack((xx, yy, xx, yy), dim=1)
        out.append((shifts.view(-1, 1, 4) + base.view(1, -1, 4)).reshape(-1, 4))
    return out


RETINA_SIZES = tuple((x, int(x * 2 ** (1.0 / 3)), int(x * 2 ** (2.0 / 3))) for x in (32, 64, 128, 256, 512))


def retina_anchors(grid_sizes, image_size):
    """retinanet _default_anchorgen(): 3 sizes x 3 ratios per location, per level (P3..P7)."""
    return rpn_anchors(grid_sizes, image_size, sizes=RETINA_SIZES)


# ---------------------------------------------------------------- RoIAlign
def roi_align(feat, rois, scale, out=7, sampling_ratio=2):
    """feat [B,C,H,W] float32 torch; rois [R,5] (b, x1, y1, x2, y2) -> [R,C,out,out]."""
    f = np.ascontiguousarray(feat.numpy(), dtype=np.float32)
    r = np.ascontiguousarray(np.asarray(rois, dtype=np.float32))
    B, C, H, W = f.shape
    R = r.shape[0]
    o = np.zeros((R, C, out, out), dtype=np.float32)
    if R:
        _lib().roi_align_ref(f.ctypes.data, B, C, H, W, r.ctypes.data, R, float(scale), out, out,
                             sampling_ratio, o.ctypes.data)
    return torch.from_numpy(o)


def level_mapper(boxes, k_min=2, k_max=5, s0=224, lvl0=4, eps=1e-6):
    """LevelMapper: floor(lvl0 + log2(sqrt(area)/s0) + eps) clamped; returns 0-based level."""
    area = (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
    s = torch.sqrt(area)
    t = torch.floor(lvl0 + torch.log2(s / s0) + torch.tensor(eps, dtype=s.dtype))
    t = torch.clamp(t, min=k_min, max=k_max)
    return t.to(torch.int64) - k_min


def multiscale_roi_align(feats, boxes_per_image, scales):
    rois = torch.cat([torch.cat([torch.full((b.shape[0], 1), i, dtype=torch.float32), b], 1)
                      for i, b in enumerate(boxes_per_image)], 0)
    levels = level_mapper(torch.cat(boxes_per_image, 0))
    C = feats[0].shape[1]
    res = torch.zeros((rois.shape[0], C, 7, 7), dtype=torch.float32)
    for lvl, (f, sc) in enumerate(zip(feats, scales)):
        idx = torch.where(levels == lvl)[0]
        if idx.numel():
            res[idx] = roi_align(f, rois[idx], sc)
    return res
