"""Candidate sets and decision chains of the detectors' post-processing tails (test infrastructure).

Each builder turns one image's pre-decision values (class probabilities / logits and decoded,
clipped boxes) into a ``flips.Side`` whose candidate ids are the same on both sides, with the
order keys and tie rules of SURVEY.md App. A (the ones the oracle and the HIP kernels fix):
  SSDLite    id = (c-1)*A + a            oracle/ssdlite.py postprocess (App. A.1 step 7)
  RPN        id = level offset + a       oracle/frcnn.py rpn (App. A.2 step 4)
  FRCNN box  id = r*(NC-1) + (c-1)       oracle/frcnn.py box_postprocess (App. A.2 step 7)
  RetinaNet  id = level offset + a*K + k oracle/retinanet.py postprocess
"""
import numpy as np
import torch
import torch.nn.functional as F

from tests.flips import Side

SSD_STAGES = [("filter", "score", 0.001, ">"), ("topk", 300, "cls", "score", "anchor"), ("nms", 0.55, "cls"),
              ("cut", 300)]
RPN_STAGES = [("topk", 1000, "level", "logit", "anchor"), ("filter", "minsize", 1e-3, ">="),
              ("filter", "score", 0.0, ">="), ("nms", 0.7, "level"), ("cut", 1000)]
BOX_STAGES = [("filter", "score", 0.05, ">"), ("filter", "minsize", 1e-2, ">="), ("nms", 0.5, "cls"), ("cut", 100)]
RETINA_STAGES = [("filter", "score", 0.05, ">"), ("topk", 1000, "level", "score", "flat"), ("nms", 0.5, "cls"),
                 ("cut", 300)]


def _np32(x):
    return x.detach().cpu().numpy().astype(np.float32) if torch.is_tensor(x) else np.asarray(x, np.float32)


def _minsize(box):
    return np.minimum(box[:, 2] - box[:, 0], box[:, 3] - box[:, 1])


# ------------------------------------------------------------------------------ SSDLite
def ssd_side(scores_t, boxes):
    """scores_t [NC, A] class probabilities, boxes [A, 4] decoded + clipped (320x320 space)."""
    scores_t, boxes = _np32(scores_t), _np32(boxes)
    NC, A = scores_t.shape
    cls = np.repeat(np.arange(1, NC), A)
    anchor = np.tile(np.arange(A), NC - 1)
    score = scores_t[1:].reshape(-1)
    return Side(score, boxes[anchor], {"cls": cls}, q={"score": score}, ties=(cls, anchor), tkties={"anchor": anchor})


def ssd_label_of(A):
    return lambda ids: ids // A + 1


def ssd_oracle_inputs(cls_logits, bbox_reg, anchors):
    """The oracle's softmax / decode / clip (oracle/ssdlite.py postprocess) for one image."""
    from oracle import tv_ops
    scores = F.softmax(cls_logits, dim=-1)
    boxes = tv_ops.clip_boxes(tv_ops.decode_boxes(bbox_reg, anchors, (10.0, 10.0, 5.0, 5.0))[:, 0], (320, 320))
    return scores.t().contiguous(), boxes


# ------------------------------------------------------------------------------ RPN
def rpn_side(objs, dels, anchors, image_size):
    """objs[l] [A_l] logits, dels[l] [A_l, 4], anchors[l] [A_l, 4] for one image; image_size (h, w)."""
    from oracle import tv_ops
    logit = np.concatenate([_np32(o) for o in objs])
    level = np.concatenate([np.full(len(o), l) for l, o in enumerate(objs)])
    anchor = np.concatenate([np.arange(len(o)) for o in objs])
    d = torch.from_numpy(np.concatenate([_np32(x).reshape(-1, 4) for x in dels]))
    a = torch.from_numpy(np.concatenate([_np32(x).reshape(-1, 4) for x in anchors]))
    box = tv_ops.clip_boxes(tv_ops.decode_boxes(d, a, (1.0, 1.0, 1.0, 1.0))[:, 0], image_size).numpy()
    score = torch.sigmoid(torch.from_numpy(logit)).numpy()
    return Side(score, box, {"level": level}, q={"minsize": _minsize(box), "score": score}, keys={"logit": logit},
                ties=(level, -logit, anchor), tkties={"anchor": anchor})


# ------------------------------------------------------------------------------ FRCNN box stage
def box_side_from_values(scores, boxes):
    """scores [R, NC] probabilities, boxes [R, NC, 4] decoded + clipped, for one image's proposals."""
    scores, boxes = _np32(scores), _np32(boxes)
    R, NC = scores.shape
    score = scores[:, 1:].reshape(-1)
    box = boxes[:, 1:].reshape(-1, 4)
    flat = np.arange(R * (NC - 1))
    cls = flat % (NC - 1) + 1
    return Side(score, box, {"cls": cls}, q={"score": score, "minsize": _minsize(box)}, ties=(flat,))


def box_side(logits, deltas, proposals, image_size):
    """The oracle's softmax / decode / clip (oracle/frcnn.py box_postprocess) for one image."""
    from oracle import tv_ops
    scores = F.softmax(torch.as_tensor(logits), -1)
    boxes = tv_ops.clip_boxes(tv_ops.decode_boxes(torch.as_tensor(deltas), torch.as_tensor(proposals),
                                                  (10.0, 10.0, 5.0, 5.0)), image_size)
    return box_side_from_values(scores, boxes)


def box_label_of(NC):
    return lambda ids: ids % (NC - 1) + 1


# ------------------------------------------------------------------------------ RetinaNet
def retina_sides(cls_a, reg_a, cls_b, reg_b, anchors, image_size, thr=0.05):
    """Both sides of one image on the same candidate set: every (level, anchor, class) whose score
    passes `thr` on either side (all others are dropped by the first filter on both)."""
    from oracle import tv_ops
    sides_in = []
    offs, lv, fl, keep_all = 0, [], [], []
    sa = [torch.sigmoid(torch.as_tensor(c)).numpy().reshape(-1) for c in cls_a]
    sb = [torch.sigmoid(torch.as_tensor(c)).numpy().reshape(-1) for c in cls_b]
    K = cls_a[0].shape[-1]
    for l in range(len(cls_a)):
        idx = np.nonzero((sa[l] > thr) | (sb[l] > thr))[0]
        keep_all.append(idx)
        lv.append(np.full(len(idx), l))
        fl.append(idx)
    level, flat = np.concatenate(lv), np.concatenate(fl)
    for cls_all, reg_all, s in ((cls_a, reg_a, sa), (cls_b, reg_b, sb)):
        score = np.concatenate([s[l][keep_all[l]] for l in range(len(s))]).astype(np.float32)
        bl = []
        for l in range(len(s)):
            ai = keep_all[l] // K
            d = torch.as_tensor(reg_all[l]).reshape(-1, 4)[ai]
            bl.append(tv_ops.clip_boxes(tv_ops.decode_boxes(d, anchors[l][ai], (1.0, 1.0, 1.0, 1.0))[:, 0],
                                        image_size).numpy())
        box = np.concatenate(bl) if bl else np.zeros((0, 4), np.float32)
        cls = flat % K
        sides_in.append(Side(score, box, {"level": level, "cls": cls}, q={"score": score}, ties=(level, flat),
                             tkties={"flat": flat}))
    return sides_in[0], sides_in[1], (lambda ids: flat[ids] % K)
