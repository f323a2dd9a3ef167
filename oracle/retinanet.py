"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

CPU restatement of torchvision's ``retinanet_resnet50_fpn_v2`` eval forward, the third model of
torch_models/detect.py:34-38 (``--model`` other than ssd/faster_rcnn).  torchvision state_dict keys
(edgeml_amd.arch.retinanet_table, pinned by the published parameter count 38,198,935):
  * GeneralizedRCNNTransform: min 800, max 1333, ImageNet mean/std, pad to /32 (as FRCNN);
  * ResNet-50 body (BatchNorm2d eval) -> C3, C4, C5 (returned_layers [2, 3, 4]);
  * FPN without norm (1x1 / 3x3 convs with bias, nearest top-down), LastLevelP6P7(2048, 256):
    P6 = conv3x3 s2 on C5, P7 = conv3x3 s2 on relu(P6);
  * RetinaNetHead: per branch 4 x (conv3x3 no bias + GroupNorm(32, eps 1e-5) + ReLU), then
    cls_logits (9 x K) / bbox_reg (9 x 4) conv3x3 with bias; outputs (N, HWA, K) per level;
  * anchors: sizes (x, int(x 2^1/3), int(x 2^2/3)) for x in 32..512, ratios 0.5/1/2;
  * postprocess_detections: per level sigmoid, score > 0.05, topk(min(1000, n)) over the flattened
    (anchor, class) scores, decode (1,1,1,1), clip; then batched_nms(0.5) by label over all levels,
    [:300]; transform.postprocess rescale.
"""
import torch
import torch.nn.functional as F

from . import tv_ops
from .frcnn import MEAN, STD, MIN_SIZE, MAX_SIZE, DIVISIBLE, conv, resnet_body
from .ssdlite import _SD

SCORE_THRESH, NMS_THRESH, DETS, TOPK = 0.05, 0.5, 300, 1000
GN_GROUPS, GN_EPS = 32, 1e-5
A = 9


def fpn_p6p7(cs, sd):
    """C3..C5 -> P3..P7."""
    p = "backbone.fpn."
    c3, c4, c5 = cs
    last = conv(c5, sd, p + "inner_blocks.2.0", bias=True)
    res = [conv(last, sd, p + "layer_blocks.2.0", bias=True)]
    for i, c in ((1, c4), (0, c3)):
        lat = conv(c, sd, f"{p}inner_blocks.{i}.0", bias=True)
        last = lat + F.interpolate(last, size=lat.shape[-2:], mode="nearest")
        res.insert(0, conv(last, sd, f"{p}layer_blocks.{i}.0", bias=True))
    p6 = conv(c5, sd, p + "extra_blocks.p6", 2, bias=True)
    p7 = conv(F.relu(p6), sd, p + "extra_blocks.p7", 2, bias=True)
    return res + [p6, p7]


def head(feats, sd, num_classes):
    cls_all, reg_all = [], []
    for f in feats:
        outs = []
        for br, last, k in (("classification_head", "cls_logits", num_classes), ("regression_head", "bbox_reg", 4)):
            t = f
            for i in range(4):
                q = f"head.{br}.conv.{i}."
                t = conv(t, sd, q + "0")
                t = F.relu(F.group_norm(t, GN_GROUPS, sd[q + "1.weight"], sd[q + "1.bias"], GN_EPS))
            o = conv(t, sd, f"head.{br}.{last}", bias=True)
            N, _, H, W = o.shape
            outs.append(o.view(N, -1, k, H, W).permute(0, 3, 4, 1, 2).reshape(N, -1, k))
        cls_all.append(outs[0])
        reg_all.append(outs[1])
    return cls_all, reg_all


def postprocess(cls_all, reg_all, anchors, image_shapes):
    dets = []
    for n, shape in enumerate(image_shapes):
        bl, sl, ll = [], [], []
        for cl, rg, an in zip(cls_all, reg_all, anchors):
            K = cl.shape[-1]
            scores = torch.sigmoid(cl[n]).flatten()
            keep = torch.where(scores > SCORE_THRESH)[0]
            sc = scores[keep]
            k = min(TOPK, keep.numel())
            order = torch.from_numpy(tv_ops.topk_stable(sc.numpy(), k)).long()
            sc, idx = sc[order], keep[order]
            anchor_idx = torch.div(idx, K, rounding_mode="floor")
            labels = idx % K
            boxes = tv_ops.decode_boxes(rg[n][anchor_idx], an[anchor_idx], (1.0, 1.0, 1.0, 1.0))[:, 0]
            bl.append(tv_ops.clip_boxes(boxes, shape))
            sl.append(sc)
            ll.append(labels)
        boxes, scores, labels = torch.cat(bl), torch.cat(sl), torch.cat(ll)
        keep = torch.from_numpy(tv_ops.batched_nms(boxes.numpy(), scores.numpy(), labels.numpy(), NMS_THRESH))
        keep = keep[:DETS]
        dets.append({"boxes": boxes[keep], "scores": scores[keep], "labels": labels[keep]})
    return dets


class RetinaNetOracle:
    """Callable with the torchvision detection-model contract (detect.py:78)."""

    def __init__(self, state_dict, num_classes=91):
        self.sd = {k: v.detach().to(torch.float32) if v.is_floating_point() else v
                   for k, v in state_dict.items()}
        self.num_classes = num_classes

    @torch.no_grad()
    def forward_raw(self, images, hook=None):
        sd = _SD(self.sd)
        x, sizes = tv_ops.transform(list(images), MEAN, STD, MIN_SIZE, MAX_SIZE, divisible=DIVISIBLE)
        c2, c3, c4, c5 = resnet_body(x, sd, hook)
        feats = fpn_p6p7((c3, c4, c5), sd)
        cls_all, reg_all = head(feats, sd, self.num_classes)
        anchors = tv_ops.retina_anchors([f.shape[-2:] for f in feats], tuple(x.shape[-2:]))
        self.used_keys = sd.used
        return cls_all, reg_all, anchors, sizes, feats

    @torch.no_grad()
    def __call__(self, images):
        imgs = list(images)
        orig = [(int(i.shape[-2]), int(i.shape[-1])) for i in imgs]
        cls_all, reg_all, anchors, sizes, _ = self.forward_raw(imgs)
        dets = postprocess(cls_all, reg_all, anchors, sizes)
        for d, s, o in zip(dets, sizes, orig):
            d["boxes"] = tv_ops.rescale_boxes(d["boxes"], s, o)
        return dets
