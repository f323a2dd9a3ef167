"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

CPU restatement of torchvision's ``fasterrcnn_resnet50_fpn_v2`` eval forward, the strong detector
built at torch_models/detect.py:30 (COCO weights) / detect.py:32 (--model-path).  Architecture per
SURVEY.md Appendix A.2; torchvision state_dict keys.
"""
import torch
import torch.nn.functional as F

from . import tv_ops
from .ssdlite import _SD

BN_EPS = 1e-5
MEAN = [0.485, 0.456, 0.406]
STD = [0.229, 0.224, 0.225]
MIN_SIZE, MAX_SIZE, DIVISIBLE = 800, 1333, 32
RPN_PRE_NMS, RPN_POST_NMS, RPN_NMS, RPN_MIN_SIZE, RPN_SCORE = 1000, 1000, 0.7, 1e-3, 0.0
BOX_SCORE, BOX_NMS, BOX_DETS, BOX_MIN_SIZE = 0.05, 0.5, 100, 1e-2
LAYERS = (("layer1", 3, 64, 1), ("layer2", 4, 128, 2), ("layer3", 6, 256, 2), ("layer4", 3, 512, 2))


def bn(x, sd, p, hook=None):
    if hook is not None:
        hook(p, x)
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, BN_EPS)


def conv(x, sd, p, stride=1, bias=False):
    w = sd[p + ".weight"]
    k = w.shape[-1]
    return F.conv2d(x, w, sd[p + ".bias"] if bias else None, stride, (k - 1) // 2)


def resnet_body(x, sd, hook=None):
    """ResNet-50 v1.5 -> C2..C5."""
    p = "backbone.body."
    x = F.relu(bn(conv(x, sd, p + "conv1", 2), sd, p + "bn1", hook))
    x = F.max_pool2d(x, 3, 2, 1)
    outs = []
    for name, nblk, width, stride in LAYERS:
        for b in range(nblk):
            q = f"{p}{name}.{b}."
            s = stride if b == 0 else 1
            y = F.relu(bn(conv(x, sd, q + "conv1"), sd, q + "bn1", hook))
            y = F.relu(bn(conv(y, sd, q + "conv2", s), sd, q + "bn2", hook))
            y = bn(conv(y, sd, q + "conv3"), sd, q + "bn3", hook)
            if b == 0:
                idn = bn(conv(x, sd, q + "downsample.0", s), sd, q + "downsample.1", hook)
            else:
                idn = x
            x = F.relu(y + idn)
        outs.append(x)
    return outs


def fpn(cs, sd, hook=None):
    """FeaturePyramidNetwork with BN + LastLevelMaxPool -> P2..P6."""
    p = "backbone.fpn."

    def inner(i, t):
        return bn(conv(t, sd, f"{p}inner_blocks.{i}.0"), sd, f"{p}inner_blocks.{i}.1", hook)

    def layer(i, t):
        return bn(conv(t, sd, f"{p}layer_blocks.{i}.0"), sd, f"{p}layer_blocks.{i}.1", hook)

    last = inner(3, cs[3])
    res = [layer(3, last)]
    for i in (2, 1, 0):
        lat = inner(i, cs[i])
        td = F.interpolate(last, size=lat.shape[-2:], mode="nearest")
        last = lat + td
        res.insert(0, layer(i, last))
    res.append(F.max_pool2d(res[-1], 1, 2, 0))
    return res


def rpn_head(feats, sd, padded_size):
    """RPNHead over every level + AnchorGenerator: per level objectness logits
    [N, H*W*A], deltas [N, H*W*A, 4] in (y, x, a) order, and the level's anchors."""
    p = "rpn.head."
    objs, dels = [], []
    for f in feats:
        t = F.relu(conv(f, sd, p + "conv.0.0", bias=True))
        t = F.relu(conv(t, sd, p + "conv.1.0", bias=True))
        o = conv(t, sd, p + "cls_logits", bias=True)
        d = conv(t, sd, p + "bbox_pred", bias=True)
        N, A, H, W = o.shape
        objs.append(o.view(N, A, 1, H, W).permute(0, 3, 4, 1, 2).reshape(N, -1))
        dels.append(d.view(N, A, 4, H, W).permute(0, 3, 4, 1, 2).reshape(N, -1, 4))
    anchors = tv_ops.rpn_anchors([f.shape[-2:] for f in feats], padded_size)
    return objs, dels, anchors


def rpn(feats, sd, image_shapes, padded_size):
    """RegionProposalNetwork eval -> list of [<=1000, 4] proposals."""
    return rpn_filter(*rpn_head(feats, sd, padded_size), image_shapes)


def rpn_filter(objs, dels, anchors, image_shapes):
    """RegionProposalNetwork.filter_proposals over the head outputs of rpn_head."""
    out = []
    for n in range(objs[0].shape[0]):
        bl, sl, ll = [], [], []
        for lvl, (o, d, a) in enumerate(zip(objs, dels, anchors)):
            k = min(RPN_PRE_NMS, o.shape[1])
            idx = torch.from_numpy(tv_ops.topk_stable(o[n].numpy(), k))
            boxes = tv_ops.decode_boxes(d[n][idx], a[idx], (1.0, 1.0, 1.0, 1.0))[:, 0]
            bl.append(boxes)
            sl.append(torch.sigmoid(o[n][idx]))
            ll.append(torch.full((k,), lvl, dtype=torch.int64))
        boxes, scores, lvls = torch.cat(bl), torch.cat(sl), torch.cat(ll)
        boxes = tv_ops.clip_boxes(boxes, image_shapes[n])
        keep = tv_ops.remove_small(boxes, RPN_MIN_SIZE)
        boxes, scores, lvls = boxes[keep], scores[keep], lvls[keep]
        keep = torch.where(scores >= RPN_SCORE)[0]
        boxes, scores, lvls = boxes[keep], scores[keep], lvls[keep]
        keep = torch.from_numpy(tv_ops.batched_nms(boxes.numpy(), scores.numpy(), lvls.numpy(), RPN_NMS))
        keep = keep[:RPN_POST_NMS]
        out.append(boxes[keep])
    return out


def box_head(x, sd, hook=None):
    """FastRCNNConvFCHead + FastRCNNPredictor."""
    p = "roi_heads.box_head."
    for i in range(4):
        x = F.relu(bn(conv(x, sd, f"{p}{i}.0"), sd, f"{p}{i}.1", hook))
    x = x.flatten(1)
    x = F.relu(F.linear(x, sd[p + "5.weight"], sd[p + "5.bias"]))
    q = "roi_heads.box_predictor."
    return (F.linear(x, sd[q + "cls_score.weight"], sd[q + "cls_score.bias"]),
            F.linear(x, sd[q + "bbox_pred.weight"], sd[q + "bbox_pred.bias"]))


def box_postprocess(logits, deltas, proposals, image_shapes):
    """RoIHeads.postprocess_detections."""
    dets = []
    counts = [p.shape[0] for p in proposals]
    boxes_all = tv_ops.decode_boxes(deltas, torch.cat(proposals), (10.0, 10.0, 5.0, 5.0))
    scores_all = F.softmax(logits, -1)
    nc = logits.shape[-1]
    for boxes, scores, shape in zip(boxes_all.split(counts), scores_all.split(counts), image_shapes):
        boxes = tv_ops.clip_boxes(boxes, shape)
        labels = torch.arange(nc).view(1, -1).expand_as(scores)
        boxes, scores, labels = boxes[:, 1:].reshape(-1, 4), scores[:, 1:].reshape(-1), labels[:, 1:].reshape(-1)
        inds = torch.where(scores > BOX_SCORE)[0]
        boxes, scores, labels = boxes[inds], scores[inds], labels[inds]
        keep = tv_ops.remove_small(boxes, BOX_MIN_SIZE)
        boxes, scores, labels = boxes[keep], scores[keep], labels[keep]
        keep = torch.from_numpy(tv_ops.batched_nms(boxes.numpy(), scores.numpy(), labels.numpy(), BOX_NMS))
        keep = keep[:BOX_DETS]
        dets.append({"boxes": boxes[keep], "scores": scores[keep], "labels": labels[keep]})
    return dets


class FasterRCNNOracle:
    """Callable with the torchvision detection-model contract (detect.py:78)."""

    def __init__(self, state_dict, num_classes=91, dtype=torch.float32):
        """dtype=torch.float64: the dense arithmetic (ResNet body, FPN, RPN head, box head and
        predictor: every conv / linear, BatchNorm and activation) runs in float64, the ground truth
        of bench.py's ORIE leg.  The transform, the proposal filter, MultiScaleRoIAlign (on the FPN
        features rounded to float32) and the post-processing stay float32 as in the reference, on
        float32-rounded inputs."""
        self.dtype = dtype
        self.sd = {k: v.detach().to(dtype) if v.is_floating_point() else v
                   for k, v in state_dict.items()}
        self.num_classes = num_classes

    @torch.no_grad()
    def forward_raw(self, images, hook=None):
        sd = _SD(self.sd)
        x, sizes = tv_ops.transform(list(images), MEAN, STD, MIN_SIZE, MAX_SIZE, divisible=DIVISIBLE)
        feats = fpn(resnet_body(x.to(self.dtype), sd, hook), sd, hook)
        objs, dels, anchors = rpn_head(feats, sd, tuple(x.shape[-2:]))
        objs, dels = [o.to(torch.float32) for o in objs], [d.to(torch.float32) for d in dels]
        self.last_rpn = (objs, dels, anchors)  # the proposal filter's inputs (end-to-end parity tests)
        props = rpn_filter(objs, dels, anchors, sizes)
        logits, deltas = self.box_stage(feats, props, sizes, hook, sd)
        self.used_keys = sd.used
        return logits, deltas, props, sizes, feats

    @torch.no_grad()
    def box_stage(self, feats, props, sizes, hook=None, sd=None):
        """MultiScaleRoIAlign + box head + predictor over given proposals (a list of [R_i, 4])."""
        sd = _SD(self.sd) if sd is None else sd
        mh = max(s[0] for s in sizes)
        scales = [2.0 ** round(float(torch.tensor(f.shape[-2] / mh).log2())) for f in feats[:4]]
        roi = tv_ops.multiscale_roi_align([f.to(torch.float32) for f in feats[:4]], props, scales)
        if hook is not None:
            hook("__roi_features__", roi)
        logits, deltas = box_head(roi.to(self.dtype), sd, hook)
        return logits.to(torch.float32), deltas.to(torch.float32)

    @torch.no_grad()
    def rpn_raw(self, feats, padded_size):
        """The RPN head outputs and anchors the proposal filter consumes (see rpn_head)."""
        return rpn_head(feats, _SD(self.sd), padded_size)

    @torch.no_grad()
    def __call__(self, images):
        imgs = list(images)
        orig = [(int(i.shape[-2]), int(i.shape[-1])) for i in imgs]
        logits, deltas, props, sizes, _ = self.forward_raw(imgs)
        dets = box_postprocess(logits, deltas, props, sizes)
        for d, s, o in zip(dets, sizes, orig):
            d["boxes"] = tv_ops.rescale_boxes(d["boxes"], s, o)
        return dets
