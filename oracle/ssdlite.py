"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

CPU restatement (PyTorch-CPU functional ops + oracle.tv_ops) of torchvision's
``ssdlite320_mobilenet_v3_large`` eval forward, the weak detector built at
torch_models/detect.py:24 (reduced tail, COCO weights) and detect.py:26 (full tail, --model-path).
Architecture per SURVEY.md Appendix A.1; state_dict keys are torchvision's, so a real checkpoint
loads unchanged.
"""
import torch
import torch.nn.functional as F

from . import tv_ops

BN_EPS = 1e-3
SCORE_THRESH = 0.001
NMS_THRESH = 0.55
DETS_PER_IMG = 300
TOPK_CANDIDATES = 300
SIZE = (320, 320)


def mnv3_config(reduced_tail):
    """(in, kernel, expanded, out, use_se, activation, stride) — SURVEY A.1 step 2."""
    c4 = 80 if reduced_tail else 160
    e4 = 480 if reduced_tail else 960
    return [
        (16, 3, 16, 16, False, "RE", 1), (16, 3, 64, 24, False, "RE", 2),
        (24, 3, 72, 24, False, "RE", 1), (24, 5, 72, 40, True, "RE", 2),
        (40, 5, 120, 40, True, "RE", 1), (40, 5, 120, 40, True, "RE", 1),
        (40, 3, 240, 80, False, "HS", 2), (80, 3, 200, 80, False, "HS", 1),
        (80, 3, 184, 80, False, "HS", 1), (80, 3, 184, 80, False, "HS", 1),
        (80, 3, 480, 112, True, "HS", 1), (112, 3, 672, 112, True, "HS", 1),
        (112, 5, 672, c4, True, "HS", 2), (c4, 5, e4, c4, True, "HS", 1),
        (c4, 5, e4, c4, True, "HS", 1),
    ]


def _act(x, kind):
    if kind == "RE":
        return F.relu(x)
    if kind == "HS":
        return F.hardswish(x)
    if kind == "R6":
        return F.relu6(x)
    return x


class _SD:
    """state_dict view that records which keys were read (tests assert full coverage)."""

    def __init__(self, sd):
        self.sd = sd
        self.used = set()

    def __getitem__(self, k):
        self.used.add(k)
        return self.sd[k]


def conv_bn(x, sd, p, stride=1, groups=1, act=None, hook=None, eps=BN_EPS):
    """Conv2dNormActivation: conv (no bias) -> BN(eval) -> act.  p = module prefix."""
    w = sd[p + ".0.weight"]
    k = w.shape[-1]
    x = F.conv2d(x, w, None, stride, (k - 1) // 2, 1, groups)
    if hook is not None:
        hook(p + ".1", x)
    x = F.batch_norm(x, sd[p + ".1.running_mean"], sd[p + ".1.running_var"], sd[p + ".1.weight"],
                     sd[p + ".1.bias"], False, 0.0, eps)
    return _act(x, act)


def squeeze_excite(x, sd, p):
    s = F.adaptive_avg_pool2d(x, 1)
    s = F.relu(F.conv2d(s, sd[p + ".fc1.weight"], sd[p + ".fc1.bias"]))
    s = F.hardsigmoid(F.conv2d(s, sd[p + ".fc2.weight"], sd[p + ".fc2.bias"]))
    return s * x


def inverted_residual(x, sd, cnf, prefixes, hook=None):
    """InvertedResidual; prefixes = (expand|None, dw, se|None, project) module prefixes."""
    cin, k, exp, cout, se, act, stride = cnf
    pe, pd, ps, pp = prefixes
    y = x
    if exp != cin:
        y = conv_bn(y, sd, pe, act=act, hook=hook)
    y = conv_bn(y, sd, pd, stride=stride, groups=exp, act=act, hook=hook)
    if se:
        y = squeeze_excite(y, sd, ps)
    y = conv_bn(y, sd, pp, act=None, hook=hook)
    if stride == 1 and cin == cout:
        y = y + x
    return y


def _block_prefixes(cnf, base):
    cin, k, exp, cout, se, act, stride = cnf
    j = 0
    pe = None
    if exp != cin:
        pe = f"{base}.{j}"
        j += 1
    pd = f"{base}.{j}"
    j += 1
    ps = None
    if se:
        ps = f"{base}.{j}"
        j += 1
    return pe, pd, ps, f"{base}.{j}"


def backbone(x, sd, reduced_tail, hook=None):
    """SSDLiteFeatureExtractorMobileNet -> 6 feature maps."""
    cfg = mnv3_config(reduced_tail)
    feats = []
    x = conv_bn(x, sd, "backbone.features.0.0", stride=2, act="HS", hook=hook)
    for i in range(12):
        x = inverted_residual(x, sd, cfg[i], _block_prefixes(cfg[i], f"backbone.features.0.{i + 1}.block"), hook)
    # C4 block split at its expansion conv (map0 = expansion output, 672 ch, stride 16)
    cin, k, exp, cout, se, act, stride = cfg[12]
    x = conv_bn(x, sd, "backbone.features.0.13", act=act, hook=hook)
    feats.append(x)
    y = conv_bn(x, sd, "backbone.features.1.0.1", stride=stride, groups=exp, act=act, hook=hook)
    y = squeeze_excite(y, sd, "backbone.features.1.0.2")
    x = conv_bn(y, sd, "backbone.features.1.0.3", act=None, hook=hook)
    for i in (13, 14):
        x = inverted_residual(x, sd, cfg[i], _block_prefixes(cfg[i], f"backbone.features.1.{i - 12}.block"), hook)
    x = conv_bn(x, sd, "backbone.features.1.3", act="HS", hook=hook)
    feats.append(x)
    for e in range(4):
        p = f"backbone.extra.{e}"
        x = conv_bn(x, sd, p + ".0", act="R6", hook=hook)
        x = conv_bn(x, sd, p + ".1", stride=2, groups=x.shape[1], act="R6", hook=hook)
        x = conv_bn(x, sd, p + ".2", act="R6", hook=hook)
        feats.append(x)
    return feats


def head(feats, sd, num_classes, hook=None):
    """SSDLiteHead -> cls_logits [N, A, K], bbox_regression [N, A, 4]."""
    outs = {}
    for name, cols in (("classification_head", num_classes), ("regression_head", 4)):
        res = []
        for i, f in enumerate(feats):
            p = f"head.{name}.module_list.{i}"
            y = conv_bn(f, sd, p + ".0", groups=f.shape[1], act="R6", hook=hook)
            y = F.conv2d(y, sd[p + ".1.weight"], sd[p + ".1.bias"])
            N, _, H, W = y.shape
            y = y.view(N, -1, cols, H, W).permute(0, 3, 4, 1, 2).reshape(N, -1, cols)
            res.append(y)
        outs[name] = torch.cat(res, 1)
    return outs["classification_head"], outs["regression_head"]


def postprocess(cls_logits, bbox_reg, anchors, num_classes):
    """SSD.postprocess_detections, boxes still in 320x320 space."""
    dets = []
    scores_all = F.softmax(cls_logits, dim=-1)
    for reg, scores in zip(bbox_reg, scores_all):
        boxes = tv_ops.decode_boxes(reg, anchors, (10.0, 10.0, 5.0, 5.0))[:, 0]
        boxes = tv_ops.clip_boxes(boxes, SIZE)
        ib, isc, il = [], [], []
        for label in range(1, num_classes):
            s = scores[:, label]
            keep = torch.where(s > SCORE_THRESH)[0]
            s = s[keep]
            b = boxes[keep]
            k = min(TOPK_CANDIDATES, s.shape[0])
            order = torch.from_numpy(tv_ops.topk_stable(s.numpy(), k))
            ib.append(b[order])
            isc.append(s[order])
            il.append(torch.full((k,), label, dtype=torch.int64))
        ib, isc, il = torch.cat(ib), torch.cat(isc), torch.cat(il)
        keep = torch.from_numpy(tv_ops.batched_nms(ib.numpy(), isc.numpy(), il.numpy(), NMS_THRESH))
        keep = keep[:DETS_PER_IMG]
        dets.append({"boxes": ib[keep], "scores": isc[keep], "labels": il[keep]})
    return dets


class SSDLiteOracle:
    """Callable with the torchvision detection-model contract (detect.py:78)."""

    def __init__(self, state_dict, num_classes=91, reduced_tail=None, dtype=torch.float32):
        """dtype=torch.float64: the convolutions, BatchNorm, activations and SE of the backbone and
        head run in float64 (the higher-precision ground truth of bench.py's ORIE leg); the
        transform before them and the post-processing after them stay float32 as in the reference,
        on the head outputs rounded to float32."""
        self.dtype = dtype
        self.sd = {k: v.detach().to(dtype) if v.is_floating_point() else v
                   for k, v in state_dict.items()}
        if reduced_tail is None:
            reduced_tail = self.sd["backbone.features.1.3.0.weight"].shape[1] == 80
        self.reduced_tail = reduced_tail
        self.num_classes = num_classes
        self.anchors = None

    @torch.no_grad()
    def forward_raw(self, images, hook=None):
        """images: list/tensor of [3,H,W] float32 in [0,1] -> (cls_logits, bbox_reg, sizes)."""
        sd = _SD(self.sd)
        x, sizes = tv_ops.transform(list(images), [0.5] * 3, [0.5] * 3, 320, 320, fixed=SIZE)
        feats = backbone(x.to(self.dtype), sd, self.reduced_tail, hook)
        cls, reg = head(feats, sd, self.num_classes, hook)
        cls, reg = cls.to(torch.float32), reg.to(torch.float32)
        if self.anchors is None:
            self.anchors = tv_ops.ssd_default_boxes([f.shape[-2:] for f in feats], SIZE)
        self.used_keys = sd.used
        return cls, reg, feats

    @torch.no_grad()
    def __call__(self, images):
        imgs = list(images)
        orig = [(int(i.shape[-2]), int(i.shape[-1])) for i in imgs]
        cls, reg, _ = self.forward_raw(imgs)
        dets = postprocess(cls, reg, self.anchors, self.num_classes)
        for d, o in zip(dets, orig):
            d["boxes"] = tv_ops.rescale_boxes(d["boxes"], SIZE, o)
        return dets
