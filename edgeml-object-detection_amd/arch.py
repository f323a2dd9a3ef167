"""Architecture tables for the two detectors on the hot path.

These are the torchvision ``state_dict`` layouts of the models constructed at
torch_models/detect.py:24/26 (``ssdlite320_mobilenet_v3_large``) and detect.py:30/32
(``fasterrcnn_resnet50_fpn_v2``), restated from SURVEY.md Appendix A so that a real torchvision
checkpoint passed through ``--model-path`` (detect.py:39-41) loads unchanged.

Only shapes and names live here; the HIP execution plan is in ``models.py``.
"""
from collections import OrderedDict


def make_divisible(v, divisor=8, min_value=None):
    """torchvision.models._utils._make_divisible."""
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


# (in, kernel, expanded, out, use_se, activation, stride) — SURVEY A.1 step 2
def mnv3_blocks(reduced_tail):
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


def block_prefixes(cnf, base):
    """Module prefixes of an InvertedResidual's (expand, depthwise, SE, project) sub-layers."""
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


class _Table:
    def __init__(self):
        self.t = OrderedDict()

    def conv(self, p, cout, cin, k, bias=False):
        self.t[p + ".weight"] = (cout, cin, k, k)
        if bias:
            self.t[p + ".bias"] = (cout,)

    def bn(self, p, c):
        self.t[p + ".weight"] = (c,)
        self.t[p + ".bias"] = (c,)
        self.t[p + ".running_mean"] = (c,)
        self.t[p + ".running_var"] = (c,)
        self.t[p + ".num_batches_tracked"] = ()

    def cna(self, p, cout, cin, k, groups=1):
        """Conv2dNormActivation: p.0 conv (no bias), p.1 BatchNorm2d."""
        self.conv(p + ".0", cout, cin // groups, k)
        self.bn(p + ".1", cout)

    def linear(self, p, cout, cin):
        self.t[p + ".weight"] = (cout, cin)
        self.t[p + ".bias"] = (cout,)


def ssdlite_feature_channels(reduced_tail):
    c4 = 80 if reduced_tail else 160
    return [672, 6 * c4, 512, 256, 256, 128]


def ssdlite_table(num_classes=91, reduced_tail=True):
    """state_dict (name -> shape) of ssdlite320_mobilenet_v3_large."""
    T = _Table()
    cfg = mnv3_blocks(reduced_tail)
    T.cna("backbone.features.0.0", 16, 3, 3)

    def ir(cnf, base):
        cin, k, exp, cout, se, act, stride = cnf
        pe, pd, ps, pp = block_prefixes(cnf, base)
        if pe:
            T.cna(pe, exp, cin, 1)
        T.cna(pd, exp, exp, k, groups=exp)
        if ps:
            sq = make_divisible(exp // 4, 8)
            T.conv(ps + ".fc1", sq, exp, 1, bias=True)
            T.conv(ps + ".fc2", exp, sq, 1, bias=True)
        T.cna(pp, cout, exp, 1)

    for i in range(12):
        ir(cfg[i], f"backbone.features.0.{i + 1}.block")
    cin, k, exp, cout, se, act, stride = cfg[12]
    T.cna("backbone.features.0.13", exp, cin, 1)
    T.cna("backbone.features.1.0.1", exp, exp, k, groups=exp)
    sq = make_divisible(exp // 4, 8)
    T.conv("backbone.features.1.0.2.fc1", sq, exp, 1, bias=True)
    T.conv("backbone.features.1.0.2.fc2", exp, sq, 1, bias=True)
    T.cna("backbone.features.1.0.3", cout, exp, 1)
    for i in (13, 14):
        ir(cfg[i], f"backbone.features.1.{i - 12}.block")
    c4 = cfg[14][3]
    T.cna("backbone.features.1.3", 6 * c4, c4, 1)
    prev = 6 * c4
    for e, out in enumerate((512, 256, 256, 128)):
        mid = out // 2
        T.cna(f"backbone.extra.{e}.0", mid, prev, 1)
        T.cna(f"backbone.extra.{e}.1", mid, mid, 3, groups=mid)
        T.cna(f"backbone.extra.{e}.2", out, mid, 1)
        prev = out
    for name, cols in (("classification_head", num_classes), ("regression_head", 4)):
        for i, c in enumerate(ssdlite_feature_channels(reduced_tail)):
            p = f"head.{name}.module_list.{i}"
            T.cna(p + ".0", c, c, 3, groups=c)
            T.conv(p + ".1", 6 * cols, c, 1, bias=True)
    return T.t


RESNET_LAYERS = (("layer1", 3, 64, 1), ("layer2", 4, 128, 2), ("layer3", 6, 256, 2), ("layer4", 3, 512, 2))


def frcnn_table(num_classes=91):
    """state_dict (name -> shape) of fasterrcnn_resnet50_fpn_v2 (IntermediateLayerGetter drops avgpool/fc)."""
    T = _Table()
    p = "backbone.body."
    T.conv(p + "conv1", 64, 3, 7)
    T.bn(p + "bn1", 64)
    inplanes = 64
    for name, nblk, width, stride in RESNET_LAYERS:
        for b in range(nblk):
            q = f"{p}{name}.{b}."
            T.conv(q + "conv1", width, inplanes, 1)
            T.bn(q + "bn1", width)
            T.conv(q + "conv2", width, width, 3)
            T.bn(q + "bn2", width)
            T.conv(q + "conv3", width * 4, width, 1)
            T.bn(q + "bn3", width * 4)
            if b == 0:
                T.conv(q + "downsample.0", width * 4, inplanes, 1)
                T.bn(q + "downsample.1", width * 4)
            inplanes = width * 4
    for i, c in enumerate((256, 512, 1024, 2048)):
        T.cna(f"backbone.fpn.inner_blocks.{i}", 256, c, 1)
        T.cna(f"backbone.fpn.layer_blocks.{i}", 256, 256, 3)
    T.conv("rpn.head.conv.0.0", 256, 256, 3, bias=True)
    T.conv("rpn.head.conv.1.0", 256, 256, 3, bias=True)
    T.conv("rpn.head.cls_logits", 3, 256, 1, bias=True)
    T.conv("rpn.head.bbox_pred", 12, 256, 1, bias=True)
    for i in range(4):
        T.cna(f"roi_heads.box_head.{i}", 256, 256, 3)
    T.linear("roi_heads.box_head.5", 1024, 256 * 7 * 7)
    T.linear("roi_heads.box_predictor.cls_score", num_classes, 1024)
    T.linear("roi_heads.box_predictor.bbox_pred", num_classes * 4, 1024)
    return T.t


RETINA_ANCHORS = 9  # 3 sizes x 3 aspect ratios per location (_default_anchorgen)


def resnet50_body(T, p="backbone.body."):
    """ResNet-50 v1.5 without avgpool/fc (IntermediateLayerGetter), BatchNorm2d."""
    T.conv(p + "conv1", 64, 3, 7)
    T.bn(p + "bn1", 64)
    inplanes = 64
    for name, nblk, width, stride in RESNET_LAYERS:
        for b in range(nblk):
            q = f"{p}{name}.{b}."
            T.conv(q + "conv1", width, inplanes, 1)
            T.bn(q + "bn1", width)
            T.conv(q + "conv2", width, width, 3)
            T.bn(q + "bn2", width)
            T.conv(q + "conv3", width * 4, width, 1)
            T.bn(q + "bn3", width * 4)
            if b == 0:
                T.conv(q + "downsample.0", width * 4, inplanes, 1)
                T.bn(q + "downsample.1", width * 4)
            inplanes = width * 4


def retinanet_table(num_classes=91):
    """state_dict (name -> shape) of retinanet_resnet50_fpn_v2 (detect.py:34-38): ResNet-50 body,
    FPN over C3..C5 without norm (convs with bias) + LastLevelP6P7(2048, 256) (P6 from C5),
    RetinaNetHead with GroupNorm(32) towers (4 x conv3x3 no bias + GN + ReLU) per branch."""
    T = _Table()
    resnet50_body(T)
    for i, c in enumerate((512, 1024, 2048)):
        T.conv(f"backbone.fpn.inner_blocks.{i}.0", 256, c, 1, bias=True)
        T.conv(f"backbone.fpn.layer_blocks.{i}.0", 256, 256, 3, bias=True)
    T.conv("backbone.fpn.extra_blocks.p6", 256, 2048, 3, bias=True)
    T.conv("backbone.fpn.extra_blocks.p7", 256, 256, 3, bias=True)
    for br, out, last in (("classification_head", RETINA_ANCHORS * num_classes, "cls_logits"),
                          ("regression_head", RETINA_ANCHORS * 4, "bbox_reg")):
        for i in range(4):
            T.conv(f"head.{br}.conv.{i}.0", 256, 256, 3)
            T.t[f"head.{br}.conv.{i}.1.weight"] = (256,)  # GroupNorm(32, 256)
            T.t[f"head.{br}.conv.{i}.1.bias"] = (256,)
        T.conv(f"head.{br}.{last}", out, 256, 3, bias=True)
    return T.t


def param_count(table):
    """Learnable parameters (what torchvision's model cards count): excludes BN buffers."""
    n = 0
    for k, s in table.items():
        if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
            continue
        c = 1
        for d in s:
            c *= d
        n += c
    return n
