"""The library's lowering (csrc/lower.hip, the only one: the Python model objects run its plans) against
independent host restatements, on the CPU:
  * weight packing (edgedet_model_pack): BatchNorm folding in float64, the (kh, kw, ci) K order padded
    to 32, the three bf16 planes, depthwise tap-major weights, FC6's (c, h, w) -> (h, w, c) permutation,
    the predictor's [bbox | cls] rows, GroupNorm affine parameters, at the offsets the records use;
  * plan constants (edgedet_model_prepare_host): the anchors against edgeml_amd.anchors (pinned to the
    oracle's generators in tests/test_host.py) and the rescale ratios;
  * state_dict validation.
tests/test_gpu_native_model.py runs the same plans through the pure C-ABI on the GPU.
"""
import numpy as np
import pytest
import torch

from edgeml_amd import anchors as anc
from edgeml_amd import models, native, ops, synthetic
from edgeml_amd.plan import fold_bn, pack_conv_weight, pack_dw_weight, split_bf16x3


@pytest.fixture(scope="module")
def built():
    cache = {}

    def get(kind, nc=91, rt=True):
        key = (kind, nc, rt)
        if key not in cache:
            sd = synthetic.synthetic_state_dict(kind, nc, rt, seed=3, calibrated=False)
            cls = {"ssd": models.SSDLite320, "faster_rcnn": models.FasterRCNNFPNv2,
                   "retinanet": models.RetinaNetFPNv2}[kind]
            m = cls(sd, nc, rt) if kind == "ssd" else cls(sd, nc)
            cache[key] = (sd, m)
        return cache[key]
    return get


def _np(t):
    return t.detach().cpu().to(torch.float64).numpy()


def _blob_f32(m, ptr, n):
    """n floats of the packed blob at a record's weight pointer (CPU plans point into the model's
    blob tensor)."""
    off = ptr - m.weights("cpu").data_ptr()
    assert off % 4 == 0 and 0 <= off < m.blob.size
    return m.blob[off:off + 4 * n].view(np.float32)


def _op(P, name):
    return next(op for op in P.ops if op.name == name)


def _check_conv(m, op, w_oihw, b, cin_pad=None):
    wp, K, Kpad, _ = pack_conv_weight(w_oihw, cin_pad)
    cout = wp.shape[0]
    assert op.i[12] == K and op.i[13] == Kpad
    np.testing.assert_array_equal(_blob_f32(m, op.p[1], cout * Kpad), wp.reshape(-1))
    np.testing.assert_array_equal(_blob_f32(m, op.p[2], cout), np.asarray(b, np.float32))
    planes = _blob_f32(m, op.p[6], (3 * cout * Kpad + 1) // 2).view(np.uint16)[:3 * cout * Kpad]
    np.testing.assert_array_equal(planes, split_bf16x3(wp).reshape(-1))


@pytest.mark.parametrize("rt", [True, False])
def test_ssd_packing_matches_restatement(built, rt):
    sd, m = built("ssd", 91 if rt else 21, rt)
    P = m.build_plan(2, 320, 320)
    s = lambda k: _np(sd[k])  # noqa: E731
    fb = lambda p: fold_bn(s(p + ".0.weight"), s(p + ".1.weight"), s(p + ".1.bias"),  # noqa: E731
                           s(p + ".1.running_mean"), s(p + ".1.running_var"), 1e-3)
    p = "backbone.features.0.4.block.0"  # expand 1x1 + BN (eps 1e-3)
    _check_conv(m, _op(P, p), *fb(p))
    p = "backbone.features.0.4.block.1"  # depthwise, tap-major
    w, b = fb(p)
    op = _op(P, p)
    np.testing.assert_array_equal(_blob_f32(m, op.p[1], w.size), pack_dw_weight(w).reshape(-1))
    np.testing.assert_array_equal(_blob_f32(m, op.p[2], b.size), b)
    # block 0.2 as one MBCONV record: expand [Cexp][i12], depthwise tap-major, project [Cout][i13]
    p = "backbone.features.0.2.block"
    op = _op(P, p)
    assert op.kind == ops.MBCONV
    (w1, b1), (wd, bd), (w2, b2) = fb(p + ".0"), fb(p + ".1"), fb(p + ".2")
    for (w, b), kw, kb, kld in (((w1, b1), 1, 2, 12), ((w2, b2), 5, 6, 13)):
        wp, _, Kpad, _ = pack_conv_weight(w)
        assert op.i[kld] == Kpad
        np.testing.assert_array_equal(_blob_f32(m, op.p[kw], wp.size), wp.reshape(-1))
        np.testing.assert_array_equal(_blob_f32(m, op.p[kb], b.size), b)
    np.testing.assert_array_equal(_blob_f32(m, op.p[3], wd.size), pack_dw_weight(wd).reshape(-1))
    np.testing.assert_array_equal(_blob_f32(m, op.p[4], bd.size), bd)
    p = "head.classification_head.module_list.0.1"  # 1x1 with bias, no BN
    _check_conv(m, _op(P, p), s(p + ".weight").astype(np.float32), s(p + ".bias"))
    p = "backbone.features.0.4.block.2"  # SqueezeExcitation: fc1 [S][C], fc2 transposed [S][C]
    op = _op(P, p)
    C, S = op.i[1], op.i[2]
    np.testing.assert_array_equal(_blob_f32(m, op.p[1], S * C), s(p + ".fc1.weight").astype(np.float32).reshape(-1))
    np.testing.assert_array_equal(_blob_f32(m, op.p[3], S * C),
                                  s(p + ".fc2.weight")[:, :, 0, 0].T.astype(np.float32).reshape(-1))


def test_frcnn_packing_matches_restatement(built):
    sd, m = built("faster_rcnn")
    P = m.build_plan(1, 480, 640)
    s = lambda k: _np(sd[k])  # noqa: E731
    q = "backbone.body."
    w, b = fold_bn(s(q + "conv1.weight"), s(q + "bn1.weight"), s(q + "bn1.bias"), s(q + "bn1.running_mean"),
                   s(q + "bn1.running_var"), 1e-5)
    _check_conv(m, _op(P, q + "conv1.weight"), w, b, cin_pad=4)
    w6 = s("roi_heads.box_head.5.weight").astype(np.float32).reshape(1024, 256, 7, 7).transpose(0, 2, 3, 1)
    _check_conv(m, _op(P, "roi_heads.box_head.5"), w6.reshape(1024, -1)[:, :, None, None],
                s("roi_heads.box_head.5.bias"))
    pr = "roi_heads.box_predictor."
    wp = np.concatenate([s(pr + "bbox_pred.weight"), s(pr + "cls_score.weight")], 0).astype(np.float32)
    bp = np.concatenate([s(pr + "bbox_pred.bias"), s(pr + "cls_score.bias")], 0)
    _check_conv(m, _op(P, "roi_heads.box_predictor"), wp[:, :, None, None], bp)


def test_retinanet_packing_matches_restatement(built):
    sd, m = built("retinanet")
    P = m.build_plan(1, 480, 640)
    s = lambda k: _np(sd[k])  # noqa: E731
    q = "head.classification_head.conv.0."
    _check_conv(m, _op(P, q + "0@0"), s(q + "0.weight").astype(np.float32), np.zeros(256))  # no bias
    gn = _op(P, q + "1@0")
    np.testing.assert_array_equal(_blob_f32(m, gn.p[1], 256), s(q + "1.weight").astype(np.float32))
    np.testing.assert_array_equal(_blob_f32(m, gn.p[2], 256), s(q + "1.bias").astype(np.float32))
    p = "backbone.fpn.extra_blocks.p7"
    op = _op(P, p + ".weight")
    assert op.i[24] == 1  # relu(P6) applied by P7's input load
    _check_conv(m, op, s(p + ".weight").astype(np.float32), s(p + ".bias"))


def _const(P, name):
    return P.buffer(name).tensor().numpy()


@pytest.mark.parametrize("B,H,W", [(2, 480, 640), (1, 427, 640)])
def test_plan_constants_match_restatement(built, B, H, W):
    _, ssd = built("ssd")
    P = ssd.build_plan(B, H, W)
    np.testing.assert_array_equal(_const(P, "anchors"), anc.ssd_default_boxes(ssd.grids, (320, 320)))
    np.testing.assert_array_equal(_const(P, "ratio"),
                                  np.tile(np.float32([np.float32(W) / np.float32(320), np.float32(H) / np.float32(320)]),
                                          (B, 1)))
    _, fr = built("faster_rcnn")
    P = fr.build_plan(B, H, W)
    Ho, Wo, Hp, Wp = P.resized
    assert (Ho, Wo) == fr.resized_size(H, W)
    grids = [tuple(f.shape[1:3]) for f in P.feats]
    for lvl, a in enumerate(anc.rpn_anchors(grids, (Hp, Wp))):
        np.testing.assert_array_equal(_const(P, f"rpn.anchors@{lvl}"), a)
    np.testing.assert_array_equal(_const(P, "ratio"), np.tile(np.float32([np.float32(W) / np.float32(Wo),
                                                                           np.float32(H) / np.float32(Ho)]), (B, 1)))
    _, rn = built("retinanet")
    P = rn.build_plan(B, H, W)
    _, _, Hp, Wp = P.resized
    na = P.level_anchors
    sel = next(op for op in P.ops if op.kind == ops.RETINA_SELECT)
    grids = []
    for lvl in range(len(na)):
        conv = _op(P, f"head.classification_head.cls_logits@{lvl}")
        grids.append((conv.i[4], conv.i[5]))
    assert [gh * gw * 9 for gh, gw in grids] == na and sel.i[2] == sum(na)
    np.testing.assert_array_equal(_const(P, "anchors"), np.concatenate(anc.retina_anchors(grids, (Hp, Wp)), 0))


def test_pack_rejects_bad_state_dict(built):
    sd, _ = built("ssd")
    bad = dict(sd)
    bad.pop("head.regression_head.module_list.5.1.bias")
    with pytest.raises(ops.EdgeDetError, match="missing parameter"):
        native.pack_state_dict("ssd", bad, 91, True)
    bad = dict(sd)
    bad["backbone.features.0.0.0.weight"] = torch.zeros(16, 3, 3, 2)
    with pytest.raises(ops.EdgeDetError, match="size mismatch"):
        native.pack_state_dict("ssd", bad, 91, True)


def test_fused_block_lowering(built, monkeypatch):
    """The whole-block MBCONV lowering (default; EDGEDET_MB_BLOCK=0 turns it off) replaces blocks 0.2
    and 0.3."""
    _, m = built("ssd")
    B, H, W = 5, 300, 400  # a shape no other test lowers (the library caches plans per shape)
    for v, n in (("1", 2), ("0", 0)):
        monkeypatch.setenv("EDGEDET_MB_BLOCK", v)
        native.release("ssd", B, H, W)
        P = m.build_plan(B, H, W)
        assert sum(op.kind == ops.MBCONV for op in P.ops) == n
    native.release("ssd", B, H, W)


def test_model_records_entry_resolves_external_pointers(built):
    """edgedet_model_records with caller-owned images / outputs (the graph-capture path of a foreign
    host): those records point there, every other pointer into the workspace or the weights."""
    _, m = built("faster_rcnn")
    B, H, W = 1, 480, 640
    ext = [0x10000000 * (k + 1) for k in range(5)]
    rec = native.records("faster_rcnn", B, H, W, 0x7000000000, 0x8000000000, 91, True, False, images=ext[0],
                         outputs=tuple(ext[1:]))
    P = m.build_plan(B, H, W)
    assert len(rec) == len(P.records) and (rec["kind"] == P.records["kind"]).all()
    assert ext[0] in set(int(v) for v in rec[0]["p"])
    merge = rec[-1]
    assert [int(merge["p"][j]) for j in (6, 7, 8, 9)] == [ext[2], ext[3], ext[4], ext[1]]
