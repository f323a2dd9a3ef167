"""GPU unit parity: each libedgedet kernel against an fp32 CPU reference of the same op.

Conv / depthwise: torch fp32 CPU conv2d (NCHW) of the same folded weights (float tolerance).
RoIAlign / NMS: the oracle's C restatement of torchvision's CPU kernels (oracle/c/tvops_ref.c);
NMS indices must match exactly, RoIAlign values bit-for-bit (same op order, no contraction).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _act(y, act):
    return {None: y, "RE": F.relu(y), "R6": F.relu6(y), "HS": F.hardswish(y)}[act]


CONV_CASES = [
    (2, 17, 19, 4, 16, 3, 2, "HS", False),      # SSD stem shape class (Cin padded to 4)
    (2, 20, 20, 112, 672, 1, 1, "HS", False),   # expansion 1x1
    (3, 10, 10, 480, 80, 1, 1, None, True),     # projection with residual
    (1, 25, 23, 64, 64, 3, 1, "RE", False),     # ResNet 3x3
    (1, 26, 26, 128, 256, 3, 2, "RE", True),    # strided 3x3 + residual
    (1, 40, 36, 4, 64, 7, 2, "RE", False),      # ResNet stem 7x7 (Cin padded to 4)
    (2, 7, 7, 256, 24, 1, 1, None, False),      # narrow Cout
    (4, 1, 1, 1024, 455, 1, 1, None, False),    # FC as 1x1 (predictor shape)
    (2, 33, 31, 24, 72, 1, 1, "RE", False),     # K=24 (one partial K stage)
    (1, 9, 9, 16, 16, 1, 1, None, True),        # K=16 with residual
]


def _conv_case(B, H, W, Cin, Cout, k, s, act, res, tile=0, se=False, x6=False):
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    sc = torch.rand(B, Cin, generator=g) if se else None
    pad = (k - 1) // 2
    xin = x * sc[:, :, None, None] if se else x
    ref = F.conv2d(xin, w, b, s, pad)
    r = torch.randn_like(ref) if res else None
    if res:
        ref = ref + r
    ref = _act(ref, act)
    wp, K, Kpad, _ = pack_conv_weight(w.numpy())
    wdev = torch.from_numpy(wp).to(DEV)
    w3 = ops.split_bf16x3(wdev) if x6 else None
    out = ops.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV), wdev, b.to(DEV), Cout,
                          k, s, pad, act, r.permute(0, 2, 3, 1).contiguous().to(DEV) if res else None, tile=tile,
                          in_scale=sc.to(DEV) if se else None, w3=w3)
    got = out.permute(0, 3, 1, 2).cpu()
    err = (got - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_matches_torch(case):
    _conv_case(*case)


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("case", [CONV_CASES[i] for i in (1, 2, 4, 5, 8)])
def test_conv_every_lds_tile(case, tile):
    _conv_case(*case, tile=tile)


@pytest.mark.parametrize("tile", [10, 11, 12, 13, 14, 15, 16, 17])
@pytest.mark.parametrize("case", [(2, 20, 20, 112, 672, 1, 1, "HS", False), (3, 10, 10, 40, 120, 1, 1, None, True),
                                  (2, 33, 31, 24, 72, 1, 1, "RE", False), (1, 9, 9, 16, 16, 1, 1, None, True),
                                  (2, 13, 11, 96, 24, 1, 1, "R6", False), (2, 20, 20, 672, 24, 1, 1, None, False),
                                  (3, 10, 10, 480, 80, 1, 1, None, True), (2, 5, 5, 512, 546, 1, 1, None, False),
                                  (1, 3, 3, 1000, 36, 1, 1, "HS", False)])
@pytest.mark.parametrize("se", [False, True])
def test_conv_direct_pointwise(case, tile, se):
    _conv_case(*case, tile=tile, se=se)


@pytest.mark.parametrize("tile", [33, 34, 35])
@pytest.mark.parametrize("case", [(2, 33, 31, 24, 72, 1, 1, "RE", False), (1, 9, 9, 16, 16, 1, 1, None, True),
                                  (2, 13, 11, 64, 24, 1, 1, "R6", False), (3, 20, 20, 72, 24, 1, 1, None, True),
                                  (2, 17, 19, 16, 64, 1, 1, "HS", False), (2, 10, 10, 72, 40, 1, 1, None, False),
                                  (1, 7, 7, 40, 96, 1, 1, "RE", True), (2, 40, 40, 20, 36, 1, 1, "HS", False)])
@pytest.mark.parametrize("se", [False, True])
def test_conv_pointwise_stream(case, tile, se):
    """Tiles 33-35, the streaming 1x1 kernel of the narrow SSDLite layers (exact fp32 MFMA, 8-deep K
    chunks, weights in registers): ragged row blocks, a Cin that is not a multiple of 8, residual,
    SE input scale, Cout not a multiple of 32."""
    _conv_case(*case, tile=tile, se=se)


def test_conv_pointwise_stream_refuses_wide():
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    x = torch.randn(1, 4, 4, 480, device=DEV)
    wp = torch.from_numpy(pack_conv_weight(torch.randn(128, 480, 1, 1).numpy())[0]).to(DEV)
    with pytest.raises(ops.EdgeDetError):
        ops.conv2d_nhwc(x, wp, torch.zeros(128, device=DEV), 128, 1, 1, 0, None, tile=33)


@pytest.mark.parametrize("B,H,W,C,k,s,act", [(2, 20, 20, 72, 5, 2, "RE"), (3, 10, 10, 672, 5, 1, "HS"),
                                              (2, 3, 3, 128, 3, 2, "R6"), (1, 40, 40, 64, 3, 1, "RE"),
                                              (2, 13, 7, 16, 3, 2, "RE"), (1, 1, 1, 480, 3, 2, "HS"),
                                              (2, 9, 11, 40, 5, 2, "HS"), (1, 160, 160, 16, 3, 1, "RE"),
                                              (2, 6, 9, 8, 3, 1, None), (1, 7, 5, 12, 7, 2, "RE")])
def test_dwconv_matches_torch(B, H, W, C, k, s, act):
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_dw_weight
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(C, 1, k, k, generator=g) / k
    b = torch.randn(C, generator=g) * 0.1
    ref = _act(F.conv2d(x, w, b, s, (k - 1) // 2, 1, C), act)
    out = ops.dwconv2d_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV), torch.from_numpy(pack_dw_weight(w.numpy())).to(DEV),
                            b.to(DEV), k, s, (k - 1) // 2, act)
    err = (out.permute(0, 3, 1, 2).cpu() - ref).abs().max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("B,H,W,C,k,s,act", [(2, 40, 40, 72, 5, 2, "RE"), (3, 10, 10, 672, 5, 1, "HS"),
                                              (2, 20, 20, 120, 5, 1, "RE"), (1, 5, 5, 960, 5, 1, "HS"),
                                              (2, 13, 7, 40, 3, 2, "HS"), (1, 2, 2, 24, 5, 1, "RE"),
                                              (33, 3, 3, 8, 7, 1, "RE")])
def test_dwconv_se_partial_sums(B, H, W, C, k, s, act):
    """Fused depthwise + SE squeeze: the output matches torch and the partial sums add up to the
    per-channel spatial sum of that output."""
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_dw_weight
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(C, 1, k, k, generator=g) / k
    b = torch.randn(C, generator=g) * 0.1
    ref = _act(F.conv2d(x, w, b, s, (k - 1) // 2, 1, C), act)
    y, part = ops.dwconv2d_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV),
                                torch.from_numpy(pack_dw_weight(w.numpy())).to(DEV), b.to(DEV), k, s, (k - 1) // 2,
                                act, se_part=True)
    assert (y.permute(0, 3, 1, 2).cpu() - ref).abs().max().item() < 1e-5
    tot = part.sum(1).cpu()
    assert torch.allclose(tot, ref.sum((2, 3)), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("B,H,W", [(2, 320, 320), (1, 37, 50), (3, 2, 3), (1, 33, 31)])
def test_ssd_stem_matches_torch(B, H, W):
    """SSDLite features.0.0 + features.0.1 fused (csrc/layers.hip ssd_stem_kernel) against torch fp32:
    hardswish(conv3x3 s2) -> relu(depthwise 3x3) -> 1x1 projection + residual."""
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight, pack_dw_weight
    g = torch.Generator().manual_seed(H * W + B)
    x = torch.randn(B, 3, H, W, generator=g)
    w0 = torch.randn(16, 3, 3, 3, generator=g) / 27 ** 0.5
    b0 = torch.randn(16, generator=g) * 0.1
    wd = torch.randn(16, 1, 3, 3, generator=g) / 3
    bd = torch.randn(16, generator=g) * 0.1
    w1 = torch.randn(16, 16, 1, 1, generator=g) / 4
    b1 = torch.randn(16, generator=g) * 0.1
    s = F.hardswish(F.conv2d(x, w0, b0, 2, 1))
    ref = F.conv2d(F.relu(F.conv2d(s, wd, bd, 1, 1, 1, 16)), w1, b1) + s
    x4 = torch.cat([x, torch.zeros(B, 1, H, W)], 1).permute(0, 2, 3, 1).contiguous()
    dev = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    got = ops.ssd_stem_nhwc(x4.to(DEV), dev(pack_conv_weight(w0.numpy(), 4)[0]), b0.to(DEV),
                            dev(pack_dw_weight(wd.numpy())), bd.to(DEV), dev(pack_conv_weight(w1.numpy())[0]),
                            b1.to(DEV))
    err = (got.permute(0, 3, 1, 2).cpu() - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("H0,W0,u8", [(640, 640, True), (480, 640, True), (427, 640, False), (37, 29, True)])
def test_ssd_stem_folded_transform_bit_identical(H0, W0, u8):
    """The SSD stem with the transform folded into its input loads (SSD_STEM record with a source image,
    the plans' default) equals the transform record followed by the stem on its NHWC4 output, bit for
    bit, for uint8 and float sources and resize ratios above and below 1."""
    import ctypes
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight, pack_dw_weight
    B, S = 3, 320
    g = torch.Generator().manual_seed(H0 + W0)
    img8 = torch.randint(0, 256, (B, 3, H0, W0), generator=g, dtype=torch.uint8)
    src = (img8 if u8 else img8.float() / 255).to(DEV)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    w0p, _, ld0, _ = pack_conv_weight((torch.randn(16, 3, 3, 3, generator=g) / 5).numpy(), 4)
    w1p, _, ld1, _ = pack_conv_weight((torch.randn(16, 16, 1, 1, generator=g) / 4).numpy())
    wts = [dev(w0p), torch.randn(16, generator=g).to(DEV) * 0.1, dev(pack_dw_weight((torch.randn(16, 1, 3, 3, generator=g) / 3).numpy())),
           torch.randn(16, generator=g).to(DEV) * 0.1, dev(w1p), torch.randn(16, generator=g).to(DEV) * 0.1]
    x4 = torch.full((B, S, S, 4), float("nan"), device=DEV)
    Ho = (S - 1) // 2 + 1
    outs = [torch.full((B, Ho, Ho, 16), float("nan"), device=DEV) for _ in range(2)]
    rec = np.zeros(3, dtype=ops.OP_DTYPE)
    rec[0]["kind"] = ops.PREPROCESS
    rec[0]["i"][:7] = [B, H0, W0, S, S, S, S]
    rec[0]["p"][2 if u8 else 0] = src.data_ptr()
    rec[0]["p"][1] = x4.data_ptr()
    rec[0]["f"][:6] = 0.5
    for k, fused in ((1, False), (2, True)):
        rec[k]["kind"] = ops.SSD_STEM
        rec[k]["i"][:9] = [B, S, S, Ho, Ho, ld0, ld1, H0 if fused else 0, W0 if fused else 0]
        if fused:
            rec[k]["p"][9 if u8 else 8] = src.data_ptr()
            rec[k]["f"][:6] = 0.5
        else:
            rec[k]["p"][0] = x4.data_ptr()
        for j, t in enumerate(wts):
            rec[k]["p"][1 + j] = t.data_ptr()
        rec[k]["p"][7] = outs[k - 1].data_ptr()
    ops.check(ops.lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 3, ops.stream_handle()))
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])
    if u8:  # the uint8 source (each tap's x / 255 and (v - mean) / std by layers.hip div_fast, checked
        # exact on every uint8 operand) equals the host's float image / 255
        srcf = (img8.float() / 255).to(DEV)
        outf = torch.full_like(outs[1], float("nan"))
        rf = rec[2:3].copy()
        rf[0]["p"][9] = 0
        rf[0]["p"][8] = srcf.data_ptr()
        rf[0]["p"][7] = outf.data_ptr()
        ops.check(ops.lib().edgedet_plan_run(rf.ctypes.data_as(ctypes.c_void_p), 1, ops.stream_handle()))
        torch.cuda.synchronize()
        assert torch.equal(outf, outs[1])


@pytest.mark.parametrize("H0,W0", [(640, 640), (480, 640), (375, 500), (427, 640), (800, 1202)])
def test_transform_u8_equals_float_image(H0, W0):
    """The transform record on the decoded uint8 image (each tap's divisions by div_fast on the device,
    bit-identical to the IEEE divisions on every uint8 operand: tests/test_fast_div.py) equals the
    transform of the host's float image / 255 (detect.py:58) bit for bit, with the FRCNN / RetinaNet
    ImageNet normalisation (divisions that are not exact) and the SSD one; and both equal the CPU
    oracle's GeneralizedRCNNTransform arithmetic (normalise, then F.interpolate bilinear on the CPU,
    oracle/tv_ops.transform) bit for bit, up- and downscaling."""
    import ctypes
    from edgeml_amd import ops
    B = 2
    g = torch.Generator().manual_seed(H0 * 7 + W0)
    img8 = torch.randint(0, 256, (B, 3, H0, W0), generator=g, dtype=torch.uint8)
    Ho, Wo = (H0 * 2 // 3, W0 * 2 // 3) if H0 > 700 else (H0 + 37, W0 + 41)
    for norm in ([0.485, 0.456, 0.406, 0.229, 0.224, 0.225], [0.5] * 6):
        outs = []
        for u8 in (True, False):
            src = (img8 if u8 else img8.float() / 255).to(DEV)
            x4 = torch.full((B, Ho, Wo, 4), float("nan"), device=DEV)
            rec = np.zeros(1, dtype=ops.OP_DTYPE)
            rec[0]["kind"] = ops.PREPROCESS
            rec[0]["i"][:7] = [B, H0, W0, Ho, Wo, Ho, Wo]
            rec[0]["p"][2 if u8 else 0] = src.data_ptr()
            rec[0]["p"][1] = x4.data_ptr()
            rec[0]["f"][:6] = norm
            ops.check(ops.lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, ops.stream_handle()))
            torch.cuda.synchronize()
            outs.append(x4.cpu())
        assert torch.isfinite(outs[0]).all()
        assert torch.equal(outs[0], outs[1]), (norm, int((outs[0] != outs[1]).sum()))
        m = torch.tensor(norm[:3])[:, None, None]
        sd = torch.tensor(norm[3:])[:, None, None]
        ref = F.interpolate((img8.float() / 255 - m) / sd, size=(Ho, Wo), mode="bilinear", align_corners=False)
        got = outs[1][..., :3].permute(0, 3, 1, 2)
        assert torch.equal(got, ref), (norm, int((got != ref).sum()), float((got - ref).abs().max()))


@pytest.mark.parametrize("B,C,S,parts", [(1, 72, 24, 16), (32, 960, 240, 1), (7, 120, 32, 5), (64, 672, 168, 2),
                                          (33, 480, 120, 16), (16, 672, 168, 6), (3, 1000, 248, 3)])
def test_se_excitation_matches_torch(B, C, S, parts):
    """SE avgpool (from `parts` partial sums) -> fc1 -> ReLU -> fc2 -> Hardsigmoid against torch fp32."""
    from edgeml_amd import ops
    g = torch.Generator().manual_seed(B + C)
    hw = 37
    part = torch.randn(B, parts, C, generator=g) * 3
    w1 = torch.randn(S, C, generator=g) / C ** 0.5
    b1 = torch.randn(S, generator=g) * 0.1
    w2 = torch.randn(C, S, generator=g) / S ** 0.5
    b2 = torch.randn(C, generator=g) * 0.1
    mean = part.sum(1) / hw
    ref = F.hardsigmoid(F.linear(F.relu(F.linear(mean, w1, b1)), w2, b2))
    got = ops.se_excitation(part.to(DEV), hw, w1.to(DEV), b1.to(DEV), w2.t().contiguous().to(DEV), b2.to(DEV))
    assert (got.cpu() - ref).abs().max().item() < 1e-5


def _rand_boxes(rs, n, scale=100.0):
    xy = rs.uniform(0, scale, (n, 2)).astype(np.float32)
    wh = rs.uniform(1, scale / 3, (n, 2)).astype(np.float32)
    return np.concatenate([xy, xy + wh], 1).astype(np.float32)


@pytest.mark.parametrize("n,thr,seed", [(0, 0.5, 0), (1, 0.5, 0), (37, 0.5, 1), (300, 0.55, 2), (1000, 0.7, 3),
                                        (1024, 0.3, 4)])
def test_nms_matches_oracle(n, thr, seed):
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(seed)
    boxes = _rand_boxes(rs, n)
    scores = rs.uniform(0, 1, n).astype(np.float32)
    if n > 10:
        scores[5:10] = scores[0]  # ties
    ref = tv_ops.nms(boxes, scores, thr) if n else np.zeros(0, np.int64)
    got = ops.nms(torch.from_numpy(boxes).to(DEV), torch.from_numpy(scores).to(DEV), thr).cpu().numpy()
    np.testing.assert_array_equal(got, ref)


def test_batched_nms_matches_oracle():
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(5)
    n = 800
    boxes = _rand_boxes(rs, n, 60.0)
    scores = rs.uniform(0, 1, n).astype(np.float32)
    idxs = rs.randint(0, 7, n).astype(np.int64)
    ref = tv_ops.batched_nms(boxes, scores, idxs, 0.5)
    got = ops.batched_nms(torch.from_numpy(boxes).to(DEV), torch.from_numpy(scores).to(DEV),
                          torch.from_numpy(idxs).to(DEV), 0.5).cpu().numpy()
    np.testing.assert_array_equal(got, ref)


def test_roi_align_matches_oracle():
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(6)
    B, C, H, W = 2, 32, 25, 31
    feat = torch.from_numpy(rs.randn(B, C, H, W).astype(np.float32))
    R = 64
    bx = _rand_boxes(rs, R, 120.0)
    bx[:4] = [[-10, -10, 5, 5], [0, 0, 1, 1], [100, 90, 130, 140], [50, 50, 50.5, 50.2]]
    rois = np.concatenate([rs.randint(0, B, (R, 1)).astype(np.float32), bx], 1).astype(np.float32)
    ref = tv_ops.roi_align(feat, rois, 0.25)
    got = ops.roi_align_nhwc(feat.permute(0, 2, 3, 1).contiguous().to(DEV), torch.from_numpy(rois).to(DEV), 0.25)
    got = got.permute(0, 3, 1, 2).cpu()
    assert torch.equal(got, ref), (got - ref).abs().max().item()


@pytest.mark.parametrize("thr", [0.5, 0.55, 0.7, 0.3, 1.0 / 3.0])
def test_nms_exact_ratio_boundaries(thr):
    """Integer-coordinate boxes make IoUs hit exact ratios (1/2, 7/10, 11/20, ...) on the threshold:
    the engine's division-free IoU test must decide exactly like the reference's float division."""
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(int(thr * 1000))
    n = 600
    xy = rs.randint(0, 12, (n, 2)).astype(np.float32)
    wh = rs.randint(1, 10, (n, 2)).astype(np.float32)
    boxes = np.concatenate([xy, xy + wh], 1).astype(np.float32)
    scores = rs.permutation(n).astype(np.float32) / n
    ref = tv_ops.nms(boxes, scores, thr)
    got = ops.nms(torch.from_numpy(boxes).to(DEV), torch.from_numpy(scores).to(DEV), thr).cpu().numpy()
    np.testing.assert_array_equal(got, ref)


# ---- bf16x6: the fp32 GEMM as six bf16 partial products (csrc/conv.hip conv_x6_kernel)
def test_split_bf16x3_device_matches_host():
    from edgeml_amd import ops
    from edgeml_amd.plan import split_bf16x3
    g = torch.Generator().manual_seed(3)
    w = torch.cat([torch.randn(40025, generator=g) * 10 ** torch.randint(-6, 4, (40025,), generator=g),
                   torch.tensor([0.0, -0.0, 1.0, -1.0, 3.0e38, 1e-38, 65504.0])]).reshape(139, 288)  # Kpad 288
    got = ops.split_bf16x3(w.to(DEV)).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, split_bf16x3(w.numpy()))


@pytest.mark.parametrize("tile", [0, 22, 23, 24, 25, 27, 28, 29, 30, 31, 32, 38, 39])
@pytest.mark.parametrize("case", [CONV_CASES[i] for i in (0, 1, 2, 3, 4, 5, 7, 8)])
def test_conv_bf16x6_matches_torch(case, tile):
    _conv_case(*case, tile=tile, x6=True)


@pytest.mark.parametrize("se", [False, True])
@pytest.mark.parametrize("case", [CONV_CASES[i] for i in (2, 3, 4, 7)] + [(2, 7, 7, 256, 200, 3, 1, "RE", False)])
def test_conv_bf16x6_presplit_bit_identical(case, se):
    """Tile 25 with the input split up front (split_act_kernel into the x3 scratch, SE scale applied
    there) equals the in-loop split bit for bit, and both match torch."""
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    B, H, W, Cin, Cout, k, s, act, res = case
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, H, W, Cin, generator=g).to(DEV)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = (torch.randn(Cout, generator=g) * 0.1).to(DEV)
    sc = torch.rand(B, Cin, generator=g).to(DEV) if se else None
    Ho, Wo = (H + 2 * ((k - 1) // 2) - k) // s + 1, (W + 2 * ((k - 1) // 2) - k) // s + 1
    r = torch.randn(B, Ho, Wo, Cout, generator=g).to(DEV) if res else None
    wp = torch.from_numpy(pack_conv_weight(w.numpy())[0]).to(DEV)
    w3 = ops.split_bf16x3(wp)
    outs = [ops.conv2d_nhwc(x, wp, b, Cout, k, s, (k - 1) // 2, act, r, tile=25, in_scale=sc, w3=w3, presplit=ps)
            for ps in (False, True)]
    assert torch.equal(outs[0], outs[1])
    xin = x.permute(0, 3, 1, 2).cpu() * (sc.cpu()[:, :, None, None] if se else 1)
    ref = F.conv2d(xin, w, b.cpu(), s, (k - 1) // 2)
    if res:
        ref = ref + r.permute(0, 3, 1, 2).cpu()
    ref = _act(ref, act)
    err = (outs[1].permute(0, 3, 1, 2).cpu() - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("case", [CONV_CASES[6], CONV_CASES[7], (2, 20, 20, 672, 546, 1, 1, None, False),
                                  (3, 10, 10, 480, 546, 1, 1, None, False), (1, 9, 9, 64, 64, 3, 1, None, False)])
def test_conv_bf16x6_split_k(case):
    """Tile 26: the 256 x 128 bf16x6 tile with K in two halves added into a zeroed output (the first
    half adds the bias).  Matches torch, and two runs are bit-identical (a + b == b + a)."""
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    _conv_case(*case, tile=26, x6=True)
    B, H, W, Cin, Cout, k, s, act, res = case
    g = torch.Generator().manual_seed(9)
    x = torch.randn(B, H, W, Cin, generator=g).to(DEV)
    wp = torch.from_numpy(pack_conv_weight(torch.randn(Cout, Cin, k, k, generator=g).numpy())[0]).to(DEV)
    w3 = ops.split_bf16x3(wp)
    b = torch.randn(Cout, generator=g).to(DEV)
    y1, y2 = (ops.conv2d_nhwc(x, wp, b, Cout, k, s, (k - 1) // 2, None, tile=26, w3=w3) for _ in range(2))
    assert torch.equal(y1, y2)


@pytest.mark.parametrize("tile", [25, 29, 30, 31, 32, 38, 39])
@pytest.mark.parametrize("se", [False, True])
@pytest.mark.parametrize("case", [(2, 9, 9, 16, 16, 1, 1, None, True), (3, 11, 7, 24, 72, 1, 1, "HS", False),
                                  (2, 13, 10, 40, 120, 1, 1, "RE", False), (1, 20, 20, 72, 24, 1, 1, None, True)])
def test_conv_bf16x6_pointwise_ragged_cin(case, se, tile):
    """The pointwise x6b form with Cin not a multiple of 32: the chunks past Cin are zeroed (and load
    from a safe address: past the last pixel they would leave the buffer), with and without the SE
    input scale."""
    _conv_case(*case, tile=tile, se=se, x6=True)


@pytest.mark.parametrize("tile", [22, 23, 24, 25, 29, 30, 31, 32, 38, 39])
def test_conv_bf16x6_se_scale(tile):
    _conv_case(2, 10, 10, 480, 160, 1, 1, None, True, tile=tile, se=True, x6=True)


@pytest.mark.parametrize("shape", [(2, 25, 25, 256, 256, 3), (1, 13, 13, 1024, 512, 1), (1, 50, 50, 64, 128, 7)])
def test_conv_bf16x6_is_fp32_grade(shape):
    """Against a float64 reference the bf16x6 conv errs no more than the exact-fp32 MFMA conv (x1.5):
    the three dropped partial products sit below one fp32 rounding of each product."""
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    B, H, W, Cin, Cout, k = shape
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.zeros(Cout)
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, (k - 1) // 2)
    wp = torch.from_numpy(pack_conv_weight(w.numpy())[0]).to(DEV)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    errs = {}
    for name, w3 in (("f32", None), ("x6", ops.split_bf16x3(wp))):  # keys: f323, x623, x625
        for tile in (23, 25) if w3 is not None else (3,):
            y = ops.conv2d_nhwc(xd, wp, b.to(DEV), Cout, k, 1, (k - 1) // 2, None, tile=tile, w3=w3)
            errs[f"{name}{tile}"] = (y.permute(0, 3, 1, 2).double().cpu() - ref).abs().max().item()
    assert errs["x623"] <= 1.5 * errs["f323"] + 1e-7, errs
    assert errs["x625"] <= 1.5 * errs["f323"] + 1e-7, errs


@pytest.mark.parametrize("B,H,W,Cin,E,Cout,k,s,act", [
    (2, 160, 160, 16, 64, 24, 3, 2, "RE"),    # SSDLite block 0.2
    (3, 80, 80, 24, 72, 24, 3, 1, "RE"),      # block 0.3 (residual)
    (1, 37, 29, 12, 40, 20, 5, 2, "HS"),      # ragged tiles, K = 5, a partial channel chunk
    (2, 9, 11, 32, 96, 32, 5, 1, "R6"),       # residual with the 32-channel bound
    (1, 20, 24, 8, 128, 8, 3, 1, "RE"),       # eight waves (the 128-channel bound), residual
    (2, 17, 13, 4, 17, 4, 3, 2, "HS"),        # a one-channel last wave, Cin = 4
])
def test_mbconv_block_matches_torch(B, H, W, Cin, E, Cout, k, s, act):
    """The whole InvertedResidual in one kernel (MBCONV record: expand 1x1 + act, depthwise + act,
    project 1x1, + residual when stride 1 and Cin == Cout) against torch fp32."""
    import ctypes
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight, pack_dw_weight
    g = torch.Generator().manual_seed(B * 1000 + H + E)
    x = torch.randn(B, H, W, Cin, generator=g)
    w1 = torch.randn(E, Cin, 1, 1, generator=g) / Cin ** 0.5
    b1 = torch.randn(E, generator=g) * 0.1
    wd = torch.randn(E, 1, k, k, generator=g) / k
    bd = torch.randn(E, generator=g) * 0.1
    w2 = torch.randn(Cout, E, 1, 1, generator=g) / E ** 0.5
    b2 = torch.randn(Cout, generator=g) * 0.1
    pad = (k - 1) // 2
    xc = x.permute(0, 3, 1, 2).double()
    e = _act(F.conv2d(xc, w1.double(), b1.double()), act)
    d = _act(F.conv2d(e, wd.double(), bd.double(), stride=s, padding=pad, groups=E), act)
    y = F.conv2d(d, w2.double(), b2.double())
    res = s == 1 and Cin == Cout
    if res:
        y = y + xc
    ref = y.permute(0, 2, 3, 1).float()
    Ho, Wo = ref.shape[1], ref.shape[2]
    p1, _, kp1, _ = pack_conv_weight(w1.numpy())
    p2, _, kp2, _ = pack_conv_weight(w2.numpy())
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (p1, b1.numpy(), pack_dw_weight(wd.numpy()),
                                                                     bd.numpy(), p2, b2.numpy())]
    xd = x.cuda()
    yd = torch.full((B, Ho, Wo, Cout), float("nan"), device="cuda")
    rec = np.zeros(1, dtype=ops.OP_DTYPE)
    rec[0]["kind"] = ops.MBCONV
    for j, v in enumerate((B, H, W, Cin, E, Cout, Ho, Wo, k, s, pad, ops.ACT[act], kp1, kp2, int(res))):
        rec[0]["i"][j] = v
    for j, t in enumerate([xd] + dev + [yd]):
        rec[0]["p"][j] = t.data_ptr()
    ops.check(ops.lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, ops.stream_handle()))
    torch.cuda.synchronize()
    got = yd.cpu()
    err = (got - ref).abs().max().item()
    assert torch.isfinite(got).all() and err <= 1e-4 * max(1.0, ref.abs().max().item()), err
