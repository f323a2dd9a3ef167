"""RetinaNet-R50-FPN-v2 (detect.py:34-38) on the GPU against the CPU oracle (oracle/retinanet.py).

* GN_STATS + the fused GroupNorm-apply/ReLU A-load of the conv against torch's F.group_norm + conv;
* the raw head outputs (cls logits, box regression of every level) against the oracle forward;
* the postprocess kernels on identical head outputs against the oracle's postprocess;
* the final detections of the whole model (decision-replay protocol of tests/parity_models.py).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F


pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gn_stats(x_nhwc, gamma, beta, groups=32, eps=1e-5):
    from edgeml_amd import ops
    B, H, W, C = x_nhwc.shape
    sc = torch.empty((B, C), device=DEV)
    sh = torch.empty((B, C), device=DEV)
    rec = np.zeros(1, dtype=ops.OP_DTYPE)
    rec[0]["kind"] = ops.GN_STATS
    rec[0]["i"][:4] = [B, H * W, C, groups]
    for j, t in enumerate((x_nhwc, gamma, beta, sc, sh)):
        rec[0]["p"][j] = t.data_ptr()
    rec[0]["f"][0] = eps
    import ctypes
    ops.check(ops.lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, ops.stream_handle()))
    return sc, sh


@pytest.mark.parametrize("B,H,W", [(2, 25, 25), (1, 7, 13), (3, 50, 40)])
def test_group_norm_stats_match_torch(B, H, W):
    g = torch.Generator().manual_seed(B * H)
    x = torch.randn(B, 256, H, W, generator=g) * 3 + 1
    gamma = torch.rand(256, generator=g) + 0.5
    beta = torch.randn(256, generator=g)
    ref = F.group_norm(x, 32, gamma, beta, 1e-5)
    sc, sh = _gn_stats(x.permute(0, 2, 3, 1).contiguous().to(DEV), gamma.to(DEV), beta.to(DEV))
    got = x.to(DEV) * sc[:, :, None, None] + sh[:, :, None, None]
    assert (got.cpu() - ref).abs().max().item() < 2e-5


@pytest.mark.parametrize("tile", [0, 3, 23, 25])
def test_conv_fused_groupnorm_relu_input(tile):
    """conv(relu(GN(x))) with the GN apply + ReLU fused into the conv's A-operand load."""
    from edgeml_amd import ops
    from edgeml_amd.plan import pack_conv_weight
    g = torch.Generator().manual_seed(tile)
    B, H, W = 2, 20, 18
    x = torch.randn(B, 256, H, W, generator=g)
    gamma, beta = torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g)
    w = torch.randn(256, 256, 3, 3, generator=g) / 48.0
    b = torch.randn(256, generator=g) * 0.1
    ref = F.conv2d(F.relu(F.group_norm(x, 32, gamma, beta, 1e-5)), w, b, 1, 1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    sc, sh = _gn_stats(xd, gamma.to(DEV), beta.to(DEV))
    wp = torch.from_numpy(pack_conv_weight(w.numpy())[0]).to(DEV)
    w3 = ops.split_bf16x3(wp) if tile in (0, 23, 25) else None
    import ctypes
    Cin = Cout = 256
    y = torch.empty((B, H, W, Cout), device=DEV)
    K = 9 * Cin
    rec = np.zeros(1, dtype=ops.OP_DTYPE)
    rec[0]["kind"] = ops.CONV
    vals = [B, H, W, Cin, H, W, Cout, 3, 3, 1, 1, 0, K, K, Cin, Cout, Cout, H * W * Cin, H * W * Cout, H * W * Cout, 0,
            H, W, tile, 1]
    rec[0]["i"][:len(vals)] = vals
    for j, t in enumerate((xd, wp, b.to(DEV), y, None, sc, w3, sh)):
        rec[0]["p"][j] = 0 if t is None else t.data_ptr()
    ops.check(ops.lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, ops.stream_handle()))
    err = (y.permute(0, 3, 1, 2).cpu() - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


@pytest.fixture(scope="module")
def retina():
    from edgeml_amd import models, synthetic
    sd = synthetic.synthetic_state_dict("retinanet", 91, seed=0)
    return sd, models.RetinaNetFPNv2(sd, 91).to(DEV)


def test_retinanet_raw_heads_match_oracle(retina):
    from edgeml_amd import synthetic
    from oracle.retinanet import RetinaNetOracle
    sd, model = retina
    imgs = synthetic.make_batch(2, 640, 640, seed=41)
    cls_ref, reg_ref, _, _, _ = RetinaNetOracle(sd, 91).forward_raw(list(imgs))
    plan = model.plan(2, 640, 640)
    plan.input.tensor().copy_(imgs.to(DEV))
    plan.run()
    torch.cuda.synchronize()
    cls = plan.cls_logits.tensor().cpu()
    reg = plan.bbox_regression.tensor().cpu()
    ec = (cls - torch.cat(cls_ref, 1)).abs().max().item()
    er = (reg - torch.cat(reg_ref, 1)).abs().max().item()
    print(f"retinanet raw: max|dcls|={ec:.3e} max|dreg|={er:.3e}")
    assert ec < 2e-3 and er < 2e-3


def test_retinanet_postprocess_on_identical_heads(retina):
    """The device postprocess fed the oracle's own head outputs: the decision replay of those head
    values (host sigmoid / decode) reproduces the device rows to 1 ulp, with no flip."""
    from edgeml_amd import ops, synthetic
    from oracle import retinanet as R
    import ctypes
    from tests import chains
    from tests.flips import check_replay_reproduces, replay
    sd, model = retina
    imgs = synthetic.make_batch(2, 640, 640, seed=43)
    o = R.RetinaNetOracle(sd, 91)
    cls_ref, reg_ref, anchors, sizes, _ = o.forward_raw(list(imgs))
    plan = model.plan(2, 640, 640)
    plan.input.tensor().copy_(imgs.to(DEV))
    plan.run()  # fills every buffer; then overwrite the heads and re-run only the postprocess ops
    plan.cls_logits.tensor().copy_(torch.cat(cls_ref, 1).to(DEV))
    plan.bbox_regression.tensor().copy_(torch.cat(reg_ref, 1).to(DEV))
    tail = plan.records[[k for k, op in enumerate(plan.ops) if op.kind in (ops.RETINA_SELECT, ops.RETINA_CLASS_NMS,
                                                                          ops.MERGE_TOPK)]]
    tail = np.ascontiguousarray(tail)
    tail["i"][:, ops.LANE_FIELD] = 0
    ops.check(ops.lib().edgedet_plan_run(tail.ctypes.data_as(ctypes.c_void_p), len(tail), ops.stream_handle()))
    torch.cuda.synchronize()
    counts = plan.out_count.tensor().cpu().tolist()
    scale = np.float32(640) / np.float32(800)
    for j in range(2):
        n = counts[j]
        sA, _, label_of = chains.retina_sides([c[j] for c in cls_ref], [r[j] for r in reg_ref],
                                              [c[j] for c in cls_ref], [r[j] for r in reg_ref], anchors, sizes[j])
        tA = replay(sA, chains.RETINA_STAGES)
        check_replay_reproduces(tA, sA, plan.out_box.tensor()[j, :n].cpu().numpy(),
                                plan.out_score.tensor()[j, :n].cpu().numpy(),
                                plan.out_label.tensor()[j, :n].cpu().numpy(), label_of, scale=scale, rtol=2e-6)
        ref = R.postprocess([c[j:j + 1] for c in cls_ref], [r[j:j + 1] for r in reg_ref], anchors, sizes[j:j + 1])[0]
        check_replay_reproduces(tA, sA, ref["boxes"].numpy(), ref["scores"].numpy(), ref["labels"].numpy(), label_of)
        assert n > 0


@pytest.mark.parametrize("h,w,n", [(480, 640, 1), (640, 640, 2), (427, 640, 1), (375, 500, 1)])
def test_retinanet_detections_match_oracle(retina, h, w, n):
    from edgeml_amd import synthetic
    from tests import parity_models as PM
    sd, model = retina
    imgs = synthetic.make_batch(n, h, w, seed=47 + h)
    plan = model.plan(n, h, w)
    plan.input.tensor().copy_(imgs.to(DEV))
    plan.run()
    torch.cuda.synchronize()
    rep = PM.retina_check(plan, sd, 91, imgs, f"retinanet {n}x{h}x{w}")
    print(rep)
    assert rep["rows"] > 0
