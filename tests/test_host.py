"""CPU tests of the host side: architecture tables, anchors, plan lowering, the C-ABI library."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_param_counts_match_published():
    """SURVEY.md §6 known answers (torchvision model cards)."""
    from edgeml_amd import arch
    assert arch.param_count(arch.ssdlite_table(91, True)) == 3_440_060
    assert arch.param_count(arch.ssdlite_table(91, False)) == 5_198_540
    assert arch.param_count(arch.frcnn_table(91)) == 43_712_278
    assert arch.param_count(arch.retinanet_table(91)) == 38_198_935  # RetinaNet_ResNet50_FPN_V2_Weights


def test_ssd_anchors_match_oracle():
    from edgeml_amd import anchors
    from oracle import tv_ops
    grids = [(20, 20), (10, 10), (5, 5), (3, 3), (2, 2), (1, 1)]
    a = anchors.ssd_default_boxes(grids)
    b = tv_ops.ssd_default_boxes(grids).numpy()
    assert a.shape == (3234, 4)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("hp,wp", [(800, 800), (608, 800), (800, 1088)])
def test_rpn_anchors_match_oracle(hp, wp):
    from edgeml_amd import anchors
    from oracle import tv_ops
    grids = [(hp // 4, wp // 4), (hp // 8, wp // 8), (hp // 16, wp // 16), (hp // 32, wp // 32),
             ((hp // 32 + 1) // 2, (wp // 32 + 1) // 2)]
    for x, y in zip(anchors.rpn_anchors(grids, (hp, wp)), tv_ops.rpn_anchors(grids, (hp, wp))):
        np.testing.assert_array_equal(x, y.numpy())
    if (hp, wp) == (800, 800):
        assert sum(len(x) for x in anchors.rpn_anchors(grids, (hp, wp))) == 159_882


def test_fold_bn_matches_conv_then_bn():
    import torch.nn.functional as F
    from edgeml_amd.plan import fold_bn
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 8, 9, 9, generator=g)
    w = torch.randn(16, 8, 3, 3, generator=g)
    gam, bet = torch.rand(16, generator=g) + 0.5, torch.randn(16, generator=g)
    mu, var = torch.randn(16, generator=g), torch.rand(16, generator=g) + 0.1
    ref = F.batch_norm(F.conv2d(x, w, None, 1, 1), mu, var, gam, bet, False, 0.0, 1e-3)
    wf, bf = fold_bn(w.numpy(), gam.numpy(), bet.numpy(), mu.numpy(), var.numpy(), 1e-3)
    got = F.conv2d(x, torch.from_numpy(wf), torch.from_numpy(bf), 1, 1)
    assert (got - ref).abs().max() < 1e-4


def test_pack_conv_weight_layout():
    from edgeml_amd.plan import pack_conv_weight
    w = np.arange(2 * 3 * 3 * 3, dtype=np.float32).reshape(2, 3, 3, 3)
    p, K, Kpad, cin = pack_conv_weight(w, cin_pad=4)
    assert (K, Kpad, cin) == (36, 64, 4)
    # element (o, kh, kw, ci) at column (kh*3 + kw)*4 + ci
    for o, ci, kh, kw in [(0, 0, 0, 0), (1, 2, 2, 1), (1, 1, 0, 2)]:
        assert p[o, (kh * 3 + kw) * 4 + ci] == w[o, ci, kh, kw]
    assert np.all(p[:, 3::4][:, :9] == 0) and np.all(p[:, 36:] == 0)


def test_fastdiv_emulation():
    """csrc/common.hpp FastDiv (multiply-high) for every divisor the kernels use."""
    def make(d):
        s = 0
        while (1 << s) < d:
            s += 1
        m = ((1 << 32) * ((1 << s) - d)) // d + 1
        return m & 0xffffffff, s

    rs = np.random.RandomState(0)
    for d in [1, 2, 3, 4, 7, 13, 24, 40, 49, 100, 112, 160, 400, 1600, 2500, 40000, 160000, 12544, 3234]:
        m, s = make(d)
        ns = np.concatenate([np.arange(0, 5000), rs.randint(0, 2 ** 31 - 1, 5000)]).astype(np.uint64)
        q = ((((ns * np.uint64(m)) >> np.uint64(32)) + ns) >> np.uint64(s))
        np.testing.assert_array_equal(q, ns // np.uint64(d))


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "edgedet.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(edgedet_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from edgeml_amd import ops
    lib = ops.lib()
    declared = _declared_symbols()
    assert set(declared) == set(ops.EXPORTS), declared
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.edgedet_target() == b"gfx950"
    assert lib.edgedet_version() >= (1 << 16)
    assert lib.edgedet_conv_weight_k(3, 3, 4) == 64


def test_op_record_layout_matches_header():
    from edgeml_amd import ops
    with open(os.path.join(ROOT, "include", "edgedet.h")) as f:
        txt = f.read()
    ints = int(re.search(r"#define EDGEDET_OP_INTS (\d+)", txt).group(1))
    ptrs = int(re.search(r"#define EDGEDET_OP_PTRS (\d+)", txt).group(1))
    dbls = int(re.search(r"#define EDGEDET_OP_DBLS (\d+)", txt).group(1))
    flts = int(re.search(r"#define EDGEDET_OP_FLTS (\d+)", txt).group(1))
    assert (ints, ptrs, dbls, flts) == (ops.OP_INTS, ops.OP_PTRS, ops.OP_DBLS, ops.OP_FLTS)
    kinds = dict(re.findall(r"EDGEDET_OP_([A-Z_]+) = (\d+)", txt))
    for k, v in kinds.items():
        assert getattr(ops, k) == int(v), k


def test_unit_ops_refuse_cpu_tensors():
    from edgeml_amd import ops
    with pytest.raises(ValueError):
        ops.nms(torch.zeros(3, 4), torch.zeros(3), 0.5)


def test_models_refuse_cpu_device():
    from edgeml_amd import models
    m = models.ssdlite320_mobilenet_v3_large()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.to("cpu")


def test_state_dict_validation():
    from edgeml_amd import models, synthetic
    sd = synthetic.synthetic_state_dict("ssd", 91, True)
    sd.pop("head.regression_head.module_list.0.1.bias")
    with pytest.raises(RuntimeError, match="missing keys"):
        models.SSDLite320(sd, 91, True)


def test_ssd_plan_lowering():
    """The op list covers every layer and the arena/offset bookkeeping is consistent."""
    from edgeml_amd import models, ops
    m = models.ssdlite320_mobilenet_v3_large()
    P = m.build_plan(4, 640, 480)
    kinds = [op.kind for op in P.ops]
    # the transform is folded into the fused stem (its own record only with EDGEDET_SSD_STEM_FUSE=0)
    assert ops.PREPROCESS not in kinds and ops.SSD_STEM in kinds and kinds[-1] == ops.SSD_POSTPROCESS
    stem = P.ops[kinds.index(ops.SSD_STEM)]
    assert [stem.i[k] for k in (1, 2, 7, 8)] == [320, 320, 640, 480] and P.resized == (320, 320, 320, 320)
    # one chain at B = 4: no side lanes (the head branches are grouped launches, not lanes)
    assert kinds.count(ops.FORK) == kinds.count(ops.JOIN) == 0
    pp = P.ops[-1]
    assert [pp.i[k] for k in range(5)] == [4, 3234, 91, 300, 300]
    assert {op.lane for op in P.ops} == {0}
    # the heads: two GROUP records, the twelve depthwise convs then the twelve 1x1 convs
    g = [k for k, kd in enumerate(kinds) if kd == ops.GROUP]
    assert len(g) == 2 and [P.ops[k].i[0] for k in g] == [12, 12]
    assert kinds[g[0] + 1:g[0] + 13] == [ops.DWCONV] * 12 and kinds[g[1] + 1:g[1] + 13] == [ops.CONV] * 12
    assert [P.ops[k].name for k in range(g[1] + 1, g[1] + 13)][:2] == [
        "head.classification_head.module_list.0.1", "head.regression_head.module_list.0.1"]
    # convs: stem 1 + blocks 0-11 (block 0 has no expansion: 1 + 11*2) + C4 split 2 + blocks 13-14 (2*2)
    #        + last 1 + extras 4*2 + head 6*2
    n_conv = kinds.count(ops.CONV)
    # with the fused stem (SSD_STEM = features.0.0 + block 0's depthwise and projection) one
    # depthwise and two convs fewer
    n_dw = kinds.count(ops.DWCONV)
    stem = kinds.count(ops.SSD_STEM)
    assert stem == (0 if os.environ.get("EDGEDET_SSD_STEM_FUSE") == "0" else 1)
    # blocks 0.2 and 0.3 (no SE, <= 32 channels in and out) as single MBCONV ops: one depthwise and
    # two convs fewer each
    mb = kinds.count(ops.MBCONV)
    assert mb == (0 if os.environ.get("EDGEDET_MB_BLOCK") == "0" else 2)
    heads = 12
    assert n_dw == 15 + 4 + heads - stem - mb
    assert n_conv == 1 + 23 + 2 + 4 + 1 + 8 + heads - 2 * stem - 2 * mb
    assert kinds.count(ops.SE_FC) == 8
    assert m.grids == [(20, 20), (10, 10), (5, 5), (3, 3), (2, 2), (1, 1)]
    for op in P.ops:
        if op.kind == ops.CONV:
            assert op.i[12] == op.i[7] * op.i[8] * op.i[3] and op.i[13] % 32 == 0


@pytest.mark.parametrize("kind,B,H,W", [("ssd", 16, 480, 640), ("faster_rcnn", 2, 427, 640), ("retinanet", 1, 640, 640)])
def test_plan_buffers_partition_the_workspace(kind, B, H, W):
    """edgedet_model_buffers: every buffer inside the workspace, 256-byte aligned, none overlapping,
    and every record pointer into the workspace lands inside one of them."""
    from edgeml_amd import models
    m = {"ssd": models.ssdlite320_mobilenet_v3_large, "faster_rcnn": models.fasterrcnn_resnet50_fpn_v2,
         "retinanet": models.retinanet_resnet50_fpn_v2}[kind]()
    P = m.build_plan(B, H, W)
    spans = sorted((b.off, b.off + b.nbytes, n) for n, b in P.buffers.items())
    for (a0, a1, na), (b0, _, nb) in zip(spans, spans[1:]):
        assert a1 <= b0, (na, nb)
    assert all(o % 256 == 0 for o, _, _ in spans) and spans[-1][1] <= P.arena_bytes
    base, top = P.arena.data_ptr(), P.arena.data_ptr() + P.arena_bytes
    for op in P.ops:
        for v in op.p.values():
            ptr = v.ptr() if hasattr(v, "ptr") else v
            if v is not None and base <= ptr < top:
                assert any(base + o <= ptr < base + e for o, e, _ in spans), op.name
    assert len(P.ops) == len(P.records) and all(op.name for op in P.ops)


def test_frcnn_plan_lowering():
    from edgeml_amd import models, ops
    m = models.fasterrcnn_resnet50_fpn_v2()
    P = m.build_plan(2, 480, 640)
    assert m.resized_size(480, 640) == (800, 1066)
    pre = P.ops[0]
    assert pre.i[5] == 800 and pre.i[6] == 1088  # padded to /32
    kinds = [op.kind for op in P.ops]
    assert kinds.count(ops.ROI_ALIGN) == 1 and kinds.count(ops.RPN_LEVEL_NMS) == 1
    assert kinds.count(ops.CONV) == 1 + 16 * 3 + 4 + 8 + 5 * 4 + 4 + 2


def test_split_bf16x3_is_exact():
    """The three bf16 planes of plan.split_bf16x3 sum back to the fp32 value exactly (negated in the
    odd 32-wide K blocks: the bf16x6 kernels' sign-alternated stages), each term is a bf16 bit pattern,
    and the terms shrink by >= 2^8 (RN split: |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|)."""
    import numpy as np
    from edgeml_amd.plan import split_bf16x3
    rng = np.random.default_rng(0)
    w = (rng.standard_normal(100000) * 10.0 ** rng.integers(-8, 8, 100000)).astype(np.float32).reshape(625, 160)
    planes = split_bf16x3(w)
    vals = (planes.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    sign = np.where((np.arange(160) // 32) % 2 == 1, -1.0, 1.0)
    assert np.array_equal(vals.sum(0), w.astype(np.float64) * sign)
    assert np.array_equal(vals.sum(0)[:, :32], w[:, :32].astype(np.float64))
    a = np.abs(w.astype(np.float64))
    assert np.all(np.abs(vals[1]) <= a * 2.0 ** -8 * (1 + 1e-7))
    assert np.all(np.abs(vals[2]) <= a * 2.0 ** -16 * (1 + 1e-7))


def test_reward_ensembles_are_the_reference_draws():
    """edgeml_amd.reward.ensembles = reward.py:34-38 under np.random.seed(seed + i) (oracle harness)."""
    import numpy as np
    from edgeml_amd import reward
    for n, e in ((1, 5), (7, 0), (30, 10), (30, 100)):
        E, ens = reward.ensembles(n, e, seed=3)
        assert E == min(e, n - 1) and ens.shape == (n, E)
        for i in range(n):
            np.random.seed(3 + i)
            idx = np.arange(n - 1)
            if i < n - 1:
                idx[i:] += 1
            np.testing.assert_array_equal(ens[i], np.random.permutation(idx)[:E])
            assert i not in ens[i]


def test_reward_entries_sorted_by_class_then_conf():
    import numpy as np
    from edgeml_amd import reward
    tp = lambda n: np.zeros((n, 1), bool)  # noqa: E731
    weak = [(tp(3), np.array([0.2, 0.9, 0.5]), np.array([1, 1, 7])), (tp(0), np.array([]), np.array([]))]
    strong = [(tp(1), np.array([0.95]), np.array([1])), (tp(2), np.array([0.9, 0.3]), np.array([1, 3]))]
    labels = [np.array([1, 3]), np.array([])]
    C, lab_cnt, img, flag, seg = reward._entries(weak, strong, labels)
    assert C == 2 and seg.tolist() == [0, 4, 5]  # class 7 has no labels: dropped
    np.testing.assert_array_equal(img, [0, 0, 1, 0, 1])       # conf .95(s), .9(w,img0), .9(s,img1), .2 | 3: .3
    np.testing.assert_array_equal(flag >> 1, [1, 0, 1, 0, 1])
    np.testing.assert_array_equal(lab_cnt, [[1, 1], [0, 0]])


@pytest.mark.parametrize("hp,wp", [(800, 800), (608, 800)])
def test_retina_anchors_match_oracle(hp, wp):
    import numpy as np
    from edgeml_amd import anchors
    from oracle import tv_ops
    grids = [((hp + s - 1) // s, (wp + s - 1) // s) for s in (8, 16, 32, 64, 128)]
    ours = anchors.retina_anchors(grids, (hp, wp))
    ref = tv_ops.retina_anchors(grids, (hp, wp))
    for a, b in zip(ours, ref):
        assert a.shape[0] == b.shape[0] and a.shape[0] % 9 == 0
        np.testing.assert_array_equal(a, b.numpy())


def test_estimator_state_layout_matches_library():
    """edgeml_amd.estimator.MlpSpec and csrc/estimator.hip mlp_layout agree on the state size."""
    import ctypes
    from edgeml_amd import estimator, ops
    for dims in ([145, 16, 16, 16, 16, 1], [205, 16, 16, 16, 16, 1], [8, 1], [30, 64, 1]):
        spec = estimator.MlpSpec(dims)
        arr = (ctypes.c_int32 * len(dims))(*dims)
        assert ops.lib().edgedet_mlp_state_size(len(dims) - 1, arr) == spec.ns
    spec = estimator.MlpSpec([145, 16, 16, 16, 16, 1])
    assert spec.np == 145 * 16 + 16 + 2 * 16 + 3 * (16 * 16 + 16 + 2 * 16) + 16 + 1


def test_estimator_host_helpers_follow_the_reference():
    """parse_path (lib/utils.py:8-22, absolute paths lose their root as os.path.join(*parts) does),
    the rank normalisation (regression.py:431-434) and the init bounds (kaiming_uniform_)."""
    import numpy as np
    from edgeml_amd import estimator
    assert estimator.parse_path("runs/est") == ("runs/est_best", "runs/est_last")
    assert estimator.parse_path("/tmp/x/est") == ("tmp/x/est_best", "tmp/x/est_last")
    assert estimator.parse_path("") == ("", "")
    tr = np.array([0.3, 0.1, 0.2, 0.5])
    a, b = estimator.normalize_rewards(tr, np.array([0.25, 0.6]))
    np.testing.assert_array_equal(a, [0.75, 0.25, 0.5, 1.0])
    np.testing.assert_array_equal(b, [0.5, 1.0])
    spec = estimator.MlpSpec([145, 16, 1])
    s = spec.init_state(np.random.default_rng(0))
    w = spec.unpack(s)["linear_stacks.0.0.weight"]
    assert np.abs(w).max() <= np.sqrt(6 / 145) and np.abs(w).max() > 0.9 * np.sqrt(6 / 145)
    assert (spec.unpack(s)["linear_stacks.0.1.running_var"] == 1).all()


def test_ssd_chain_split_covers_the_batch(monkeypatch):
    """SSDLite batch chains (csrc/lower.hip SSDLite::lower): the batch split as evenly as possible over
    the chains (earlier chains +1), each chain's input a batch slice of the plan's input."""
    from edgeml_amd import models, native
    m = models.ssdlite320_mobilenet_v3_large()
    for B, n, want in [(32, 0, 2), (33, 0, 2), (10, 0, 1), (40, 4, 4), (24, 3, 3)]:
        monkeypatch.setenv("EDGEDET_SSD_CHAINS", str(n))
        native.release("ssd", B, 320, 320)
        P = m.build_plan(B, 320, 320)
        parts = [P.buffer(f"backbone.features.0.13#{c}").shape[0] for c in range(P.chains)] if P.chains > 1 else [B]
        assert P.chains == want and sum(parts) == B and max(parts) - min(parts) <= 1
        assert parts == sorted(parts, reverse=True)
        native.release("ssd", B, 320, 320)


def test_bench_attaches_committed_pmc_traffic():
    """bench.attach_traffic takes the committed rocprofv3 PMC summary for the roofline launch: the
    same layer in any batch chain ("#k" copies have one shape and grid), never a different shape."""
    import importlib.util
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("_bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    with open(os.path.join(root, "profiles", "pmc_ssd.json")) as f:
        pmc = json.load(f)
    base = pmc["launch"].split("#")[0]
    for k in (0, 1):
        roof = {"launch": f"{base}#{k}", "grid_wg": pmc["grid_wg"], "traffic": None, "kernel": pmc["kernel"]}
        bench.attach_traffic(roof, "ssd")
        assert roof["traffic"] == pmc["hbm_bytes_per_launch"]
    for roof in ({"launch": base + "#0", "grid_wg": pmc["grid_wg"] + 1, "traffic": None},
                 {"launch": "backbone.features.0.0#0", "grid_wg": pmc["grid_wg"], "traffic": None},
                 {"launch": base + "#0", "grid_wg": pmc["grid_wg"], "traffic": None, "kernel": "other_kernel"}):
        bench.attach_traffic(roof, "ssd")
        assert roof["traffic"] is None
