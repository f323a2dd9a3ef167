"""The §8(b) unit operators beyond the plan (csrc/unitops.hip) against the oracle (oracle/tv_ops.py):
NMS / batched NMS with no size cap (n up to SSD's 27,000 candidates, the large-n sort + bitmask +
blocked-scan path above 1024), per-segment top-k, and BoxCoder decode (+ clip)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _boxes(rs, n, spread=600.0, size=60.0):
    xy = rs.uniform(0, spread, (n, 2)).astype(np.float32)
    wh = rs.uniform(1, size, (n, 2)).astype(np.float32)
    return np.concatenate([xy, xy + wh], 1).astype(np.float32)


@pytest.mark.parametrize("n", [1024, 1025, 4097, 27000])
def test_large_nms_matches_oracle(n):
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(n)
    boxes = _boxes(rs, n)
    scores = rs.uniform(0, 1, n).astype(np.float32)
    scores[100:400] = scores[7]  # a block of ties: lower index first
    scores[n // 2:n // 2 + 50] = 0.25
    for thr in (0.5, 0.7):
        ref = tv_ops.nms(boxes, scores, thr)
        got = ops.nms(torch.from_numpy(boxes).to(DEV), torch.from_numpy(scores).to(DEV), thr).cpu().numpy()
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("n,groups", [(27000, 90), (5000, 3)])
def test_large_batched_nms_matches_oracle(n, groups):
    """SSD's postprocess call: up to 90 classes x 300 candidates through one batched_nms."""
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(groups)
    boxes = _boxes(rs, n, 320.0, 80.0)
    scores = rs.uniform(0, 1, n).astype(np.float32)
    scores[::97] = 0.5
    idxs = rs.randint(0, groups, n).astype(np.int64)
    ref = tv_ops.batched_nms(boxes, scores, idxs, 0.55)
    got = ops.batched_nms(torch.from_numpy(boxes).to(DEV), torch.from_numpy(scores).to(DEV),
                          torch.from_numpy(idxs).to(DEV), 0.55).cpu().numpy()
    np.testing.assert_array_equal(got, ref)


def test_nms_ws_entry_and_empty():
    import ctypes
    from edgeml_amd import ops
    L = ops.lib()
    assert L.edgedet_nms_workspace_size(1024) == 0 and L.edgedet_nms_workspace_size(30000) > 30000 * 470 * 8
    assert ops.nms(torch.zeros((0, 4), device=DEV), torch.zeros(0, device=DEV), 0.5).numel() == 0
    rs = np.random.RandomState(1)
    n = 3000
    b = torch.from_numpy(_boxes(rs, n)).to(DEV)
    s = torch.from_numpy(rs.uniform(0, 1, n).astype(np.float32)).to(DEV)
    keep = torch.empty(n, dtype=torch.int64, device=DEV)
    nk = torch.zeros(1, dtype=torch.int32, device=DEV)
    small = torch.empty(16, dtype=torch.uint8, device=DEV)
    rc = L.edgedet_nms_ws(ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(s.data_ptr()), n, 0.5,
                          ctypes.c_void_p(keep.data_ptr()), ctypes.c_void_p(nk.data_ptr()),
                          ctypes.c_void_p(small.data_ptr()), 16, ops.stream_handle())
    assert rc < 0 and b"workspace too small" in L.edgedet_last_error()
    # the allocator path of the plain C entry (hipMallocAsync on the stream) equals the ws path
    rc = L.edgedet_nms(ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(s.data_ptr()), n, 0.5,
                       ctypes.c_void_p(keep.data_ptr()), ctypes.c_void_p(nk.data_ptr()), ops.stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    got = keep[:int(nk.item())].cpu()
    assert torch.equal(got, ops.nms(b, s, 0.5).cpu())


@pytest.mark.parametrize("k", [1, 300, 1000])
def test_topk_segments_matches_topk_stable(k):
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(k)
    lens = [0, 1, k - 1 if k > 1 else 1, k, k + 1, 3234, 20000, 5]
    vals = [rs.uniform(0, 1, n).astype(np.float32) for n in lens]
    vals[5][::3] = vals[5][0]  # ties across the cut
    vals[6] = np.round(vals[6] * 50).astype(np.float32) / 50  # heavy ties
    flat = np.concatenate(vals).astype(np.float32)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ov, oi, oc = ops.topk_segments(torch.from_numpy(flat).to(DEV), torch.from_numpy(off).to(DEV), k)
    ov, oi, oc = ov.cpu().numpy(), oi.cpu().numpy(), oc.cpu().numpy()
    for s, v in enumerate(vals):
        want = tv_ops.topk_stable(v, k)
        assert oc[s] == len(want)
        np.testing.assert_array_equal(oi[s, :oc[s]], want)
        np.testing.assert_array_equal(ov[s, :oc[s]], v[want])


@pytest.mark.parametrize("weights,clip", [((10.0, 10.0, 5.0, 5.0), (320, 320)), ((1.0, 1.0, 1.0, 1.0), (800, 1088)),
                                          ((10.0, 10.0, 5.0, 5.0), None)])
def test_box_decode_matches_oracle(weights, clip):
    from edgeml_amd import ops
    from oracle import tv_ops
    rs = np.random.RandomState(3)
    n = 5000
    refs = _boxes(rs, n, 800.0, 200.0)
    d = (rs.randn(n, 4) * 2).astype(np.float32)
    d[:50, 2:] = 30.0  # beyond the log(1000/16) clamp
    want = tv_ops.decode_boxes(d, refs, weights)[:, 0]
    if clip is not None:
        want = tv_ops.clip_boxes(want, clip)
    got = ops.box_decode(torch.from_numpy(d).to(DEV), torch.from_numpy(refs).to(DEV), weights,
                         image_size=clip).cpu()
    # exp() of two libraries (device expf vs torch CPU) may differ by an ulp; everything else is the
    # same op order
    torch.testing.assert_close(got, want, rtol=3e-7, atol=1e-4)
    assert math.isclose(float(got[:50, 2:].max()), float(want[:50, 2:].max()), rel_tol=1e-6)
