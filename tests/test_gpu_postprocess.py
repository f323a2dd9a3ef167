"""Bit-exact parity of the SSD postprocess tail (SSD.postprocess_detections after softmax/decode:
per class score > t, top-k, batched_nms, [:dets], rescale) against the CPU oracle, for both device
paths: SSD_POSTPROCESS (class top-k pool + global-order greedy) and SSD_CLASS_NMS + MERGE_TOPK.

Inputs are the class probabilities / decoded boxes the reference would feed that tail, so every
discrete decision (threshold, top-k ties, IoU > thr, [:dets] cut) is checked exactly.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PATHS = ("image", "class")


def ref_postprocess(scores_t, boxes, topk, dets, thr, iou, ratio):
    """oracle restatement of ssdlite.postprocess's selection tail (oracle/ssdlite.py:154-176)."""
    from oracle import tv_ops
    out = []
    B, NC, A = scores_t.shape
    for b in range(B):
        ib, isc, il = [], [], []
        for c in range(1, NC):
            s = scores_t[b, c]
            keep = np.nonzero(s > np.float32(thr))[0]
            order = tv_ops.topk_stable(s[keep], min(topk, keep.size))
            ib.append(boxes[b][keep][order])
            isc.append(s[keep][order])
            il.append(np.full(order.size, c, np.int64))
        ib, isc, il = np.concatenate(ib), np.concatenate(isc), np.concatenate(il)
        k = tv_ops.batched_nms(ib, isc, il, iou)[:dets] if isc.size else np.zeros(0, np.int64)
        sc = np.asarray([ratio[b, 0], ratio[b, 1], ratio[b, 0], ratio[b, 1]], np.float32)
        out.append((ib[k] * sc, isc[k], il[k]))
    return out


def run_and_compare(scores_t, boxes, topk, dets, thr, iou, ratio, path):
    from edgeml_amd import ops
    ref = ref_postprocess(scores_t, boxes, topk, dets, thr, iou, ratio)
    ob, osc, olab, ocnt = ops.ssd_postprocess(torch.from_numpy(scores_t).cuda(), torch.from_numpy(boxes).cuda(),
                                              topk, dets, thr, iou, torch.from_numpy(ratio).cuda(), path=path)
    ob, osc, olab, ocnt = ob.cpu().numpy(), osc.cpu().numpy(), olab.cpu().numpy(), ocnt.cpu().numpy()
    for b, (rb, rs, rl) in enumerate(ref):
        n = int(ocnt[b])
        assert n == rs.size, (path, b, n, rs.size)
        np.testing.assert_array_equal(olab[b, :n], rl, err_msg=f"{path} labels image {b}")
        np.testing.assert_array_equal(osc[b, :n], rs, err_msg=f"{path} scores image {b}")
        np.testing.assert_array_equal(ob[b, :n], rb, err_msg=f"{path} boxes image {b}")
    return ocnt


def _softmax(x):
    e = np.exp(x - x.max(1, keepdims=True))
    return (e / e.sum(1, keepdims=True)).astype(np.float32)


def _boxes(rs, B, A, size=320.0, cluster=None):
    if cluster is None:
        c = rs.uniform(0, size, (B, A, 2))
    else:  # a few centres -> heavy overlap
        cen = rs.uniform(0, size, (B, cluster, 2))
        c = cen[:, rs.randint(0, cluster, A)] + rs.normal(0, 3.0, (B, A, 2))
    wh = rs.uniform(4, 80, (B, A, 2))
    bx = np.concatenate([c - wh / 2, c + wh / 2], -1)
    return np.clip(bx, 0, size).astype(np.float32)


@pytest.mark.parametrize("path", PATHS)
def test_model_scores_postprocess_exact(path):
    """The engine's own head outputs of a synthetic batch (SSDLite320, 91 classes, 3234 anchors)."""
    from edgeml_amd import models, synthetic
    m = models.ssdlite320_mobilenet_v3_large()
    m.to("cuda")
    imgs = synthetic.make_batch(4, 480, 640, seed=5)
    plan = m.plan(4, 480, 640)
    plan.input.tensor().copy_(imgs.cuda())
    plan.run()
    torch.cuda.synchronize()
    st = plan.scores_t.tensor().cpu().numpy()
    bx = plan.boxes.tensor().cpu().numpy()
    ratio = np.tile(np.asarray([640 / 320, 480 / 320], np.float32), (4, 1))
    cnt = run_and_compare(st, bx, 300, 300, 0.001, 0.55, ratio, path)
    assert (cnt == 300).all()


@pytest.mark.parametrize("path", PATHS)
def test_ties_and_clusters_exact(path):
    """Scores quantised to 8 levels (ties everywhere) on clustered boxes (heavy suppression)."""
    rs = np.random.RandomState(3)
    B, NC, A = 3, 91, 3234
    st = _softmax(rs.normal(0, 2, (B, NC, A)).astype(np.float32))
    st = (np.floor(st * 8 * NC) / (8 * NC)).astype(np.float32)
    bx = _boxes(rs, B, A, cluster=12)
    ratio = rs.uniform(0.5, 3, (B, 2)).astype(np.float32)
    run_and_compare(st, bx, 300, 300, 0.001, 0.55, ratio, path)


@pytest.mark.parametrize("path", PATHS)
def test_many_rounds_identical_boxes(path):
    """Every anchor has the same box, so each class keeps exactly one: the image kernel walks the
    whole 90 x 300 pool (many rounds) and still stops correctly."""
    rs = np.random.RandomState(4)
    B, NC, A = 2, 91, 3234
    st = _softmax(rs.normal(0, 1, (B, NC, A)).astype(np.float32))
    bx = np.tile(np.asarray([10, 20, 110, 90], np.float32), (B, A, 1))
    ratio = np.ones((B, 2), np.float32)
    cnt = run_and_compare(st, bx, 300, 300, 0.001, 0.55, ratio, path)
    assert (cnt == 90).all()


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("nc,a,topk,dets,thr", [(21, 500, 300, 300, 0.01), (91, 3234, 300, 300, 0.2),
                                                 (91, 3234, 300, 300, 1.0), (21, 3234, 100, 10, 0.001),
                                                 (91, 64, 300, 1024, 0.0)])
def test_shapes_and_thresholds_exact(path, nc, a, topk, dets, thr):
    """VOC class count, few anchors (take-all), thresholds leaving few or no candidates, short and
    long detection lists."""
    rs = np.random.RandomState(nc + a + dets)
    B = 2
    st = _softmax(rs.normal(0, 3, (B, nc, a)).astype(np.float32))
    bx = _boxes(rs, B, a, cluster=40)
    ratio = rs.uniform(0.5, 3, (B, 2)).astype(np.float32)
    cnt = run_and_compare(st, bx, topk, dets, thr, 0.55, ratio, path)
    if thr >= 1.0:  # probabilities never exceed 1
        assert (cnt == 0).all()


def _pools(st, bx, topk, dets, thr, select):
    from edgeml_amd import ops
    out = ops.ssd_postprocess(torch.from_numpy(st).cuda(), torch.from_numpy(bx).cuda(), topk, dets, thr, 0.55,
                              None, path="image", select=select, pool=True)
    return [t.cpu() for t in out]


@pytest.mark.parametrize("case", ["random", "quantised", "all_equal", "max_anchors", "few_valid", "topk_gt_half"])
def test_block_select_pool_equals_wave_select(case):
    """The default class selection (four waves per class, counts summed through LDS) writes the same
    candidate pool, slot for slot, as the one-wave form, and the same detections: ties at the top-k
    threshold that span the waves' register ranges are taken lowest anchor first by both."""
    rs = np.random.RandomState(11)
    B, NC, A, topk, thr = 2, 91, 3234, 300, 0.001
    if case == "random":
        st = _softmax(rs.normal(0, 2, (B, NC, A)).astype(np.float32))
    elif case == "quantised":
        st = _softmax(rs.normal(0, 2, (B, NC, A)).astype(np.float32))
        st = (np.floor(st * 4 * NC) / (4 * NC)).astype(np.float32)
    elif case == "all_equal":  # every key ties: the threshold's equal run covers all four waves
        st = np.full((B, NC, A), 1.0 / NC, np.float32)
    elif case == "max_anchors":
        A = 64 * 52
        st = _softmax(rs.normal(0, 2, (B, NC, A)).astype(np.float32))
    elif case == "few_valid":  # take-all path, and classes with no candidate
        st = _softmax(rs.normal(0, 3, (B, NC, A)).astype(np.float32))
        thr = 0.3
    else:  # most anchors kept: the threshold sits low, ties in the last wave's range
        NC, A, topk = 21, 500, 400
        st = _softmax(rs.normal(0, 1, (B, NC, A)).astype(np.float32))
        st = (np.round(st * 64) / 64).astype(np.float32)
    bx = _boxes(rs, B, A, cluster=30)
    a = _pools(st, bx, topk, 300, thr, "block")
    b = _pools(st, bx, topk, 300, thr, "wave")
    for x, y, name in zip(a, b, ("box", "score", "label", "count", "pool_key", "pool_ref")):
        if name == "pool_ref":  # slots past the written count hold no anchor (key 0)
            x = torch.where(a[4] != 0, x, -1)
            y = torch.where(b[4] != 0, y, -1)
        assert torch.equal(x, y), (case, name)
