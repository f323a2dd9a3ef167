"""Side-lane -> side-lane waits (EDGEDET_OP_WAIT) run directly and captured into a hipGraph
(a capture of that topology crashed inside the HIP runtime in round 2, when the
experiment re-recorded one shared event per lane; every WAIT now records its own event).  A chain
lane 1 -> lane 2 -> lane 3 of dependent convs must give the sequential result, replay after replay."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from edgeml_amd import ops
from edgeml_amd.plan import Plan, WeightPack, conv_op, pack_conv_weight

pytestmark = pytest.mark.gpu


def _build(lanes):
    g = torch.Generator().manual_seed(3)
    C = 32
    ws = [torch.randn(C, C, 3, 3, generator=g) * 0.1 for _ in range(3)]
    pack = WeightPack()
    refs = []
    for w in ws:
        wp, K, Kpad, _ = pack_conv_weight(w.numpy())
        refs.append((pack.add(wp), pack.add(np.zeros(C, np.float32)), K, Kpad))
    P = Plan(pack, "cuda")
    shape = (2, 12, 12, C)
    bufs = [P.buf(shape, name=f"t{k}") for k in range(4)]
    if lanes:
        P.fork(3)
    for k in range(3):
        if lanes:
            P.lane(k + 1)
            if k:
                P.wait(k + 1, k)
        w, b, K, Kpad = refs[k]
        conv_op(P, bufs[k], shape, w, b, C, 3, 1, 1, "RE", bufs[k + 1], shape, K, Kpad, name=f"c{k}")
    if lanes:
        P.join()
    P.finalize()
    x = torch.randn(2, C, 12, 12, generator=g)
    bufs[0].tensor().copy_(x.permute(0, 2, 3, 1).cuda())
    ref = x
    for w in ws:
        ref = F.relu(F.conv2d(ref, w, padding=1))
    return P, bufs[3], ref.permute(0, 2, 3, 1)


def test_side_lane_wait_chain_direct_and_captured():
    seq, out_seq, ref = _build(False)
    seq.run()
    torch.cuda.synchronize()
    torch.testing.assert_close(out_seq.tensor().cpu(), ref, rtol=1e-4, atol=1e-4)
    P, out, _ = _build(True)
    assert sum(op.kind == ops.WAIT for op in P.ops) == 2
    P.run()
    torch.cuda.synchronize()
    assert torch.equal(out.tensor().cpu(), out_seq.tensor().cpu())
    s = torch.cuda.Stream()
    P.capture(s)
    for _ in range(5):
        out.tensor().zero_()
        torch.cuda.synchronize()
        P.replay(s)
        s.synchronize()
        assert torch.equal(out.tensor().cpu(), out_seq.tensor().cpu())
    assert ops.lib().edgedet_lane_sets() >= 1


def test_lane_set_takeover_keeps_older_graphs_valid():
    """The LRU takeover of csrc/exec.hip lanes_for: at most 16 lane sets per device, a caller stream
    beyond that takes over the least recently used set (re-keyed, never destroyed).  Capture the side
    lane chain on 33 distinct caller streams (so every earlier stream's set has been taken over at
    least once, whatever sets other tests left), then replay the OLDEST graph on its own stream and the
    newest on its stream, interleaved: both give the sequential result."""
    import ctypes
    seq, out_seq, _ = _build(False)
    seq.run()
    torch.cuda.synchronize()
    want = out_seq.tensor().cpu()
    P, out, _ = _build(True)
    L = ops.lib()
    streams, graphs = [], []
    try:
        for k in range(33):
            s = torch.cuda.Stream()
            g = ctypes.c_void_p()
            ops.check(L.edgedet_graph_create(P.records.ctypes.data_as(ctypes.c_void_p), len(P.records),
                                             ops.stream_handle(s), ctypes.byref(g)))
            streams.append(s)
            graphs.append(g)
        assert L.edgedet_lane_sets() <= 16
        for r in range(3):
            for k in (0, 32, 16):
                out.tensor().zero_()
                torch.cuda.synchronize()
                ops.check(L.edgedet_graph_launch(graphs[k], ops.stream_handle(streams[k])))
                streams[k].synchronize()
                assert torch.equal(out.tensor().cpu(), want), (r, k)
    finally:
        torch.cuda.synchronize()
        for g in graphs:
            L.edgedet_graph_destroy(g)
