"""The model-level C-ABI's lowering (csrc/lower.hip) against the Python host's (models.py, plan.py),
on the CPU: the native library must build the identical plan — the same packed weight bytes, the
same workspace size and constants, and byte-identical op records (every shape, tile, pointer,
threshold and lane) — so a non-Python host running edgedet_model_forward runs exactly what the
Python model object runs (tests/test_gpu_native_model.py then checks the detections on the GPU).
"""
import numpy as np
import pytest
import torch

from edgeml_amd import models, native, ops, synthetic


def _python_plan(model, B, H, W, u8):
    P = model.build_plan(B, H, W, u8)  # device None -> the plan finalises on the CPU
    P.finalize()
    return P


CASES = [
    ("ssd", 91, True, 2, 480, 640, False),
    ("ssd", 91, True, 16, 640, 640, True),    # two batch chains on stream lanes
    ("ssd", 21, False, 3, 427, 640, False),   # full tail, VOC classes
    ("faster_rcnn", 91, True, 1, 480, 640, False),
    ("faster_rcnn", 21, True, 2, 612, 612, True),
    ("faster_rcnn", 91, True, 1, 427, 640, True),  # fp32 resize scale: 799 x 1199
]


@pytest.fixture(scope="module")
def built():
    cache = {}

    def get(kind, nc, rt):
        key = (kind, nc, rt)
        if key not in cache:
            sd = synthetic.synthetic_state_dict(kind, nc, rt, seed=3, calibrated=False)
            m = models.SSDLite320(sd, nc, rt) if kind == "ssd" else models.FasterRCNNFPNv2(sd, nc)
            cache[key] = (sd, m)
        return cache[key]
    return get


@pytest.mark.parametrize("kind,nc,rt", [("ssd", 91, True), ("ssd", 21, False), ("faster_rcnn", 91, True)])
def test_packed_weights_identical(built, kind, nc, rt):
    sd, m = built(kind, nc, rt)
    blob = native.pack_state_dict(kind, sd, nc, rt)
    host = m.pack.upload("cpu").numpy().view(np.uint8)
    assert blob.size == host.size == native.weights_size(kind, nc, rt)
    assert np.array_equal(blob, host)


@pytest.mark.parametrize("kind,nc,rt,B,H,W,u8", CASES)
def test_records_and_constants_identical(built, kind, nc, rt, B, H, W, u8):
    sd, m = built(kind, nc, rt)
    P = _python_plan(m, B, H, W, u8)
    ws = native.workspace_size(kind, B, H, W, nc, rt, u8)
    assert ws == P.arena_bytes
    rec = native.records(kind, B, H, W, P.weights.device_blob.data_ptr(), P.arena.data_ptr(), nc, rt, u8)
    assert len(rec) == len(P.records)
    for k, (a, b) in enumerate(zip(rec, P.records)):
        assert a.tobytes() == b.tobytes(), (k, P.ops[k].name, a, b)
    host = np.zeros(ws, np.uint8)
    ops.check(ops.lib().edgedet_model_prepare_host(native._kind(kind), nc, int(rt), B, H, W, int(u8),
                                                   host.ctypes.data, ws))
    assert np.array_equal(host, P.arena.numpy())  # constants at the same offsets, nothing else written


def test_pack_rejects_bad_state_dict(built):
    sd, _ = built("ssd", 91, True)
    bad = dict(sd)
    bad.pop("head.regression_head.module_list.5.1.bias")
    with pytest.raises(ops.EdgeDetError, match="missing parameter"):
        native.pack_state_dict("ssd", bad, 91, True)
    bad = dict(sd)
    bad["backbone.features.0.0.0.weight"] = torch.zeros(16, 3, 3, 2)
    with pytest.raises(ops.EdgeDetError, match="size mismatch"):
        native.pack_state_dict("ssd", bad, 91, True)


def test_records_identical_with_fused_blocks(built, monkeypatch):
    """The opt-in whole-block MBCONV lowering (EDGEDET_MB_BLOCK=1) is mirrored by the native host."""
    sd, m = built("ssd", 91, True)
    monkeypatch.setattr(models, "MB_BLOCK_FUSE", True)
    monkeypatch.setenv("EDGEDET_MB_BLOCK", "1")
    B, H, W = 5, 300, 400  # a shape no other test lowers (the native host caches plans per shape)
    P = _python_plan(m, B, H, W, False)
    assert sum(op.kind == ops.MBCONV for op in P.ops) == 2
    rec = native.records("ssd", B, H, W, P.weights.device_blob.data_ptr(), P.arena.data_ptr(), 91, True, False)
    assert len(rec) == len(P.records)
    for k, (a, b) in enumerate(zip(rec, P.records)):
        assert a.tobytes() == b.tobytes(), (k, P.ops[k].name)
