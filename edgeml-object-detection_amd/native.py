"""The detector call of torch_models/detect.py:78 through the model-level C-ABI (include/edgedet.h
"model forward"): what a non-Python host binds.  Here it is driven from Python (ctypes) to check it
against the Python model object and to show the binding a maintainer would write.

    blob = native.pack_state_dict("ssd", state_dict, 91)           # edgedet_model_pack (host)
    det = native.NativeDetector("ssd", blob, 91).to("cuda")         # weights to the device once
    out = det(images)                                               # edgedet_model_forward

Everything below the ctypes calls is libedgedet.so: the lowering (csrc/lower.hip), the plan executor
and the kernels.  This module adds no arithmetic.
"""
import ctypes

import numpy as np
import torch

from . import ops

KIND = {"ssd": 0, "faster_rcnn": 1, "frcnn": 1, "retinanet": 2}


def _kind(name):
    if name not in KIND:
        raise ValueError(f"native model kind must be one of {sorted(KIND)}, got {name!r}")
    return KIND[name]


def weights_size(kind, num_classes=91, reduced_tail=True):
    n = ops.lib().edgedet_model_weights_size(_kind(kind), num_classes, int(bool(reduced_tail)))
    if n < 0:
        ops.check(int(n))
    return int(n)


def pack_state_dict(kind, state_dict, num_classes=91, reduced_tail=True):
    """edgedet_model_pack: torchvision-named tensors -> the packed weight blob (host uint8 array)."""
    names, vals, sizes, keep = [], [], [], []
    for k, v in state_dict.items():
        if k.endswith("num_batches_tracked"):
            continue
        a = np.ascontiguousarray(v.detach().cpu().numpy() if torch.is_tensor(v) else v, dtype=np.float32)
        keep.append(a)
        names.append(k.encode())
        vals.append(a.ctypes.data)
        sizes.append(a.size)
    n = len(names)
    c_names = (ctypes.c_char_p * n)(*names)
    c_vals = (ctypes.c_void_p * n)(*vals)
    c_sizes = (ctypes.c_int64 * n)(*sizes)
    blob = np.zeros(weights_size(kind, num_classes, reduced_tail), np.uint8)
    ops.check(ops.lib().edgedet_model_pack(_kind(kind), num_classes, int(bool(reduced_tail)), n, c_names, c_vals,
                                           c_sizes, blob.ctypes.data))
    return blob


def workspace_size(kind, B, H, W, num_classes=91, reduced_tail=True, u8=False):
    n = ops.lib().edgedet_model_workspace_size(_kind(kind), num_classes, int(bool(reduced_tail)), B, H, W, int(u8))
    if n < 0:
        ops.check(int(n))
    return int(n)


def records(kind, B, H, W, weights, workspace, num_classes=91, reduced_tail=True, u8=False, images=0, outputs=(0,) * 4):
    """The op records the native forward runs (pointers against the given bases)."""
    L = ops.lib()
    args = (_kind(kind), num_classes, int(bool(reduced_tail)), B, H, W, int(u8), weights, workspace, images, *outputs)
    n = L.edgedet_model_records(*args, None, 0)
    if n < 0:
        ops.check(int(n))
    rec = np.zeros(int(n), dtype=ops.OP_DTYPE)
    m = L.edgedet_model_records(*args, rec.ctypes.data, int(n))
    if m != n:
        ops.check(int(m) if m < 0 else -1)
    return rec


BUFFER_DTYPE = np.dtype([("name", "S96"), ("offset", "<i8"), ("nbytes", "<i8"), ("dtype", "<i4"), ("ndim", "<i4"),
                         ("shape", "<i8", 6)])


def buffers(kind, B, H, W, num_classes=91, reduced_tail=True, u8=False):
    """The plan's workspace buffers (edgedet_model_buffers): name, offset, nbytes, dtype, ndim, shape."""
    L = ops.lib()
    args = (_kind(kind), num_classes, int(bool(reduced_tail)), B, H, W, int(u8))
    n = L.edgedet_model_buffers(*args, None, 0)
    if n < 0:
        ops.check(int(n))
    out = np.zeros(int(n), dtype=BUFFER_DTYPE)
    m = L.edgedet_model_buffers(*args, out.ctypes.data, int(n))
    if m != n:
        ops.check(int(m) if m < 0 else -1)
    return out


def op_names(kind, B, H, W, num_classes=91, reduced_tail=True, u8=False):
    """The layer name of every record of the plan (edgedet_model_op_names)."""
    L = ops.lib()
    args = (_kind(kind), num_classes, int(bool(reduced_tail)), B, H, W, int(u8))
    n = L.edgedet_model_op_names(*args, None, 0)
    if n < 0:
        ops.check(int(n))
    buf = ctypes.create_string_buffer(int(n))
    m = L.edgedet_model_op_names(*args, buf, int(n))
    if m != n:
        ops.check(int(m) if m < 0 else -1)
    return buf.value.decode().split("\n")


def release(kind, B, H, W, num_classes=91, reduced_tail=True, u8=False):
    """Drop the library's cached lowering of this shape (it is rebuilt on next use)."""
    ops.check(ops.lib().edgedet_model_release(_kind(kind), num_classes, int(bool(reduced_tail)), B, H, W, int(u8)))


class NativeDetector:
    """model(images) through edgedet_model_forward; same contract as edgeml_amd.models' detectors
    (detect.py:78-81): [3,H,W] float images in [0, 1] or uint8 -> [{"boxes", "scores", "labels"}]."""

    def __init__(self, kind, blob, num_classes=91, reduced_tail=True):
        self.kind, self.k = kind, _kind(kind)
        self.num_classes, self.reduced_tail = num_classes, int(bool(reduced_tail))
        self.blob = blob
        self.weights = None
        self.ws = {}

    def to(self, device):
        self.device = torch.device(device)
        self.weights = torch.from_numpy(self.blob).to(self.device)
        return self

    def workspace(self, B, H, W, u8):
        key = (B, H, W, u8)
        if key not in self.ws:
            n = workspace_size(self.kind, B, H, W, self.num_classes, self.reduced_tail, u8)
            ws = torch.zeros(n, dtype=torch.uint8, device=self.device)
            ops.check(ops.lib().edgedet_model_prepare(self.k, self.num_classes, self.reduced_tail, B, H, W, int(u8),
                                                      ws.data_ptr(), ops.stream_handle()))
            self.ws[key] = ws
        return self.ws[key]

    @torch.no_grad()
    def __call__(self, images):
        x = images if torch.is_tensor(images) and images.dim() == 4 else torch.stack(list(images))
        u8 = x.dtype == torch.uint8
        x = x.to(self.device, torch.uint8 if u8 else torch.float32).contiguous()
        B, _, H, W = x.shape
        K = ops.lib().edgedet_model_max_detections(self.k)
        count = torch.zeros(B, dtype=torch.int32, device=self.device)
        boxes = torch.zeros((B, K, 4), dtype=torch.float32, device=self.device)
        scores = torch.zeros((B, K), dtype=torch.float32, device=self.device)
        labels = torch.zeros((B, K), dtype=torch.int64, device=self.device)
        ws = self.workspace(B, H, W, u8)
        ops.check(ops.lib().edgedet_model_forward(self.k, self.num_classes, self.reduced_tail, self.weights.data_ptr(),
                                                  x.data_ptr(), B, H, W, int(u8), ws.data_ptr(), count.data_ptr(),
                                                  boxes.data_ptr(), scores.data_ptr(), labels.data_ptr(),
                                                  ops.stream_handle()))
        n = count.cpu().tolist()
        return [{"boxes": boxes[b, :n[b]], "scores": scores[b, :n[b]], "labels": labels[b, :n[b]]} for b in range(B)]
