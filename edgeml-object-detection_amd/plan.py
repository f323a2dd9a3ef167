"""Static execution plans: the host side of the engine.

A detector forward for a fixed (batch, height, width) is, in the library (csrc/lower.hip), lowered
once into
  * a packed weight blob (BatchNorm folded in float64, conv weights K-contiguous
    [Cout][KH][KW][Cin] with K padded to 32 plus their bf16 planes, depthwise weights tap-major
    [K*K][C], SE fc weights transposed), uploaded once per model and shared by every plan of it;
  * one workspace (256-byte aligned carve-outs) holding every activation, the input staging buffer
    and the output buffers;
  * an array of edgedet_op records (numpy, layout = include/edgedet.h) that libedgedet.so runs
    directly or captures into a hipGraph replayed per batch.
NativePlan is that plan on the Python side: the workspace as one torch allocation, the records
resolved against it, and the named buffers.  Plan / conv_op below build records by hand for the
unit tests of single kernels.  Nothing here computes detections: every FLOP runs in the HIP kernels
of libedgedet.so.
"""
import ctypes
import os

import numpy as np
import torch

from . import ops

ALIGN = 256

# Conv math of the compute-bound conv tiles: "bf16x6" (fp32 GEMM as six bf16 partial products on the
# bf16 matrix cores, error below one fp32 rounding per product; csrc/conv.hip) or "f32"
# (v_mfma_f32_32x32x2_f32).  Override with EDGEDET_CONV_MATH=f32.
CONV_MATH = os.environ.get("EDGEDET_CONV_MATH", "bf16x6")
if CONV_MATH not in ("bf16x6", "f32"):
    raise ValueError(f"EDGEDET_CONV_MATH must be 'bf16x6' or 'f32', got {CONV_MATH!r}")


# Measured tile per conv shape on gfx950 (tools/tune_conv.py); shapes not listed fall back to the
# library's heuristic (csrc/conv.hip choose_tile).
_TILES_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "conv_tiles_gfx950.json")
# Pre-split conv inputs for the 256 x 128 bf16x6 tile (csrc/conv.hip split_act_kernel): one x3 scratch
# per lane, sized for the largest input it serves; only where an input transform is fused (as the
# library's lowering, csrc/lower.hip conv_op).
CONV_TILES = {}
if os.path.exists(_TILES_PATH) and os.environ.get("EDGEDET_CONV_TUNED", "1") == "1":
    import json as _json
    with open(_TILES_PATH) as _f:
        CONV_TILES.update(_json.load(_f).get("tiles", {}))


def conv_key(op):
    """Shape key of a CONV op for the tuned tile table."""
    i = op.i
    lin = int(i[7] == 1 and i[8] == 1 and i[9] == 1 and i[10] == 0)
    return ",".join(str(int(v)) for v in (i[0], i[1], i[2], i[3], i[4], i[5], i[6], i[7], i[9], lin,
                                           int(op.p.get(6) is not None), int(op.p.get(7) is not None)))


def _bf16_rn(x):
    """float32 array -> (bf16 bit patterns as uint16, the bf16 values as float32), round to nearest even."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16)).astype(np.uint32)
    return r.astype(np.uint16), (r << np.uint32(16)).view(np.float32)


def split_bf16x3(w):
    """fp32 packed weights w [Cout, Kpad] -> uint16 [3, Cout, Kpad]: x0 = RN(x), x1 = RN(x - x0),
    x2 = RN(x - x0 - x1) (= exact) of x = w, and of x = -w in the odd 32-wide K blocks (k // 32 odd):
    the weight operand of the bf16x6 conv tiles, whose sign-alternated stages subtract those blocks'
    sums (csrc/conv.hip conv_x6b_body; the same arithmetic as split_bf16x3_kernel)."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    assert w.shape[-1] % 32 == 0, "rows of Kpad, a multiple of 32"
    w = np.where((np.arange(w.shape[-1]) // 32) % 2 == 1, -w, w).astype(np.float32)
    h0, f0 = _bf16_rn(w)
    r1 = (w - f0).astype(np.float32)
    h1, f1 = _bf16_rn(r1)
    r2 = (r1 - f1).astype(np.float32)
    h2, _ = _bf16_rn(r2)
    return np.stack([h0, h1, h2])


# ------------------------------------------------------------------------------ weights
class WeightPack:
    """Host-side collection of float32 arrays packed into one device blob."""

    def __init__(self):
        self.arrays = []
        self.size = 0  # in floats
        self.device_blob = None

    def add_u16(self, arr):
        """Add a uint16 array (bf16 bit patterns) of even length, stored bit-exact in the float blob."""
        a = np.ascontiguousarray(arr, dtype=np.uint16).reshape(-1)
        if a.size % 2:
            a = np.concatenate([a, np.zeros(1, np.uint16)])
        return self.add(a.view(np.float32))

    def add(self, arr):
        if isinstance(arr, np.ndarray) and arr.dtype == np.float32:
            a = np.ascontiguousarray(arr).reshape(-1)
        else:
            a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32)).reshape(-1)
        off = self.size
        self.arrays.append((off, a))
        self.size = off + ((a.size + 63) // 64) * 64
        return WRef(self, off, a.size)

    def upload(self, device):
        if self.device_blob is not None and self.device_blob.device == torch.device(device):
            return self.device_blob
        host = np.zeros(self.size, dtype=np.float32)
        for off, a in self.arrays:
            host[off:off + a.size] = a
        self.device_blob = torch.from_numpy(host).to(device)
        return self.device_blob


class WRef:
    def __init__(self, pack, off, n):
        self.pack, self.off, self.n = pack, off, n
        self.split = None  # WRef of the bf16x3 planes of a packed conv weight (conv_op p6)

    def ptr(self):
        return self.pack.device_blob.data_ptr() + 4 * self.off


def fold_bn(w, gamma, beta, mean, var, eps):
    """Eval BatchNorm folded into the preceding bias-free conv (float64 math, float32 result)."""
    w = np.asarray(w, dtype=np.float64)
    scale = np.asarray(gamma, np.float64) / np.sqrt(np.asarray(var, np.float64) + eps)
    wf = w * scale.reshape((-1,) + (1,) * (w.ndim - 1))
    bf = np.asarray(beta, np.float64) - np.asarray(mean, np.float64) * scale
    return wf.astype(np.float32), bf.astype(np.float32)


def pack_conv_weight(w_oihw, cin_pad=None):
    """[Cout][Cin][KH][KW] -> [Cout][Kpad] with K = KH*KW*Cin ordered (kh, kw, ci), zero padded."""
    w = np.asarray(w_oihw, dtype=np.float32)
    cout, cin, kh, kw = w.shape
    if cin_pad and cin_pad > cin:
        w = np.concatenate([w, np.zeros((cout, cin_pad - cin, kh, kw), np.float32)], axis=1)
        cin = cin_pad
    k = kh * kw * cin
    kpad = (k + 31) // 32 * 32
    out = np.zeros((cout, kpad), dtype=np.float32)
    out[:, :k] = w.transpose(0, 2, 3, 1).reshape(cout, k)
    return out, k, kpad, cin


def pack_dw_weight(w_c1kk):
    w = np.asarray(w_c1kk, dtype=np.float32)
    c, _, kh, kw = w.shape
    return w.reshape(c, kh * kw).T.copy()


# ------------------------------------------------------------------------------ arena + ops
_ESIZE = {}


def _esize(dtype):
    if dtype not in _ESIZE:
        _ESIZE[dtype] = torch.empty(0, dtype=dtype).element_size()
    return _ESIZE[dtype]


class Buf:
    """A carve-out of the plan arena (float32 unless dtype says otherwise)."""

    def __init__(self, shape, dtype=torch.float32, name=""):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = dtype
        self.name = name
        self.nbytes = int(np.prod(self.shape)) * _esize(dtype)
        self.off = None
        self.plan = None

    def ptr(self):
        return self.plan.arena.data_ptr() + self.off

    def tensor(self):
        n = int(np.prod(self.shape))
        es = _esize(self.dtype)
        flat = self.plan.arena[self.off:self.off + n * es].view(self.dtype)
        return flat.view(self.shape)


class BufView:
    """A batch slice of a Buf: images [b0, b0 + n) of a buffer whose leading dimension is the batch
    (the per-chain inputs / outputs of a batch-split plan)."""

    def __init__(self, buf, b0, n):
        self.buf, self.b0, self.n = buf, b0, n
        per = buf.nbytes // buf.shape[0]
        self.byte_off = b0 * per
        self.shape = (n,) + tuple(buf.shape[1:])
        self.dtype = buf.dtype

    def ptr(self):
        return self.buf.ptr() + self.byte_off

    def tensor(self):
        return self.buf.tensor()[self.b0:self.b0 + self.n]


class Op:
    def __init__(self, kind, i=None, p=None, f=None, d=None, name="", lane=0):
        self.kind, self.name, self.lane = kind, name, lane
        self.i = dict(i or {})
        self.p = dict(p or {})
        self.f = dict(f or {})
        self.d = dict(d or {})


class Plan:
    """A lowered forward: ops + arena + weights; run() or run via a captured hipGraph."""

    def __init__(self, weights, device):
        self.weights = weights
        self.device = torch.device(device)
        self.ops = []
        self.bufs = []
        self.arena = None
        self.records = None
        self.graph = None
        self.consts = []  # host arrays uploaded into the arena at finalize (anchors, ratios)

    # building -----------------------------------------------------------------------------
    def buf(self, shape, dtype=torch.float32, name=""):
        b = Buf(shape, dtype, name)
        b.plan = self
        self.bufs.append(b)
        return b

    def const(self, arr, dtype=torch.float32, name=""):
        a = np.ascontiguousarray(arr)
        b = self.buf(a.shape, dtype, name)
        self.consts.append((b, a))
        return b

    def x3_scratch(self, n):
        """The current lane's pre-split scratch, grown to at least n uint16 (ops of one lane run in
        order on one stream, so one scratch serves all of them)."""
        lane = getattr(self, "_lane", 0)
        d = self.__dict__.setdefault("_x3", {})
        b = d.get(lane)
        if b is None:
            b = d[lane] = self.buf((n,), torch.int16, name=f"x3.lane{lane}")
        elif b.shape[0] < n:
            b.shape, b.nbytes = (n,), 2 * n
        return b

    def add(self, op):
        if op.lane == 0 and getattr(self, "_lane", 0):
            op.lane = self._lane
        self.ops.append(op)
        return op

    # concurrency ---------------------------------------------------------------------------
    def fork(self, nlanes):
        """Side lanes 1..nlanes start after everything issued so far (independent branches)."""
        self.ops.append(Op(ops.FORK, {0: nlanes}, name="fork"))
        self._forked = nlanes

    def lane(self, k):
        """Issue the following ops on lane k (0 = the caller's stream)."""
        self._lane = k

    def wait(self, lane, on):
        """Lane `lane` waits for everything issued so far on lane `on` (both forked, or 0)."""
        self.ops.append(Op(ops.WAIT, {0: lane, 1: on}, name=f"wait{lane}<-{on}"))

    def join(self):
        self._lane = 0
        self.ops.append(Op(ops.JOIN, {0: self._forked}, name="join"))
        self._forked = 0

    # finalizing ---------------------------------------------------------------------------
    def finalize(self):
        off = 0
        for b in self.bufs:
            b.off = off
            off += (b.nbytes + ALIGN - 1) // ALIGN * ALIGN
        self.arena = torch.zeros(max(off, ALIGN), dtype=torch.uint8, device=self.device)
        self.weights.upload(self.device)
        for b, a in self.consts:
            b.tensor().copy_(torch.from_numpy(a).to(b.dtype))
        rec = np.zeros(len(self.ops), dtype=ops.OP_DTYPE)
        for k, op in enumerate(self.ops):
            rec[k]["kind"] = op.kind
            for j, v in op.i.items():
                rec[k]["i"][j] = int(v)
            rec[k]["i"][ops.LANE_FIELD] = op.lane
            for j, v in op.p.items():
                if v is None:
                    rec[k]["p"][j] = 0
                elif isinstance(v, (Buf, WRef, BufView)):
                    rec[k]["p"][j] = v.ptr()
                else:
                    rec[k]["p"][j] = int(v)
            for j, v in op.f.items():
                rec[k]["f"][j] = float(v)
            for j, v in op.d.items():
                rec[k]["d"][j] = float(v)
        self.records = rec
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return self

    @property
    def arena_bytes(self):
        return 0 if self.arena is None else self.arena.numel()

    # running ------------------------------------------------------------------------------
    def run(self, stream=None):
        L = ops.lib()
        ops.check(L.edgedet_plan_run(self.records.ctypes.data_as(ctypes.c_void_p), len(self.records),
                                     ops.stream_handle(stream)))

    def capture(self, stream):
        """Capture the plan into a hipGraph on `stream` (a non-default torch.cuda.Stream)."""
        L = ops.lib()
        if self.graph is not None:
            L.edgedet_graph_destroy(self.graph)
            self.graph = None
        # warm the kernels' one-time attribute setup outside of capture
        with torch.cuda.stream(stream):
            self.run(stream)
        stream.synchronize()
        g = ctypes.c_void_p()
        ops.check(L.edgedet_graph_create(self.records.ctypes.data_as(ctypes.c_void_p), len(self.records),
                                         ops.stream_handle(stream), ctypes.byref(g)))
        self.graph = g
        # prime the instance (the library uploaded the graph; the first launches also settle the
        # runtime's per-graph state), so a timed or served batch never pays a first-launch cost
        for _ in range(2):
            self.replay(stream)
        stream.synchronize()
        return self

    def replay(self, stream):
        ops.check(ops.lib().edgedet_graph_launch(self.graph, ops.stream_handle(stream)))

    def __del__(self):
        try:
            if self.graph is not None and ops._LIB is not None:
                ops._LIB.edgedet_graph_destroy(self.graph)
        except Exception:
            pass

    def summary(self):
        kinds = {}
        for op in self.ops:
            kinds[op.kind] = kinds.get(op.kind, 0) + 1
        return {"ops": len(self.ops), "by_kind": kinds, "arena_MB": self.arena_bytes / 2 ** 20,
                "weights_MB": self.weights.size * 4 / 2 ** 20}


# ------------------------------------------------------------------------------ native plans
_DTYPES = {0: torch.float32, 1: torch.int32, 2: torch.int64, 3: torch.uint8, 4: torch.int16}


class NativeBuf:
    """A named carve-out of a NativePlan's workspace (edgedet_model_buffers)."""

    def __init__(self, plan, name, offset, nbytes, dtype, shape):
        # the workspace tensor, not the plan: no plan <-> buffer reference cycle, so a plan (its graph
        # and workspace) is released when its last user drops it, at a known point, never by a
        # garbage-collector pass on whatever thread triggers one (possibly while graphs are launching)
        self.arena, self.name, self.off, self.nbytes = plan.arena, name, int(offset), int(nbytes)
        self.dtype, self.shape = dtype, tuple(int(v) for v in shape)

    def ptr(self):
        return self.arena.data_ptr() + self.off

    def tensor(self):
        es = _esize(self.dtype)
        n = int(np.prod(self.shape))
        return self.arena[self.off:self.off + n * es].view(self.dtype).view(self.shape)


class NativePlan:
    """The library's plan of (model, B, H, W, u8): workspace, resolved records, named buffers."""

    def __init__(self, model, B, H, W, u8, device):
        from . import native
        self.model, self.B, self.H, self.W, self.u8 = model, B, H, W, u8
        self.device = torch.device(device)
        kind, nc, rt = model.kind, model.num_classes, model.reduced_tail
        self.weights = model.weights(self.device)
        self.arena = torch.zeros(native.workspace_size(kind, B, H, W, nc, rt, u8), dtype=torch.uint8,
                                 device=self.device)
        L = ops.lib()
        if self.device.type == "cuda":
            ops.check(L.edgedet_model_prepare(native._kind(kind), nc, int(rt), B, H, W, int(u8),
                                              self.arena.data_ptr(), ops.stream_handle()))
        else:
            host = np.zeros(self.arena.numel(), np.uint8)
            ops.check(L.edgedet_model_prepare_host(native._kind(kind), nc, int(rt), B, H, W, int(u8),
                                                   host.ctypes.data, host.size))
            self.arena.copy_(torch.from_numpy(host))
        self.records = native.records(kind, B, H, W, self.weights.data_ptr(), self.arena.data_ptr(), nc, rt, u8)
        self.buffers = {}
        for b in native.buffers(kind, B, H, W, nc, rt, u8):
            name = bytes(b["name"]).split(b"\0", 1)[0].decode()
            self.buffers[name] = NativeBuf(self, name, b["offset"], b["nbytes"], _DTYPES[int(b["dtype"])],
                                           b["shape"][:int(b["ndim"])])
        names = native.op_names(kind, B, H, W, nc, rt, u8)
        by_ptr = {}
        for nb in self.buffers.values():
            by_ptr.setdefault(nb.ptr(), nb)
        self.ops = []
        for k, r in enumerate(self.records):
            op = Op(int(r["kind"]), {j: int(v) for j, v in enumerate(r["i"])},
                    {j: (by_ptr.get(int(v), int(v)) if v else None) for j, v in enumerate(r["p"])},
                    {j: float(v) for j, v in enumerate(r["f"])}, {j: float(v) for j, v in enumerate(r["d"])},
                    name=names[k], lane=int(r["i"][ops.LANE_FIELD]))
            self.ops.append(op)
        self.input = self.buffer("images")
        self.out_box, self.out_score = self.buffer("out.boxes"), self.buffer("out.scores")
        self.out_label, self.out_count = self.buffer("out.labels"), self.buffer("out.count")
        # (Ho, Wo, Hp, Wp) of the transform: its own record, or the SSD stem that folds it in
        pre = next((op for op in self.ops if op.kind == ops.PREPROCESS), None)
        if pre is not None:
            self.resized = tuple(int(pre.i[j]) for j in (3, 4, 5, 6))
        else:
            stem = next(op for op in self.ops if op.kind == ops.SSD_STEM)
            self.resized = (int(stem.i[1]), int(stem.i[2]), int(stem.i[1]), int(stem.i[2]))
        self.graph = None
        model.attach(self)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def buffer(self, name):
        try:
            return self.buffers[name]
        except KeyError:
            raise KeyError(f"plan has no buffer {name!r}") from None

    def finalize(self):
        return self

    @property
    def arena_bytes(self):
        return self.arena.numel()

    run = Plan.run
    capture = Plan.capture
    replay = Plan.replay
    __del__ = Plan.__del__

    def summary(self):
        kinds = {}
        for op in self.ops:
            kinds[op.kind] = kinds.get(op.kind, 0) + 1
        return {"ops": len(self.ops), "by_kind": kinds, "arena_MB": self.arena_bytes / 2 ** 20,
                "weights_MB": self.weights.numel() / 2 ** 20}


# ------------------------------------------------------------------------------ op helpers
def conv_op(plan, x, x_shape, w, bias, cout, k, stride, pad, act, y, y_shape, K, Kpad, res=None, res_hw=None,
            in_scale=None, y_pstride=None, y_bstride=None, y_off=0, x_pstride=None, x_bstride=None, tile=0,
            name="", in_shift=None, in_relu=False):
    """Build a CONV record.  x_shape = (B, H, W, C) as laid out in x; y_shape = (B, Ho, Wo, Cout)."""
    B, H, W, C = x_shape
    _, Ho, Wo, _ = y_shape
    assert Ho == (H + 2 * pad - k) // stride + 1 and Wo == (W + 2 * pad - k) // stride + 1, name
    assert K == k * k * C, (name, K, k, C)
    xp = C if x_pstride is None else x_pstride
    yp = cout if y_pstride is None else y_pstride
    rH, rW = res_hw if res_hw is not None else (Ho, Wo)
    i = {0: B, 1: H, 2: W, 3: C, 4: Ho, 5: Wo, 6: cout, 7: k, 8: k, 9: stride, 10: pad, 11: ops.ACT[act], 12: K,
         13: Kpad, 14: xp, 15: yp, 16: cout, 17: (H * W * xp if x_bstride is None else x_bstride),
         18: (Ho * Wo * yp if y_bstride is None else y_bstride), 19: rH * rW * cout, 20: y_off, 21: rH, 22: rW,
         23: tile, 24: 1 if in_relu else 0}
    w3 = getattr(w, "split", None) if CONV_MATH == "bf16x6" else None
    op = Op(ops.CONV, i, {0: x, 1: w, 2: bias, 3: y, 4: res, 5: in_scale, 6: w3, 7: in_shift}, name=name)
    if not tile:
        t = CONV_TILES.get(conv_key(op))
        if t and (w3 is not None or t < 20):
            op.i[23] = int(t)
    if op.i[23] == 26:
        # split-K accumulates into y: only for a dense output without activation or residual, zeroed
        # by a MEMSET record right before the conv (another conv of the same shape key may not qualify)
        dense = yp == cout and y_off == 0 and (y_bstride is None or y_bstride == Ho * Wo * cout)
        if act is None and res is None and dense and w3 is not None:
            plan.add(Op(ops.MEMSET, {0: B * Ho * Wo * cout * 4}, {0: y}, name=name + ".zero"))
        else:
            op.i[23] = 25
    # only where an input transform is fused: the split pass then also takes the per-element GN / SE
    # arithmetic out of the GEMM loop (measured: GN+ReLU head conv 1.83 -> 1.74 ms); for a plain input
    # the extra pass costs more than the in-loop split (box head 2.48 -> 2.60 ms)
    xf = in_scale is not None or in_shift is not None or in_relu
    if xf and w3 is not None and C % 32 == 0 and op.i[23] in (0, 25):
        op.p[8] = plan.x3_scratch(3 * B * H * W * C + 32)  # 32 leading zeros (csrc/conv.hip X3Z)
    return plan.add(op)
