"""ctypes binding of libedgedet.so (the C-ABI declared in include/edgedet.h).

Importing this module never falls back to anything: if the library is missing or cannot be loaded
the import-time helper ``lib()`` raises ``EdgeDetUnavailable``.  ``torch`` is imported first so the
library binds to the same HIP runtime (libamdhip64.so.7) that PyTorch-ROCm already loaded, and
device pointers / streams from torch tensors are valid inside the library.
"""
import ctypes
import math
import os

import numpy as np
import torch  # noqa: F401  (must precede loading libedgedet.so: shared HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EDGEDET_LIB") or os.path.join(HERE, "libedgedet.so")  # override: A/B builds

OP_INTS, OP_PTRS, OP_DBLS, OP_FLTS = 48, 24, 8, 16

# kinds (include/edgedet.h)
MEMSET, PREPROCESS, CONV, DWCONV, CHANNEL_MEAN, SE_FC, MAXPOOL = 1, 2, 3, 4, 5, 6, 7
SSD_SCORES, SSD_CLASS_NMS, MERGE_TOPK, RPN_LEVEL_NMS, ROI_ALIGN, BOX_SCORES, BOX_CLASS_NMS = 8, 9, 10, 11, 12, 13, 14
FORK, JOIN, SSD_POSTPROCESS = 15, 16, 17
GN_STATS, RETINA_SELECT, RETINA_CLASS_NMS = 18, 19, 20
SSD_STEM = 21
MBCONV = 22
WAIT = 23
GROUP = 25  # the next i[0] records (CONV or DWCONV) issued as one grouped launch
MAX_GROUP = 12
LANE_FIELD, MAX_LANES = 47, 4

SE_PARTS = 16  # max pixel splits of the SE squeeze partial sums (csrc/kernels.hpp SE_PARTS)


def se_parts(ho, wo):
    """Pixel splits of a fused depthwise+squeeze layer: enough workgroups per image on large maps,
    and few partial sums to re-read on small ones (>= 16 four-pixel groups per split)."""
    groups = ho * ((wo + 3) // 4)
    return max(1, min(SE_PARTS, groups // 16))

# activations (csrc/common.hpp)
ACT = {None: 0, "RE": 1, "R6": 2, "HS": 3, "HSIG": 4, "SIG": 5}

OP_DTYPE = np.dtype([("kind", "<i8"), ("i", "<i8", OP_INTS), ("p", "<u8", OP_PTRS), ("d", "<f8", OP_DBLS),
                     ("f", "<f4", OP_FLTS)])
assert OP_DTYPE.itemsize == 8 + 8 * OP_INTS + 8 * OP_PTRS + 8 * OP_DBLS + 4 * OP_FLTS

EXPORTS = ("edgedet_plan_run", "edgedet_graph_create", "edgedet_graph_launch", "edgedet_graph_destroy",
           "edgedet_set_redzone",
           "edgedet_nms", "edgedet_batched_nms", "edgedet_roi_align", "edgedet_conv2d", "edgedet_conv_weight_k",
           "edgedet_dwconv2d", "edgedet_last_error", "edgedet_version", "edgedet_target", "edgedet_conv2d_ex",
           "edgedet_split_bf16x3", "edgedet_conv_tile", "edgedet_box_correct", "edgedet_orie_ap",
           "edgedet_map_eval", "edgedet_output_features", "edgedet_conv2d_x3", "edgedet_ssd_stem",
           "edgedet_mlp_state_size", "edgedet_mlp_fit", "edgedet_mlp_predict",
           "edgedet_model_weights_size", "edgedet_model_pack", "edgedet_model_workspace_size", "edgedet_model_prepare",
           "edgedet_model_prepare_host", "edgedet_model_forward", "edgedet_model_max_detections",
           "edgedet_model_records", "edgedet_ssdlite_workspace_size", "edgedet_ssdlite_forward",
           "edgedet_frcnn_workspace_size", "edgedet_frcnn_forward", "edgedet_plan_check", "edgedet_release_lanes",
           "edgedet_lane_sets", "edgedet_nms_workspace_size", "edgedet_nms_ws", "edgedet_batched_nms_ws",
           "edgedet_topk_segments", "edgedet_box_decode", "edgedet_jpeg_packet", "edgedet_jpeg_batch_packets", "edgedet_jpeg_plane_bytes", "edgedet_image_dims",
           "edgedet_jpeg_decode_batch", "edgedet_jpeg_reconstruct_host", "edgedet_model_buffers", "edgedet_model_op_names", "edgedet_model_release")


class EdgeDetUnavailable(RuntimeError):
    pass


class EdgeDetError(RuntimeError):
    pass


_LIB = None

_vp, _i64, _i32, _dbl, _flt = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_float


def lib():
    """Load libedgedet.so once (raises EdgeDetUnavailable when it is not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise EdgeDetUnavailable(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                                 f"(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise EdgeDetUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    L.edgedet_plan_run.argtypes = [_vp, _i64, _vp]
    L.edgedet_plan_check.argtypes = [_vp, _i64]
    L.edgedet_release_lanes.argtypes = [_vp]
    L.edgedet_lane_sets.restype = _i64
    L.edgedet_graph_create.argtypes = [_vp, _i64, _vp, ctypes.POINTER(_vp)]
    L.edgedet_graph_launch.argtypes = [_vp, _vp]
    L.edgedet_graph_destroy.argtypes = [_vp]
    L.edgedet_set_redzone.argtypes = [_i64]
    L.edgedet_nms.argtypes = [_vp, _vp, _i64, _dbl, _vp, _vp, _vp]
    L.edgedet_batched_nms.argtypes = [_vp, _vp, _vp, _i64, _dbl, _vp, _vp, _vp]
    L.edgedet_nms_workspace_size.argtypes = [_i64]
    L.edgedet_nms_workspace_size.restype = _i64
    L.edgedet_nms_ws.argtypes = [_vp, _vp, _i64, _dbl, _vp, _vp, _vp, _i64, _vp]
    L.edgedet_batched_nms_ws.argtypes = [_vp, _vp, _vp, _i64, _dbl, _vp, _vp, _vp, _i64, _vp]
    L.edgedet_jpeg_packet.argtypes = [_vp, _i64, _vp, _i64, _vp]
    L.edgedet_jpeg_packet.restype = _i64
    L.edgedet_jpeg_batch_packets.argtypes = [_vp, _i64, _vp, _i64, _vp, _vp, _i32]
    L.edgedet_jpeg_batch_packets.restype = _i64
    L.edgedet_jpeg_plane_bytes.argtypes = [_vp]
    L.edgedet_image_dims.argtypes = [_vp, _i64, _vp, _i32]
    L.edgedet_image_dims.restype = _i64
    L.edgedet_jpeg_plane_bytes.restype = _i64
    L.edgedet_jpeg_decode_batch.argtypes = [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _vp]
    L.edgedet_jpeg_reconstruct_host.argtypes = [_vp, _vp]
    L.edgedet_topk_segments.argtypes = [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp]
    L.edgedet_box_decode.argtypes = [_vp, _vp, _i64, _flt, _flt, _flt, _flt, _flt, _flt, _flt, _vp, _vp]
    L.edgedet_roi_align.argtypes = [_vp, _i64, _i64, _i64, _i64, _vp, _i64, _flt, _i32, _i32, _i32, _vp, _vp]
    L.edgedet_conv2d.argtypes = [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _vp,
                                 _vp, _vp]
    L.edgedet_conv2d_ex.argtypes = [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32,
                                    _vp, _vp, _i32, _vp]
    L.edgedet_conv2d_x3.argtypes = [_vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32,
                                    _i32, _vp, _vp, _i32, _vp]
    L.edgedet_split_bf16x3.argtypes = [_vp, _i64, _i64, _vp, _vp]
    L.edgedet_mlp_state_size.argtypes = [_i32, _vp]
    L.edgedet_mlp_state_size.restype = ctypes.c_int64
    L.edgedet_mlp_fit.argtypes = [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _i32, _i32, ctypes.c_float, ctypes.c_float, _vp, _i32, ctypes.c_float, _i32,
                                  ctypes.c_float, ctypes.c_uint64, _vp]
    L.edgedet_mlp_predict.argtypes = [_vp, _i64, _vp, _i64, _i32, _vp, _vp, _vp, _vp]
    _u64 = ctypes.c_uint64
    L.edgedet_model_weights_size.argtypes = [_i32, _i32, _i32]
    L.edgedet_model_weights_size.restype = _i64
    L.edgedet_model_pack.argtypes = [_i32, _i32, _i32, _i64, _vp, _vp, _vp, _vp]
    L.edgedet_model_workspace_size.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32, _i32]
    L.edgedet_model_workspace_size.restype = _i64
    L.edgedet_model_prepare.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp]
    L.edgedet_model_prepare_host.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64]
    L.edgedet_model_forward.argtypes = [_i32, _i32, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                                        _vp]
    L.edgedet_model_max_detections.argtypes = [_i32]
    L.edgedet_model_records.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _u64, _u64, _u64, _u64, _u64, _u64,
                                        _u64, _vp, _i64]
    L.edgedet_model_records.restype = _i64
    L.edgedet_model_buffers.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64]
    L.edgedet_model_buffers.restype = _i64
    L.edgedet_model_op_names.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32, _i32, ctypes.c_char_p, _i64]
    L.edgedet_model_op_names.restype = _i64
    L.edgedet_model_release.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32, _i32]
    L.edgedet_ssdlite_workspace_size.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32]
    L.edgedet_ssdlite_workspace_size.restype = _i64
    L.edgedet_ssdlite_forward.argtypes = [_vp, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]
    L.edgedet_frcnn_workspace_size.argtypes = [_i32, _i32, _i32, _i32, _i32]
    L.edgedet_frcnn_workspace_size.restype = _i64
    L.edgedet_frcnn_forward.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]
    L.edgedet_ssd_stem.argtypes = [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp]
    L.edgedet_box_correct.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _dbl, _vp, _i64, _vp]
    L.edgedet_orie_ap.argtypes = [_vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _i32, _i64, _vp, _vp, _vp]
    L.edgedet_map_eval.argtypes = [_vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp]
    L.edgedet_output_features.argtypes = [_vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp]
    L.edgedet_conv_tile.argtypes = [_vp]
    L.edgedet_conv_tile.restype = ctypes.c_int
    L.edgedet_conv_weight_k.argtypes = [_i32, _i32, _i64]
    L.edgedet_conv_weight_k.restype = _i64
    L.edgedet_dwconv2d.argtypes = [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp]
    L.edgedet_last_error.restype = ctypes.c_char_p
    L.edgedet_version.restype = _i32
    L.edgedet_target.restype = ctypes.c_char_p
    for name in ("edgedet_plan_run", "edgedet_graph_create", "edgedet_graph_launch", "edgedet_graph_destroy",
                 "edgedet_nms", "edgedet_batched_nms", "edgedet_roi_align", "edgedet_conv2d", "edgedet_dwconv2d", "edgedet_conv2d_ex", "edgedet_split_bf16x3", "edgedet_box_correct", "edgedet_orie_ap",
           "edgedet_map_eval", "edgedet_output_features", "edgedet_conv2d_x3", "edgedet_ssd_stem", "edgedet_mlp_fit",
                 "edgedet_mlp_predict"):
        getattr(L, name).restype = ctypes.c_int
    _LIB = L
    return L


def check(rc):
    if rc != 0:
        raise EdgeDetError(f"libedgedet error {rc}: {lib().edgedet_last_error().decode()}")


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or not t.is_contiguous()):
            raise ValueError("libedgedet operators take contiguous device tensors")


# ------------------------------------------------------------------------------ unit operators
def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms on the device (boxes [n,4] f32, scores [n] f32) -> int64 keep indices."""
    return batched_nms(boxes, scores, None, iou_threshold)


def batched_nms(boxes, scores, idxs, iou_threshold):
    """torchvision.ops.batched_nms on the device; result sorted by score desc, ties lower index.
    Scratch (edgedet_nms_workspace_size) grows quadratically in n: the IoU bitmask is
    8 * n * ceil(n / 64) bytes (0.5 GB at n = 65,536; 34 GB at the 524,288 cap)."""
    _need_cuda(boxes, scores, idxs)
    n = int(scores.shape[0])
    keep = torch.empty(max(n, 1), dtype=torch.int64, device=scores.device)
    nk = torch.zeros(1, dtype=torch.int32, device=scores.device)
    L = lib()
    wb = int(L.edgedet_nms_workspace_size(n))
    if wb < 0:
        check(wb)
    ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=scores.device)  # scratch from torch's allocator
    check(L.edgedet_batched_nms_ws(_ptr(boxes), _ptr(scores), _ptr(idxs), n, float(iou_threshold), _ptr(keep),
                                   _ptr(nk), _ptr(ws), wb, stream_handle()))
    return keep[:int(nk.item())]


def topk_segments(values, seg_off, k):
    """torch.topk per segment values[seg_off[s]:seg_off[s+1]] -> (values [S,k], index in segment [S,k],
    count [S]); descending, ties lower index first."""
    _need_cuda(values, seg_off)
    S = int(seg_off.shape[0]) - 1
    ov = torch.zeros((max(S, 1), k), dtype=torch.float32, device=values.device)
    oi = torch.full((max(S, 1), k), -1, dtype=torch.int64, device=values.device)
    oc = torch.zeros(max(S, 1), dtype=torch.int32, device=values.device)
    check(lib().edgedet_topk_segments(_ptr(values), _ptr(seg_off), S, int(k), _ptr(ov), _ptr(oi), _ptr(oc),
                                      stream_handle()))
    return ov[:S], oi[:S], oc[:S]


def box_decode(deltas, ref_boxes, weights, clamp=math.log(1000.0 / 16), image_size=None):
    """BoxCoder.decode_single (+ clip_boxes_to_image when image_size = (h, w) is given)."""
    _need_cuda(deltas, ref_boxes)
    n = int(deltas.shape[0])
    out = torch.empty((n, 4), dtype=torch.float32, device=deltas.device)
    h, w = image_size if image_size is not None else (0.0, 0.0)
    wx, wy, ww, wh = (float(v) for v in weights)
    check(lib().edgedet_box_decode(_ptr(deltas), _ptr(ref_boxes), n, wx, wy, ww, wh, float(clamp), float(h), float(w),
                                   _ptr(out), stream_handle()))
    return out


def roi_align_nhwc(feat_nhwc, rois, spatial_scale, output_size=7, sampling_ratio=2):
    """torchvision.ops.roi_align(aligned=False) on an NHWC map; returns [R, PH, PW, C]."""
    _need_cuda(feat_nhwc, rois)
    B, H, W, C = feat_nhwc.shape
    R = rois.shape[0]
    out = torch.empty((R, output_size, output_size, C), dtype=torch.float32, device=feat_nhwc.device)
    check(lib().edgedet_roi_align(_ptr(feat_nhwc), B, H, W, C, _ptr(rois), R, float(spatial_scale), output_size,
                                  output_size, sampling_ratio, _ptr(out), stream_handle()))
    return out


def split_bf16x3(w):
    """Device split of packed fp32 weights [Cout, Kpad] into three bf16 planes (uint16 bit patterns,
    [3, Cout, Kpad], the odd 32-wide K blocks of -w): the weights of the bf16x6 conv tiles
    (edgedet_split_bf16x3; same split as plan.split_bf16x3)."""
    _need_cuda(w)
    out = torch.empty((3,) + tuple(w.shape), dtype=torch.int16, device=w.device)
    check(lib().edgedet_split_bf16x3(_ptr(w), w.numel(), w.shape[-1], _ptr(out), stream_handle()))
    return out


def conv2d_nhwc(x, w_packed, bias, cout, k, stride, pad, act=None, res=None, tile=0, in_scale=None, w3=None,
                presplit=False):
    """Fused conv (+ folded BN) + residual + activation on NHWC; w_packed from plan.pack_conv_weight.

    tile=0 goes through the C entry point edgedet_conv2d_ex (automatic tile choice; with the split
    weight planes ``w3`` the compute-bound tiles run bf16x6); a non-zero tile (or an SE ``in_scale``
    [B, Cin]) runs one CONV plan record so every kernel variant is testable.  presplit=True hands the
    kernel an x3 scratch (edgedet_conv2d_x3: tile 25 then splits the input once, up front).
    """
    _need_cuda(x, w_packed, bias, res, in_scale, w3)
    B, H, W, Cin = x.shape
    Ho = (H + 2 * pad - k) // stride + 1
    Wo = (W + 2 * pad - k) // stride + 1
    # tile 26 (split-K) accumulates into y: it must start zeroed
    y = (torch.zeros if tile == 26 else torch.empty)((B, Ho, Wo, cout), dtype=torch.float32, device=x.device)
    x3 = torch.empty(3 * B * H * W * Cin + 32, dtype=torch.int16, device=x.device) if presplit else None
    if tile == 0 and in_scale is None:
        if x3 is not None:
            check(lib().edgedet_conv2d_x3(_ptr(x), _ptr(x3), B, H, W, Cin, _ptr(w_packed), _ptr(w3), _ptr(bias), cout,
                                          k, k, stride, pad, ACT[act], _ptr(res), _ptr(y), 0, stream_handle()))
        elif w3 is None:
            check(lib().edgedet_conv2d(_ptr(x), B, H, W, Cin, _ptr(w_packed), _ptr(bias), cout, k, k, stride, pad,
                                       ACT[act], _ptr(res), _ptr(y), stream_handle()))
        else:
            check(lib().edgedet_conv2d_ex(_ptr(x), B, H, W, Cin, _ptr(w_packed), _ptr(w3), _ptr(bias), cout, k, k,
                                          stride, pad, ACT[act], _ptr(res), _ptr(y), 0, stream_handle()))
        return y
    K = k * k * Cin
    kpad = int(lib().edgedet_conv_weight_k(k, k, Cin))
    rec = np.zeros(1, dtype=OP_DTYPE)
    rec[0]["kind"] = CONV
    vals = [B, H, W, Cin, Ho, Wo, cout, k, k, stride, pad, ACT[act], K, kpad, Cin, cout, cout, H * W * Cin,
            Ho * Wo * cout, Ho * Wo * cout, 0, Ho, Wo, tile]
    rec[0]["i"][:len(vals)] = vals
    for j, t in enumerate((x, w_packed, bias, y, res, in_scale, w3, None, x3)):
        rec[0]["p"][j] = 0 if t is None else t.data_ptr()
    check(lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, stream_handle()))
    return y


def ssd_stem_nhwc(x4, w0_packed, b0, wd_taps, bd, w1_packed, b1):
    """SSDLite features.0.0 + features.0.1 fused (csrc/layers.hip ssd_stem_kernel): x4 the NHWC4
    preprocessed images, weights packed by plan.pack_conv_weight / pack_dw_weight (folded BN)."""
    _need_cuda(x4, w0_packed, b0, wd_taps, bd, w1_packed, b1)
    B, H, W, _ = x4.shape
    y = torch.empty((B, (H + 1) // 2, (W + 1) // 2, 16), dtype=torch.float32, device=x4.device)
    check(lib().edgedet_ssd_stem(_ptr(x4), B, H, W, _ptr(w0_packed), w0_packed.shape[1], _ptr(b0), _ptr(wd_taps),
                                 _ptr(bd), _ptr(w1_packed), w1_packed.shape[1], _ptr(b1), _ptr(y), stream_handle()))
    return y


def dwconv2d_nhwc(x, w_taps, bias, k, stride, pad, act=None, se_part=False):
    """Depthwise conv (+ folded BN + act) on NHWC.  With se_part=True it runs the fused variant that
    also returns the SqueezeExcitation partial channel sums [B, se_parts(Ho, Wo), C]."""
    _need_cuda(x, w_taps, bias)
    B, H, W, C = x.shape
    Ho = (H + 2 * pad - k) // stride + 1
    Wo = (W + 2 * pad - k) // stride + 1
    y = torch.empty((B, Ho, Wo, C), dtype=torch.float32, device=x.device)
    if not se_part:
        check(lib().edgedet_dwconv2d(_ptr(x), B, H, W, C, _ptr(w_taps), _ptr(bias), k, stride, pad, ACT[act],
                                     _ptr(y), stream_handle()))
        return y
    parts = se_parts(Ho, Wo)
    part = torch.empty((B, parts, C), dtype=torch.float32, device=x.device)
    rec = np.zeros(1, dtype=OP_DTYPE)
    rec[0]["kind"] = DWCONV
    rec[0]["i"][:11] = [B, H, W, C, Ho, Wo, k, stride, pad, ACT[act], parts]
    for j, t in enumerate((x, w_taps, bias, y, part)):
        rec[0]["p"][j] = t.data_ptr()
    check(lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, stream_handle()))
    return y, part


def ssd_postprocess(scores_t, boxes, topk, dets, score_thresh, iou_threshold, ratio=None, path="image",
                    select="block", pool=False):
    """SSD.postprocess_detections tail on device buffers (per class score > t, top-k, batched NMS,
    [:dets]); scores_t [B, NC, A] class probabilities, boxes [B, A, 4] decoded + clipped.

    path="image" runs the SSD_POSTPROCESS record, path="class" the SSD_CLASS_NMS + MERGE_TOPK pair.
    select="wave" runs the image path's class selection one wave per class (the A/B form).
    Returns (out_box [B, dets, 4] scaled by ratio [B, 2], out_score, out_label, out_count), plus the
    image path's candidate pool (key, anchor) [B, NC-1, topk] when pool=True."""
    _need_cuda(scores_t, boxes, ratio)
    B, NC, A = scores_t.shape
    dev = scores_t.device
    ob = torch.zeros((B, dets, 4), dtype=torch.float32, device=dev)
    osc = torch.zeros((B, dets), dtype=torch.float32, device=dev)
    olab = torch.zeros((B, dets), dtype=torch.int64, device=dev)
    ocnt = torch.zeros((B,), dtype=torch.int32, device=dev)
    keep_alive = []
    if path == "image":
        pk = torch.empty((B, NC - 1, topk), dtype=torch.int32, device=dev)
        pr = torch.empty((B, NC - 1, topk), dtype=torch.int32, device=dev)
        rec = np.zeros(1, dtype=OP_DTYPE)
        rec[0]["kind"] = SSD_POSTPROCESS
        rec[0]["i"][:6] = [B, A, NC, topk, dets, 1 if select == "wave" else 0]
        for j, t in enumerate((scores_t, boxes, pk, pr, ratio, ob, osc, olab, ocnt)):
            rec[0]["p"][j] = 0 if t is None else t.data_ptr()
        rec[0]["f"][0] = score_thresh
        rec[0]["d"][0] = iou_threshold
        keep_alive += [pk, pr]
    else:
        NS = NC - 1
        rb = torch.empty((B, NS, topk, 4), dtype=torch.float32, device=dev)
        rs = torch.empty((B, NS, topk), dtype=torch.float32, device=dev)
        rt = torch.empty((B, NS, topk), dtype=torch.int32, device=dev)
        rl = torch.empty((B, NS, topk), dtype=torch.int32, device=dev)
        rc = torch.empty((B, NS), dtype=torch.int32, device=dev)
        rec = np.zeros(2, dtype=OP_DTYPE)
        rec[0]["kind"] = SSD_CLASS_NMS
        rec[0]["i"][:5] = [B, A, NC, topk, topk]
        for j, t in enumerate((scores_t, boxes, rb, rs, rt, rl, rc)):
            rec[0]["p"][j] = t.data_ptr()
        rec[0]["f"][0] = score_thresh
        rec[0]["d"][0] = iou_threshold
        rec[1]["kind"] = MERGE_TOPK
        rec[1]["i"][:4] = [B, NS, topk, dets]
        for j, t in enumerate((rb, rs, rt, rl, rc, ratio, ob, osc, olab, ocnt)):
            rec[1]["p"][j] = 0 if t is None else t.data_ptr()
        keep_alive += [rb, rs, rt, rl, rc]
    check(lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), len(rec), stream_handle()))
    torch.cuda.current_stream().synchronize()
    if pool and path == "image":
        return ob, osc, olab, ocnt, pk, pr
    return ob, osc, olab, ocnt


def se_excitation(part, hw, w1, b1, w2t, b2):
    """SqueezeExcitation avgpool -> fc1 -> ReLU -> fc2 -> Hardsigmoid from the squeeze partial sums
    part [B, splits, C] over hw pixels; w1 [S, C], w2t [S, C] (fc2 weight transposed).
    Returns the channel scales [B, C]."""
    _need_cuda(part, w1, b1, w2t, b2)
    B, parts, C = part.shape
    S = int(w1.shape[0])
    scale = torch.empty((B, C), dtype=torch.float32, device=part.device)
    hidden = torch.empty((B, S), dtype=torch.float32, device=part.device)
    rec = np.zeros(1, dtype=OP_DTYPE)
    rec[0]["kind"] = SE_FC
    rec[0]["i"][:5] = [B, C, S, hw, parts]
    for j, t in enumerate((part, w1, b1, w2t, b2, scale, hidden)):
        rec[0]["p"][j] = t.data_ptr()
    check(lib().edgedet_plan_run(rec.ctypes.data_as(ctypes.c_void_p), 1, stream_handle()))
    return scale
