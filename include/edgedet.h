/*
 * edgedet.h — C-ABI of libedgedet.so, the MI355X (gfx950) detection-output engine.
 *
 * This library is the native half of the drop-in replacement for the hot path of
 * torch_models/detect.py (the torchvision forward called at detect.py:78 for the models built by
 * load_weak_models, detect.py:15-42).  The reference has no FFI of its own (no native
 * code); its operator boundary is the torchvision detection-model call
 *     model(Tensor[N,3,H,W] float32 in [0,1]) -> List[{"boxes","scores","labels"}]   (detect.py:78-81)
 * and the torchvision C++ operators that call reaches (torchvision::nms, torchvision::roi_align and the
 * ATen convolutions).  Each entry point below names the reference operator it replaces.
 *
 * Conventions
 *   - every pointer is a DEVICE pointer unless its name starts with `host_`;
 *   - the caller owns every buffer (images, packed weights, workspace, outputs); nothing here
 *     allocates on the hot path;
 *   - every call is asynchronous on the given stream (hipStream_t passed as void*; NULL = default);
 *   - return value: 0 = ok, < 0 = error; edgedet_last_error() returns the message (thread-local).
 *   - activations are NHWC float32; boxes are (x1, y1, x2, y2) float32.
 */
#ifndef EDGEDET_H
#define EDGEDET_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------- plan ops */
/*
 * One step of a static execution plan.  The Python host (edgeml_amd/plan.py) lowers a detector
 * into an array of these (BatchNorm folded, weights packed, buffers carved from one arena) and the
 * native executor launches them in order.  Field meaning per `kind` is documented in plan.py and
 * csrc/exec.cpp; sizes and pointers are plain integers so the layout is identical from ctypes.
 */
#define EDGEDET_OP_INTS 48
#define EDGEDET_OP_PTRS 24
#define EDGEDET_OP_DBLS 8
#define EDGEDET_OP_FLTS 16

/* One op record.  Field layouts per kind: csrc/exec.hip (header comment), e.g. DWCONV p0 x, p1 w,
 * p2 bias, p3 y, p4 SE partial sums; GROUP i0 = members. */
typedef struct edgedet_op {
    int64_t kind;
    int64_t i[EDGEDET_OP_INTS];
    uint64_t p[EDGEDET_OP_PTRS];
    double d[EDGEDET_OP_DBLS]; /* thresholds compared in double, as the reference's CPU nms */
    float f[EDGEDET_OP_FLTS];
} edgedet_op;

enum {
    EDGEDET_OP_MEMSET = 1,        /* zero p[0] for i[0] bytes                                         */
    EDGEDET_OP_PREPROCESS = 2,    /* GeneralizedRCNNTransform: normalize, bilinear resize, zero pad   */
    EDGEDET_OP_CONV = 3,          /* conv2d + folded BN + bias + residual/upsample-add + activation   */
    EDGEDET_OP_DWCONV = 4,        /* depthwise conv2d + folded BN + activation (+ the SE squeeze)      */
    EDGEDET_OP_CHANNEL_MEAN = 5,  /* adaptive_avg_pool2d(1) (SqueezeExcitation squeeze)               */
    EDGEDET_OP_SE_FC = 6,         /* SqueezeExcitation fc1-ReLU-fc2-Hardsigmoid (standalone form)      */
    EDGEDET_OP_MAXPOOL = 7,       /* max_pool2d (ResNet stem 3x3 s2 p1, FPN LastLevelMaxPool 1x1 s2)  */
    EDGEDET_OP_SSD_SCORES = 8,    /* SSD softmax + BoxCoder.decode + clip                             */
    EDGEDET_OP_SSD_CLASS_NMS = 9, /* per (image, class): score>t, top-k, NMS                          */
    EDGEDET_OP_MERGE_TOPK = 10,   /* per image: merge kept lists, sort by score, keep[:N], rescale    */
    EDGEDET_OP_RPN_LEVEL_NMS = 11,/* per (image, FPN level): top-k logits, decode, clip, small, NMS
                                   * (with p20..p22 a chunked top-k: per-chunk lists first; with p23
                                   * the NMS split into selection / IoU mask / scan launches)        */
    EDGEDET_OP_ROI_ALIGN = 12,    /* MultiScaleRoIAlign (LevelMapper + roi_align 7x7, sr=2)          */
    EDGEDET_OP_BOX_SCORES = 13,   /* RoIHeads softmax + class-specific decode + clip                 */
    EDGEDET_OP_BOX_CLASS_NMS = 14,/* per (image, class): score>t, remove_small, NMS                   */
    EDGEDET_OP_FORK = 15,         /* side lanes 1..i[0] wait for everything issued so far on lane 0    */
    EDGEDET_OP_JOIN = 16,         /* lane 0 waits for everything issued so far on lanes 1..i[0]        */
    EDGEDET_OP_SSD_POSTPROCESS = 17,/* per image: class top-k pool, global-order greedy NMS, [:N]      */
    EDGEDET_OP_GN_STATS = 18,     /* GroupNorm statistics -> per (image, channel) scale / shift       */
    EDGEDET_OP_RETINA_SELECT = 19,/* RetinaNet per (image, level): sigmoid > t, top-k, decode, clip   */
    EDGEDET_OP_RETINA_CLASS_NMS = 20,/* RetinaNet per (image, class): NMS over the level candidates  */
    EDGEDET_OP_SSD_STEM = 21,     /* SSDLite features.0.0 + features.0.1 in one pass                  */
    EDGEDET_OP_MBCONV = 22,       /* InvertedResidual without SE: expand, depthwise, project, residual */
    EDGEDET_OP_WAIT = 23,         /* lane i[0] waits for everything issued so far on lane i[1]         */
    /* 24 is retired (round 3's grouped SSD head kernel, measured slower and removed) */
    EDGEDET_OP_GROUP = 25         /* the next i[0] records (all CONV or all DWCONV, same lane) issued as ONE
                                   * grouped kernel launch; each member stays a complete record (and is
                                   * issued alone when the members cannot share a kernel variant) */
};

/* i[EDGEDET_OP_LANE] of every record selects the stream it is issued on: 0 = the caller's stream,
 * 1..3 = side streams owned by the library (joined back by EDGEDET_OP_JOIN; captured graphs keep
 * the fork/join as graph dependencies). */
#define EDGEDET_OP_LANE 47
#define EDGEDET_MAX_LANES 4
/* members of one EDGEDET_OP_GROUP launch */
#define EDGEDET_MAX_GROUP 12

/* Run ops[0..n) on `stream`.  Shapes are checked on the host before any launch; the lane topology
 * (FORK / JOIN / WAIT and every record's lane) is checked before anything is issued. */
int edgedet_plan_run(const edgedet_op* ops, int64_t n, void* stream);
/* The lane-topology check alone (no device access): 0 or the error edgedet_plan_run would return. */
int edgedet_plan_check(const edgedet_op* ops, int64_t n);
/* The library keeps side lanes (3 streams + events) per caller stream, at most 16 sets per device: a
 * new caller stream beyond that takes over the least recently used set (sets are never destroyed:
 * captured graphs refer to them).  edgedet_release_lanes marks `stream`'s set as the next to be taken
 * over; edgedet_lane_sets returns the number of sets. */
int edgedet_release_lanes(void* stream);
int64_t edgedet_lane_sets(void);

/* Capture ops[0..n) into a hipGraph (instantiated); *graph receives an opaque handle. */
int edgedet_graph_create(const edgedet_op* ops, int64_t n, void* stream, void** graph);
int edgedet_graph_launch(void* graph, void* stream);
int edgedet_graph_destroy(void* graph);

/* Diagnostic: leave `bytes` (a multiple of 256, 0 = none, the default) unused before, between and after
 * the workspace buffers of every plan looked up from now on (the redzone is part of the plan cache key,
 * so layouts with and without gaps never mix), so a caller can fill the gaps with a canary and catch a
 * kernel writing outside its buffers (tests/test_gpu_redzone.py).  The layout changes with the
 * setting: query edgedet_model_workspace_size and run edgedet_model_prepare again after every call
 * before the next forward -- a workspace sized before the switch is too small for the new layout. */
int edgedet_set_redzone(int64_t bytes);

/* ------------------------------------------------------------------------ model forward */
/*
 * The detector call of torch_models/detect.py:78 (model(images) -> boxes / scores / labels for the
 * models load_weak_models builds, detect.py:15-42), natively: the library lowers the detector into
 * the same static plan the Python host builds (edgeml_amd/models.py; results bit-identical to it).
 *   kind         EDGEDET_MODEL_SSDLITE (ssdlite320_mobilenet_v3_large, detect.py:24/26; reduced_tail
 *                1 = the COCO-pretrained variant, 0 = the --model-path / train.py variant) or
 *                EDGEDET_MODEL_FRCNN (fasterrcnn_resnet50_fpn_v2, detect.py:30/32; reduced_tail unused) or
 *                EDGEDET_MODEL_RETINANET (retinanet_resnet50_fpn_v2, detect.py:36/38, the CLI's third model)
 *   num_classes  91 (coco) or 21 (voc), detect.py:67
 * Weights: edgedet_model_pack packs torchvision-named host tensors (a state_dict: names, fp32 values,
 * element counts; num_batches_tracked may be omitted) into a blob of edgedet_model_weights_size bytes
 * (BatchNorm folded, conv weights repacked and split into bf16 planes), which the caller copies to
 * the device once.  Images: B x [3, H, W], float in [0, 1] (input_u8 = 0, detect.py:58) or the
 * decoded uint8 bytes (input_u8 = 1, divided by 255 on the device, bit-identical).  Workspace:
 * caller-owned device memory of edgedet_model_workspace_size bytes for (B, H, W, input_u8), set up
 * once by edgedet_model_prepare (zeroes it and writes the anchors / rescale constants; synchronous).  Outputs:
 * count [B] int32, boxes [B][K][4] xyxy float in original pixels, scores [B][K] descending,
 * labels [B][K] int64, K = edgedet_model_max_detections(kind) (300 SSD / 100 FRCNN / 300 RetinaNet), the first
 * count[b] rows valid (detect.py:79-81).  forward is asynchronous on `stream`.
 */
enum { EDGEDET_MODEL_SSDLITE = 0, EDGEDET_MODEL_FRCNN = 1, EDGEDET_MODEL_RETINANET = 2 };
int64_t edgedet_model_weights_size(int32_t kind, int32_t num_classes, int32_t reduced_tail);
int edgedet_model_pack(int32_t kind, int32_t num_classes, int32_t reduced_tail, int64_t n_params,
                       const char* const* names, const float* const* host_values, const int64_t* numels,
                       void* host_blob);
int64_t edgedet_model_workspace_size(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B,
                                     int32_t H, int32_t W, int32_t input_u8);
int edgedet_model_prepare(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                          int32_t W, int32_t input_u8, void* workspace, void* stream);
/* edgedet_model_prepare into a host image of the workspace (bytes >= the workspace size): the
 * constants at their offsets, nothing else written (host-side checks and staging). */
int edgedet_model_prepare_host(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                               int32_t W, int32_t input_u8, void* host_workspace, int64_t bytes);
int edgedet_model_forward(int32_t kind, int32_t num_classes, int32_t reduced_tail, const void* weights,
                          const void* images, int32_t B, int32_t H, int32_t W, int32_t input_u8,
                          void* workspace, int32_t* count, float* boxes, float* scores, int64_t* labels,
                          void* stream);
int edgedet_model_max_detections(int32_t kind);
/* The workspace buffers of the plan (name, byte offset into the workspace, element type, shape): what a
 * host reads back for inspection (the parity tests read the head outputs, scores, proposals ...).
 * Returns the buffer count; fills out[] when cap is large enough. */
enum { EDGEDET_DT_F32 = 0, EDGEDET_DT_I32 = 1, EDGEDET_DT_I64 = 2, EDGEDET_DT_U8 = 3, EDGEDET_DT_I16 = 4 };
typedef struct edgedet_buffer {
    char name[96];
    int64_t offset;  /* bytes from the workspace base */
    int64_t nbytes;
    int32_t dtype;   /* EDGEDET_DT_* */
    int32_t ndim;
    int64_t shape[6];
} edgedet_buffer;
int64_t edgedet_model_buffers(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                              int32_t W, int32_t input_u8, edgedet_buffer* out, int64_t cap);
/* The layer name of every record ('\n'-separated, torchvision module paths): returns the bytes needed
 * (including the terminating NUL); fills out when cap is large enough. */
int64_t edgedet_model_op_names(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                               int32_t W, int32_t input_u8, char* out, int64_t cap);
/* Drop the cached plan of (B, H, W, input dtype) (at most 64 plans per model are kept, least recently
 * used evicted; records and workspaces already handed out stay valid). */
int edgedet_model_release(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H, int32_t W,
                          int32_t input_u8);
/* The op records forward would run (for graph capture: edgedet_graph_create on them, and for tests);
 * pointers resolved against the given bases (0 = the workspace's own region for images / outputs).
 * Returns the record count; fills out[] when cap is large enough. */
int64_t edgedet_model_records(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                              int32_t W, int32_t input_u8, uint64_t weights, uint64_t workspace,
                              uint64_t images, uint64_t count, uint64_t boxes, uint64_t scores,
                              uint64_t labels, edgedet_op* out, int64_t cap);
/* The per-detector names: the calls above with kind fixed. */
int64_t edgedet_ssdlite_workspace_size(int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                                       int32_t W, int32_t input_u8);
int edgedet_ssdlite_forward(const void* weights, int32_t num_classes, int32_t reduced_tail, const void* images,
                            int32_t B, int32_t H, int32_t W, int32_t input_u8, void* workspace,
                            int32_t* count, float* boxes, float* scores, int64_t* labels, void* stream);
int64_t edgedet_frcnn_workspace_size(int32_t num_classes, int32_t B, int32_t H, int32_t W, int32_t input_u8);
int edgedet_frcnn_forward(const void* weights, int32_t num_classes, const void* images, int32_t B, int32_t H,
                          int32_t W, int32_t input_u8, void* workspace, int32_t* count, float* boxes,
                          float* scores, int64_t* labels, void* stream);

/* ------------------------------------------------------------------------ unit operators */
/*
 * torchvision::nms (reference call sites: SSD postprocess, RPN filter_proposals and RoIHeads
 * postprocess_detections, all reached from detect.py:78; semantics SURVEY.md App. A.0).
 * boxes [n,4], scores [n] -> keep [n] int64 (indices, score-descending, ties lower index first),
 * *d_num_keep int32.  Suppress j when inter/(area_i+area_j-inter) > iou_threshold.  n <= 524288:
 * up to 1024 boxes one workgroup does it all; above, a radix sort, a tiled IoU bitmask and a blocked
 * greedy scan (csrc/unitops.hip).  The scratch grows QUADRATICALLY with n: the IoU bitmask alone is
 * 8 * n * ceil(n / 64) bytes (0.5 GB at n = 65,536; 34 GB at the 524,288 cap, which fits MI355X's
 * 288 GB), plus about 40 bytes per box.  edgedet_nms / edgedet_batched_nms are CONVENIENCE entry
 * points: they take that scratch from the stream-ordered allocator (hipMallocAsync on `stream`), so
 * they allocate on the calling path.  The hot path (the model plans) never calls them; a caller that
 * must not allocate uses the _ws variants with caller-owned scratch of edgedet_nms_workspace_size(n)
 * bytes instead.
 */
int edgedet_nms(const float* boxes, const float* scores, int64_t n, double iou_threshold,
                int64_t* keep, int32_t* d_num_keep, void* stream);

/*
 * torchvision::ops.batched_nms (per-group greedy NMS; result sorted by score descending, ties by
 * lower index).  Equivalent to the reference's _batched_nms_vanilla.  n <= 524288 (as edgedet_nms).
 */
int edgedet_batched_nms(const float* boxes, const float* scores, const int64_t* idxs, int64_t n,
                        double iou_threshold, int64_t* keep, int32_t* d_num_keep, void* stream);
int64_t edgedet_nms_workspace_size(int64_t n);
int edgedet_nms_ws(const float* boxes, const float* scores, int64_t n, double iou_threshold, int64_t* keep,
                   int32_t* d_num_keep, void* workspace, int64_t workspace_bytes, void* stream);
int edgedet_batched_nms_ws(const float* boxes, const float* scores, const int64_t* idxs, int64_t n,
                           double iou_threshold, int64_t* keep, int32_t* d_num_keep, void* workspace,
                           int64_t workspace_bytes, void* stream);

/*
 * torch.topk per segment (RPN filter_proposals' per-level pre_nms_top_n, SSD's per-class topk of
 * postprocess_detections; reached from detect.py:78): segment s is values[seg_off[s] .. seg_off[s+1]);
 * out_values / out_index [nseg][k] (index within the segment), out_count[s] = min(k, length).  Values
 * descending, ties lower index first (the rule the oracle fixes).  1 <= k <= 1024.
 */
int edgedet_topk_segments(const float* values, const int64_t* seg_off, int64_t nseg, int32_t k,
                          float* out_values, int64_t* out_index, int32_t* out_count, void* stream);

/*
 * torchvision BoxCoder.decode_single: deltas [n,4] against ref_boxes [n,4] (xyxy)
 * with weights (wx, wy, ww, wh), dw / dh clamped to <= clamp (log(1000/16) in torchvision); then
 * clip_boxes_to_image to [0, img_w] x [0, img_h] when both are > 0.  out [n,4]; 16-byte aligned rows.
 */
int edgedet_box_decode(const float* deltas, const float* ref_boxes, int64_t n, float wx, float wy, float ww,
                       float wh, float clamp, float img_h, float img_w, float* out, void* stream);

/*
 * torchvision::roi_align forward, aligned=False (MultiScaleRoIAlign's call),
 * on an NHWC feature map.  feat [B,H,W,C]; rois [R,5] (batch_idx, x1, y1, x2, y2);
 * out [R,PH,PW,C] (NHWC; the reference's NCHW output permuted).
 */
int edgedet_roi_align(const float* feat, int64_t B, int64_t H, int64_t W, int64_t C,
                      const float* rois, int64_t R, float spatial_scale, int32_t pooled_h,
                      int32_t pooled_w, int32_t sampling_ratio, float* out, void* stream);

/*
 * ATen conv2d (+ eval BatchNorm folded into w/bias, + activation), the layers of the torchvision
 * backbones/heads reached from detect.py:78.  x NHWC [B,H,W,Cin]; w [Cout][KH][KW][Cin] (packed:
 * K = KH*KW*Cin padded to a multiple of 32 with zeros, see edgedet_conv_weight_k); bias [Cout];
 * res (nullable) NHWC [B,Ho,Wo,Cout] added before the activation; y NHWC [B,Ho,Wo,Cout].
 * act: 0 none, 1 relu, 2 relu6, 3 hardswish, 4 hardsigmoid, 5 sigmoid.
 */
int edgedet_conv2d(const float* x, int64_t B, int64_t H, int64_t W, int64_t Cin, const float* w,
                   const float* bias, int64_t Cout, int32_t KH, int32_t KW, int32_t stride,
                   int32_t pad, int32_t act, const float* res, float* y, void* stream);
int64_t edgedet_conv_weight_k(int32_t KH, int32_t KW, int64_t Cin);

/*
 * edgedet_conv2d with the math selectable: w3 (nullable) holds the packed weight split into three
 * bf16 planes [3][Cout][Kpad] (edgedet_split_bf16x3).  With w3 the compute-bound tiles run the
 * fp32 GEMM on the bf16 matrix cores as six partial products (error below one fp32 rounding per
 * product, csrc/conv.hip "bf16x6"); without it they run v_mfma_f32_32x32x2_f32.  tile 0 = auto.
 */
int edgedet_conv2d_ex(const float* x, int64_t B, int64_t H, int64_t W, int64_t Cin, const float* w,
                      const uint16_t* w3, const float* bias, int64_t Cout, int32_t KH, int32_t KW,
                      int32_t stride, int32_t pad, int32_t act, const float* res, float* y, int32_t tile,
                      void* stream);
/*
 * edgedet_conv2d_ex with a caller-owned scratch x3 of 3 * B*H*W*Cin + 32 uint16: when the 256 x 128
 * bf16x6 tile runs (tile 25, Cin % 32 == 0) the input is split into three bf16 planes once, by a
 * separate pass into x3, instead of inside every N tile of the GEMM.  Results are bit-identical to
 * edgedet_conv2d_ex; x3 may be null (then this is edgedet_conv2d_ex).
 */
int edgedet_conv2d_x3(const float* x, uint16_t* x3, int64_t B, int64_t H, int64_t W, int64_t Cin,
                      const float* w, const uint16_t* w3, const float* bias, int64_t Cout, int32_t KH,
                      int32_t KW, int32_t stride, int32_t pad, int32_t act, const float* res, float* y,
                      int32_t tile, void* stream);
/* Packed weights w [n / kpad][kpad] fp32 -> out [3][n] bf16 bit patterns: x0 = RN(x), x1 = RN(x - x0),
 * x2 = x - x0 - x1 (exact), of x = w, and of x = -w in the odd 32-wide K blocks (k / 32 odd): the
 * bf16x6 kernels subtract those stages' sums, which cancels the matrix cores' truncation bias
 * (csrc/conv.hip conv_x6b_body).  kpad: a multiple of 32 dividing n. */
int edgedet_split_bf16x3(const float* w, int64_t n, int64_t kpad, uint16_t* out, void* stream);

/*
 * SSDLite stem + first block in one pass: y = proj(relu(dw3x3(s))) + b1 + s with
 * s = hardswish(conv3x3_s2(x) + b0) (torchvision mobilenet_v3_large features.0.0 and .0.1, folded BN).
 * x NHWC4 [B,H,W,4] (the preprocessed image); w0 [16][ld0] packed (kh, kw, ci); wd [9][16];
 * w1 [16][ld1]; y [B,(H+1)/2,(W+1)/2,16].
 */
int edgedet_ssd_stem(const float* x, int64_t B, int64_t H, int64_t W, const float* w0, int64_t ld0,
                     const float* b0, const float* wd, const float* bd, const float* w1, int64_t ld1,
                     const float* b1, float* y, void* stream);
/*
 * ORIE estimator (regression.py:242-355 fit_CNN on the stage-24 features, lib/nn_model.py:28-112
 * with linear stacks only): an MLP dims[0] -> ... -> dims[L] = 1 whose hidden layers are Linear,
 * BatchNorm1d, ReLU, Dropout(dropout); MSE loss (reward-weighted when `weighted`), Adam(lr,
 * weight_decay), MultiStepLR(milestones, gamma), `batch` rows in index order, a test pass on the
 * validation rows after every epoch.  One workgroup per fold f trains on rows tr_idx[tr_off[f] ..
 * tr_off[f+1]) with targets y[f][.] and tests on va_idx[va_off[f] .. va_off[f+1]).  State vectors
 * ([F][edgedet_mlp_state_size]: per layer W, b, and for hidden layers gamma, beta; then the running
 * mean / var) start from init; best (lowest test loss) and last are written; adam is [F][2 * params]
 * scratch; train_loss / test_loss are [F][epochs].  dims and milestones are host arrays.
 */
int64_t edgedet_mlp_state_size(int32_t L, const int32_t* dims);
int edgedet_mlp_fit(const float* x, int64_t N, int64_t D0, const float* y, const int32_t* tr_idx,
                    const int64_t* tr_off, const int32_t* va_idx, const int64_t* va_off, int32_t folds, int32_t L,
                    const int32_t* dims, const float* init, float* best, float* last, float* adam,
                    float* train_loss, float* test_loss, int32_t epochs, int32_t batch, float lr, float gamma,
                    const int32_t* milestones, int32_t n_milestones, float weight_decay, int32_t weighted,
                    float dropout, uint64_t seed, void* stream);
/* Eval-mode forward of a trained state (running statistics, no dropout): out[r] = net(x[idx[r]]). */
int edgedet_mlp_predict(const float* x, int64_t D0, const int32_t* idx, int64_t n, int32_t L, const int32_t* dims,
                        const float* state, float* out, void* stream);
/* Depthwise conv2d (+ folded BN + act).  x NHWC [B,H,W,C]; w [KH*KW][C]; bias [C]. */
int edgedet_dwconv2d(const float* x, int64_t B, int64_t H, int64_t W, int64_t C, const float* w,
                     const float* bias, int32_t K, int32_t stride, int32_t pad, int32_t act,
                     float* y, void* stream);

/* The conv kernel variant (tile id of csrc/conv.hip conv_launch: 1-6 fp32-MFMA LDS tiles, 10-12 and
 * 15 direct pointwise tiles, 13/14/16/17 split-K pointwise tiles, 21-24/27/28 bf16x6 16-deep LDS tiles,
 * 25/26, 29-32, 38 and 39 bf16x6 32-deep swizzled tiles: 256x128 (26 with split K), 128x128, 64x128,
 * 128x64, 128x256, 33-35 streaming 1x1 tiles for Cin <= 72, Cout <= 96 with dense output rows) that a CONV
 * record would run; negative on error. */
int edgedet_conv_tile(const edgedet_op* op);

/* ------------------------------------------------------------------ ORIE consumer (reward.py) */
/*
 * lib/metrics.py box_correct (lib/data.py set_data's TP flags) for many images at once: detections
 * det_xyxy [n_det][4] f64 + det_cls, labels lab_xyxy [n_lab][4] f64 + lab_cls, both grouped per image
 * by the offsets det_off / lab_off [n_img + 1]; tp [n_det] = 1 where the detection is matched at
 * IoU >= iou_thr.  max_labels = the most labels of any one image (any count; images with more than
 * 1024 labels are matched in 1024-label chunks).
 */
int edgedet_box_correct(const double* det_xyxy, const int32_t* det_cls, const int64_t* det_off,
                        const double* lab_xyxy, const int32_t* lab_cls, const int64_t* lab_off,
                        int64_t n_img, double iou_thr, uint8_t* tp, int64_t max_labels, void* stream);
/*
 * reward.py compute_orie's two ap_per_class calls (lib/metrics.py:89-148) for n_eval evaluations.
 * Entries = every detection of every image (weak and strong), sorted per class by (conf desc, image,
 * row, weak before strong); ent_img [n_ent], ent_flag [n_ent] (bit0 TP, bit1 strong), class segments
 * seg_off [n_cls + 1]; lab_cnt [n_img][n_cls] labels per image and class; evaluation e targets image
 * target[e] with ensemble ens[e][0..E) (target excluded).  ap [n_eval][2][n_cls] (weak, strong AP per
 * class, float64, bit-identical to numpy's), n_l [n_eval][n_cls] (labels of the class in the ensemble
 * plus the target; the reference's unique classes are those with n_l > 0).
 */
int edgedet_orie_ap(const int32_t* ent_img, const uint8_t* ent_flag, const int64_t* seg_off, int32_t n_cls,
                    const int32_t* lab_cnt, int64_t n_img, const int32_t* target, const int32_t* ens, int32_t E,
                    int64_t n_eval, double* ap, int32_t* n_l, void* stream);
/*
 * test.py test_map's ap_per_class over a weak/strong mixture (test.py:14-44): evaluation e uses the
 * weak detections of the images set in weak_mask[e] and the strong detections of those in
 * strong_mask[e] (bitmaps [n_eval][(n_img + 31) / 32], bit i of word i / 32).  Same entries, AP
 * layout (ap[e][0][c]) and n_l as edgedet_orie_ap.
 */
int edgedet_map_eval(const int32_t* ent_img, const uint8_t* ent_flag, const int64_t* seg_off, int32_t n_cls,
                     const int32_t* lab_cnt, int64_t n_img, const uint32_t* weak_mask, const uint32_t* strong_mask,
                     int64_t n_eval, double* ap, int32_t* n_l, void* stream);

/*
 * lib/data.py:127-160 extract_output_feature for n_img images at once: rows [n][ncol] f64 (each
 * image's detection-file rows, grouped by off [n_img + 1]); out [n_img][num_class + (ncol - 1) * k]:
 * class counts of the first k rows, then their columns 1.. flattened (zeros beyond).
 */
int edgedet_output_features(const double* rows, const int64_t* off, int64_t n_img, int32_t ncol, int32_t num_class,
                            int32_t k, double* out, void* stream);

/* ------------------------------------------------------------------ image ingest (read_image) */
/*
 * torchvision.io.read_image(path, ImageReadMode.RGB) of detect.py:55-58 for baseline JPEGs, split
 * host / device (csrc/jpeg.hip): edgedet_jpeg_packet entropy-decodes one file's bytes on the calling
 * host thread into a packet (the nonzero coefficients of every 8x8 block + the quantisation tables);
 * returns its size (written to out when cap suffices; hw = {H, W}), 0 for a JPEG it does not handle
 * (progressive, arithmetic, CMYK/RGB, other samplings: decode that file on the host), < 0 on corrupt
 * data.  edgedet_jpeg_decode_batch runs dequantisation + islow IDCT + fancy upsampling + YCbCr->RGB for
 * B packets of one H x W already on the device (packets + offsets[b]) into out [B][3][H][W] uint8,
 * byte-identical to libjpeg's default decode; planes: B * plane_stride bytes of scratch,
 * plane_stride >= max_blocks * 64 = the largest edgedet_jpeg_plane_bytes of the batch.
 * edgedet_jpeg_reconstruct_host is the same reconstruction on the host (test checker).
 */
int64_t edgedet_jpeg_packet(const uint8_t* data, int64_t size, void* out, int64_t cap, int32_t* hw);
/* A batch of n JPEG files entropy-decoded on `threads` host threads (0 = all) straight into the device
 * image edgedet_jpeg_decode_batch reads (offsets = packets = out once uploaded): out[0..8n) the int64
 * packet offsets (padded to 256 B), then the 256-B aligned packets; hw[2i..2i+1] = (H, W) of file i,
 * *max_plane_bytes = the largest plane_bytes of the batch.  Returns the span to upload; a span above
 * cap means nothing usable was written (retry with that many bytes).  0 = a file the device path does
 * not handle (decode the batch on the host), < 0 = unreadable or corrupt file.  The detect CLI's image
 * read (detect.py:55-58) for one batch in one call. */
int64_t edgedet_jpeg_batch_packets(const char* const* paths, int64_t n, void* out, int64_t cap, int32_t* hw,
                                   int64_t* max_plane_bytes, int32_t threads);
/* (H, W) of n image files from their headers (JPEG SOFn, PNG IHDR; what PIL's Image.open(path).size
 * reports, the shapes read_image returns), parsed on `threads` host threads (0 = all): hw[2i], hw[2i+1];
 * (0, 0) for a file whose header was not understood (the caller falls back).  Returns the count found. */
int64_t edgedet_image_dims(const char* const* paths, int64_t n, int32_t* hw, int32_t threads);
int64_t edgedet_jpeg_plane_bytes(const void* host_packet);
int edgedet_jpeg_decode_batch(const void* packets, const int64_t* offsets, int32_t B, int32_t H, int32_t W,
                              int32_t max_blocks, void* planes, int64_t plane_stride, uint8_t* out, void* stream);
int edgedet_jpeg_reconstruct_host(const void* host_packet, uint8_t* out);

/* --------------------------------------------------------------------------------- misc */
const char* edgedet_last_error(void);
/* Library/ABI version: (major << 16) | minor. */
int32_t edgedet_version(void);
/* Device code target the library was built for ("gfx950"). */
const char* edgedet_target(void);

#ifdef __cplusplus
}
#endif
#endif /* EDGEDET_H */
