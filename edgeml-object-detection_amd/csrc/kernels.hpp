// Parameter blocks and host launchers of every kernel (shared by the .hip units and exec.hip).
#pragma once
#include "common.hpp"

namespace edgedet {

constexpr int SE_PARTS = 16;  // pixel splits of the SE squeeze partial sums

struct ConvParams {
    const float* x;
    const float* w;
    const float* bias;
    float* y;
    const float* res;
    const float* in_scale;  // [B][Cin] or null (SE excitation)
    const void* w3;         // bf16 split planes [3][Cout][Kpad] or null (bf16x6 tiles)
    const float* in_shift;  // [B][Cin] or null: input transform x * in_scale + in_shift (GroupNorm apply)
    int in_relu;            // ReLU on the transformed input (GroupNorm + ReLU, LastLevelP6P7's relu(P6))
    void* x3;               // scratch for the pre-split input planes [3][B*H*W][Cin] bf16, or null
    int B, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, act;
    int K, Kpad, M;
    int x_pstride, y_pstride, res_pstride;
    int64_t x_bstride, y_bstride, res_bstride, y_off;
    int res_H, res_W;
    float res_sh, res_sw;  // nearest-upsample scales (in/out) for the residual
    int lin_x, lin_y, lin_res;  // dense-layout fast paths (set by conv_launch)
    int ksplit;                 // 2: K halves accumulated with atomics into a zeroed y (tile 26)
    FastDiv div_howo, div_wo, div_cin, div_kw;
    // timing probe (bench.py's in-pipeline roofline; null in every product plan): the bf16x6 kernels
    // record workgroup 0's start (stamp[0]) and the max of every workgroup's end (stamp[1]) on the
    // 100 MHz constant clock into a 16-byte slot (CONV record p9)
    unsigned long long* stamp;
};

// Up to EDGEDET_MAX_GROUP conv problems issued as one launch (conv_group_launch): problem k runs the
// workgroups [start[k], start[k + 1]).
struct ConvGroup {
    int n;
    int start[EDGEDET_MAX_GROUP + 1];
    ConvParams p[EDGEDET_MAX_GROUP];
};
int conv_group_launch(const ConvParams* ps, int n, int tile, hipStream_t s);

struct PreParams {
    const float* x;      // [B][3][H][W] float in [0, 1] (the model contract, detect.py:78), or
    const uint8_t* xu8;  // [B][3][H][W] the decoded uint8 image (detect.py:57); x / 255 on the device
    float* y;        // [B][Hp][Wp][4]
    int B, H, W, Ho, Wo, Hp, Wp;
    float mean[3], stdv[3];
    float sh, sw;  // input/output scales
    float rstd[3];  // set by the launcher: RN(1 / stdv) for the uint8 fast division (u8_fast_div)
    int fastdiv;
};

struct DwParams {
    const float* x;  // [B][H][W][C]
    const float* w;  // [K*K][C]
    const float* bias;
    float* y;        // [B][Ho][Wo][C]
    float* part;     // optional SE squeeze partial sums [B][parts][C]
    int B, H, W, C, Ho, Wo, K, stride, pad, act;
    int parts;       // pixel splits of the squeeze (1..SE_PARTS)
};

// Up to EDGEDET_MAX_GROUP depthwise problems issued as one launch (dwconv_group_launch).
struct DwGroup {
    int n;
    int start[EDGEDET_MAX_GROUP + 1];
    int nq[EDGEDET_MAX_GROUP], nwg[EDGEDET_MAX_GROUP];
    DwParams p[EDGEDET_MAX_GROUP];
};
int dwconv_group_launch(const DwParams* ps, int n, hipStream_t s);

// A whole InvertedResidual without SqueezeExcitation (csrc/layers.hip mbconv_kernel).
struct MbParams {
    const float* x;   // [B][H][W][Cin] the block input (dense NHWC)
    const float* w1;  // expand [Cexp][ld1] (packed 1x1 weight, folded BN)
    const float* b1;  // [Cexp]
    const float* wd;  // depthwise [K*K][Cexp]
    const float* bd;  // [Cexp]
    const float* w2;  // project [Cout][ld2]
    const float* b2;  // [Cout]
    float* y;         // [B][Ho][Wo][Cout]
    int B, H, W, Cin, Cexp, Cout, Ho, Wo, K, stride, pad, act, ld1, ld2, residual;
};
int mbconv_launch(const MbParams& p, hipStream_t s);


struct PoolParams {
    const float* x;
    float* y;
    int B, H, W, C, Ho, Wo, K, stride, pad;
};

struct RoiParams {
    const float* feat[4];  // NHWC per level
    int H[4], W[4];
    float scale[4];
    int nlevels;
    const float* rois;      // mode 0: [R][5] (b, x1, y1, x2, y2); mode 1: boxes [B][RMAX][4]
    const int* counts;      // mode 1: valid rois per image
    int mode, R, RMAX, B, C, PH, PW, sr;
    int k_min, k_max;       // LevelMapper levels (mode 1)
    float* out;             // [R][PH][PW][C]
};

struct SegOut {
    f32x4* box;     // [B*S][kmax]
    float* score;   // [B*S][kmax]
    uint32_t* tb;   // [B*S][kmax] merge tiebreak (position of the candidate in the reference's
                    //              concatenated candidate list, order-preserving)
    int* label;     // [B*S][kmax]
    int* count;     // [B*S]
    int kmax;
};

struct RpnLevel {
    const float* obj;      // [B][HW*A] objectness logits (dense, anchor order (y, x, a))
    const float* deltas;   // [B][HW*A][4] box deltas
    const float* anchors;  // [HW*A][4]
    int n;                 // HW*A
};

// NMS IoU threshold in exact-comparison form (detect.hip iou_gt).
struct IouThr {
    double thr;  // the reference's double threshold
    double mid;  // midpoint of the float pair (t0, t1) around thr, t1 = smallest float > thr
    int tie_up;  // round-half-even of a tie at mid goes to t1
};
IouThr make_iou_thr(double thr);

struct RpnParams {
    RpnLevel lv[5];
    int nlevels, ld, A, B, topk;
    float img_h, img_w, min_size, score_thresh;
    IouThr iou;
    // chunked top-k (optional, ckey != null): a first launch keeps each chunk's top-k of every
    // (image, level) in ckey / cidx [B][nlevels][nchunk][KC] (counts in ccount), and the level kernel
    // selects from the union of its chunks instead of streaming the whole level five times
    uint32_t* ckey;
    int* cidx;
    int* ccount;
    int chunk, nchunk;
    // split NMS (optional, split != null): selection, the IoU mask over many workgroups and the greedy
    // scan as three launches, the intermediates in this scratch (rpn_split_bytes(B * nlevels))
    void* split;
};
int64_t rpn_split_bytes(int64_t nseg);

struct MergeParams {
    const f32x4* box;
    const float* score;
    const uint32_t* tb;
    const int* label;
    const int* count;    // [B][S]
    int S, kmax, N;
    const float* ratio;  // [B][2] (rw, rh) or null
    float* out_box;      // [B][N][4]
    float* out_score;    // [B][N]
    int64_t* out_label;  // [B][N] or null
    int* out_count;      // [B]
};

struct SsdPostParams {
    const float* scores_t;  // [B][NC][A] class probabilities
    const float* boxes;     // [B][A][4] decoded, clipped
    uint32_t* pool_key;     // [B][NC-1][topk] scratch
    int* pool_ref;          // [B][NC-1][topk] scratch
    const float* ratio;     // [B][2] or null
    float* out_box;         // [B][N][4]
    float* out_score;       // [B][N]
    int64_t* out_label;     // [B][N] or null
    int* out_count;         // [B]
    int B, A, NC, topk, N;
    int select_wave;        // 1: the one-wave-per-class selection (A/B form)
    float score_thresh;
    double iou;
};

struct GnParams {
    const float* x;      // [B][HW][C] NHWC
    const float* gamma;  // [C]
    const float* beta;   // [C]
    float* scale;        // [B][C]  GroupNorm(x) = x * scale + shift
    float* shift;        // [B][C]
    int B, HW, C, G;
    float eps;
};

struct RetinaSelParams {
    const float* logits;   // [B][Atot][K]
    const float* deltas;   // [B][Atot][4]
    const float* anchors;  // [Atot][4]
    int a0[5], na[5];      // anchors of each level: [a0, a0 + na)
    int L, B, Atot, K, topk;
    float img_h, img_w, score_thresh;
    uint32_t* ckey;        // [B][L][nchunk][1024] chunk top-k keys (scratch)
    int* cidx;             // [B][L][nchunk][1024] their flat indices within the level
    int* ccount;           // [B][L][nchunk]
    int chunk, nchunk;     // flat indices per chunk; chunks per level (capacity)
};

struct RetinaNmsParams {
    const f32x4* box;      // per-(image, level) candidate lists [B][L][kin]
    const float* score;
    const int* label;
    const int* count;      // [B][L]
    int L, kin, K;
    IouThr iou;
};

int gn_stats_launch(const GnParams& p, hipStream_t s);
int retina_select_launch(const RetinaSelParams& P, SegOut out, hipStream_t s);
int retina_class_nms_launch(const RetinaNmsParams& P, int B, SegOut out, hipStream_t s);
int conv_prepare(ConvParams& p);
int conv_resolve_tile(const ConvParams& p, int tile);
int conv_launch(ConvParams p, int tile, hipStream_t s);
int preprocess_launch(const PreParams& p, hipStream_t s);
int dwconv_launch(const DwParams& p, hipStream_t s);

// SSDLite stem + features.0.1 in one pass (csrc/layers.hip ssd_stem_kernel).
struct StemParams {
    const float* x;   // [B][H][W][4] preprocessed NHWC4 image
    const float* w0;  // stem conv [16][ld0] (3x3, Cin 4, folded BN), b0 [16], hardswish
    const float* b0;
    const float* wd;  // features.0.1 depthwise [9][16], bd [16], ReLU
    const float* bd;
    const float* w1;  // features.0.1 projection [16][ld1], b1 [16], + residual (the stem output)
    const float* b1;
    float* y;         // [B][Ho][Wo][16]
    int B, H, W, Ho, Wo, ld0, ld1;
    // the transform folded in (x unused): the source image [B][3][H0][W0], float or uint8 (/ 255), its
    // normalisation, resized to H x W (scales set by the launcher)
    const float* src;
    const uint8_t* src8;
    int H0, W0;
    float mean[3], stdv[3];
    float sh, sw;
    float rstd[3];  // set by the launcher (u8_fast_div)
    int fastdiv;
};
int ssd_stem_launch(const StemParams& p, hipStream_t s);
int channel_mean_launch(const float* x, float* out, int B, int HW, int C, hipStream_t s);
int se_fc_launch(const float* part, const float* w1, const float* b1, const float* w2t, const float* b2,
                 float* hidden, float* scale, int B, int C, int S, int HW, int parts, hipStream_t s);
int maxpool_launch(const PoolParams& p, hipStream_t s);
int roi_align_launch(const RoiParams& p, hipStream_t s);
int ssd_scores_launch(const float* logits, const float* reg, const float* anchors, float* scores_t, float* boxes,
                      int B, int A, int NC, float img_h, float img_w, hipStream_t s);
int box_scores_launch(const float* pred, int ld, int cls_off, int delta_off, const float* props, const int* counts,
                      float* scores, float* boxes, int B, int R, int NC, float img_h, float img_w, hipStream_t s);
int ssd_class_nms_launch(const float* scores_t, const float* boxes, int B, int A, int NC, float score_thresh,
                         int topk, double iou, SegOut out, hipStream_t s);
int rpn_level_nms_launch(const RpnParams& P, SegOut out, hipStream_t s);
int box_class_nms_launch(const float* scores, const float* boxes, const int* counts, int B, int R, int NC,
                         float score_thresh, float min_size, double iou, SegOut out, hipStream_t s);
int merge_topk_launch(const MergeParams& P, int B, hipStream_t s);
int ssd_postprocess_launch(const SsdPostParams& P, hipStream_t s);

}  // namespace edgedet
