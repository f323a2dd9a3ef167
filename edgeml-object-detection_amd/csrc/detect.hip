// Detection post-processing on gfx950: score/decode kernels and the per-segment
// "select -> sort -> NMS" machinery (segments = (image, class) or (image, FPN level)).
//
// Reference semantics (torchvision eval path reached from torch_models/detect.py:78; restated in
// SURVEY.md App. A and oracle/tv_ops.py):
//   SSD.postprocess_detections        softmax, BoxCoder(10,10,5,5).decode, clip, per class
//                                     score > 0.001, topk(300), batched_nms(0.55), [:300]   (row a10)
//   RPN.filter_proposals              per level topk(1000) of logits, decode(1,1,1,1), sigmoid,
//                                     clip, remove_small(1e-3), score >= 0, batched_nms(0.7 by
//                                     level), [:1000]                                        (row a12)
//   RoIHeads.postprocess_detections   softmax, class-specific decode(10,10,5,5), clip, drop bg,
//                                     score > 0.05, remove_small(1e-2), batched_nms(0.5), [:100] (a15)
// batched_nms is evaluated exactly as per-group NMS (torchvision's _batched_nms_vanilla); every
// sort is by score descending with ties to the earlier candidate (the reference's stable CPU sort),
// the same rule the oracle fixes (oracle/tv_ops.py header).
//
// Segment kernel = one workgroup per segment:
//   1. block radix select (4 x 8-bit passes over an orderable uint32 key, LDS histograms) finds
//      the K-th largest key T;
//   2. ordered compaction (wave ballots + block scan, index order) keeps key > T plus the first
//      ties == T;
//   3. bitonic sort in LDS of 64-bit keys (key << 32 | ~index): score desc, index asc;
//   4. NMS: IoU bitmask (row i, 64 candidates per word; suppress j > i when
//      inter / ((area_i + area_j) - inter) > thr, division IEEE-rounded, compare in double as the
//      reference's float-vs-double comparison) in LDS, then one wave resolves the greedy scan 64
//      candidates at a time;
//   5. kept records (box, score, tiebreak, label) are written to per-segment lists that
//      merge_topk combines per image.
#include <mutex>
#include <utility>
#include <vector>

#include "kernels.hpp"

namespace edgedet {


constexpr float BBOX_CLIP = 4.135166556742356f;  // log(1000/16), as float (torch.clamp casts)

// BoxCoder.decode_single on one box (weights w, clamp dw/dh <= BBOX_CLIP), op order as torchvision.
__device__ __forceinline__ f32x4 decode_box(f32x4 d, f32x4 a, float wx, float wy, float ww, float wh) {
    const float width = a.z - a.x;
    const float height = a.w - a.y;
    const float ctr_x = a.x + 0.5f * width;
    const float ctr_y = a.y + 0.5f * height;
    const float dx = d.x / wx;
    const float dy = d.y / wy;
    float dw = d.z / ww;
    float dh = d.w / wh;
    dw = fminf(dw, BBOX_CLIP);
    dh = fminf(dh, BBOX_CLIP);
    const float pcx = dx * width + ctr_x;
    const float pcy = dy * height + ctr_y;
    const float pw = expf(dw) * width;
    const float ph = expf(dh) * height;
    const float hw = 0.5f * pw;
    const float hh = 0.5f * ph;
    return f32x4{pcx - hw, pcy - hh, pcx + hw, pcy + hh};
}

__device__ __forceinline__ f32x4 clip_box(f32x4 b, float h, float w) {
    b.x = fminf(fmaxf(b.x, 0.f), w);
    b.y = fminf(fmaxf(b.y, 0.f), h);
    b.z = fminf(fmaxf(b.z, 0.f), w);
    b.w = fminf(fmaxf(b.w, 0.f), h);
    return b;
}

// ================================================================ SSD: softmax + decode + clip
// One thread per anchor.  logits [B][A][NC] -> scores_t [B][NC][A] (class-major for the per-class
// selection), reg [B][A][4] + anchors [A][4] -> boxes [B][A][4].
__global__ void ssd_scores_kernel(const float* __restrict__ logits, const float* __restrict__ reg,
                                  const float* __restrict__ anchors, float* __restrict__ scores_t,
                                  float* __restrict__ boxes, int B, int A, int NC, float img_h, float img_w) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)B * A) return;
    const int b = (int)(idx / A), a = (int)(idx % A);
    const float* l = logits + idx * NC;
    float mx = l[0];
    for (int c = 1; c < NC; ++c) mx = fmaxf(mx, l[c]);
    float sum = 0.f;
    for (int c = 0; c < NC; ++c) sum += expf(l[c] - mx);
    const float inv = 1.f / sum;
    float* st = scores_t + (int64_t)b * NC * A + a;
    for (int c = 0; c < NC; ++c) st[(int64_t)c * A] = expf(l[c] - mx) * inv;
    const f32x4 d = *reinterpret_cast<const f32x4*>(reg + idx * 4);
    const f32x4 an = *reinterpret_cast<const f32x4*>(anchors + (int64_t)a * 4);
    f32x4 bx = decode_box(d, an, 10.f, 10.f, 5.f, 5.f);
    *reinterpret_cast<f32x4*>(boxes + idx * 4) = clip_box(bx, img_h, img_w);
}

// ================================================================ FRCNN RoIHeads: softmax + decode
// One wave per RoI, lanes over classes.  pred [B*R][ld] with cls logits at [cls_off, +NC) and class
// deltas at [delta_off, +4*NC) (delta_off 16-byte aligned); proposals [B][R][4];
// -> scores [B][R][NC], boxes [B][R][NC][4].
__global__ void box_scores_kernel(const float* __restrict__ pred, int ld, int cls_off, int delta_off,
                                  const float* __restrict__ props, const int* __restrict__ counts,
                                  float* __restrict__ scores, float* __restrict__ boxes, int B, int R, int NC,
                                  float img_h, float img_w) {
    const int lane = threadIdx.x & 63;
    const int64_t roi = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (roi >= (int64_t)B * R) return;
    const int b = (int)(roi / R), r = (int)(roi % R);
    if (r >= counts[b]) return;
    const float* row = pred + roi * ld + cls_off;
    const float* drow = pred + roi * ld + delta_off;
    float mx = -__builtin_inff();
    for (int c = lane; c < NC; c += 64) mx = fmaxf(mx, row[c]);
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int c = lane; c < NC; c += 64) sum += expf(row[c] - mx);
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.f / sum;
    const f32x4 an = *reinterpret_cast<const f32x4*>(props + roi * 4);
    for (int c = lane; c < NC; c += 64) {
        scores[roi * NC + c] = expf(row[c] - mx) * inv;
        const f32x4 d = *reinterpret_cast<const f32x4*>(drow + 4 * c);
        f32x4 bx = decode_box(d, an, 10.f, 10.f, 5.f, 5.f);
        *reinterpret_cast<f32x4*>(boxes + (roi * NC + c) * 4) = clip_box(bx, img_h, img_w);
    }
}

// ================================================================ block primitives
template <int NT>
struct BlockScan {
    // exclusive prefix of `flag` over the block in thread order; *total = block sum.
    __device__ static int exclusive(int flag, int* wsum, int& total) {
        constexpr int NW = NT / 64;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const unsigned long long bal = __ballot(flag);
        const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(bal);
        __syncthreads();
        int base = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int v = wsum[i];
            base += (i < w) ? v : 0;
            tot += v;
        }
        __syncthreads();
        total = tot;
        return base + in_wave;
    }
};

// LDS layout of a segment kernel with capacity KC (power of two, >= 64).
template <int KC>
struct SegSmem {
    static constexpr int NWORDS = KC / 64;
    unsigned long long mask[KC * NWORDS];  // IoU bitmask rows
    unsigned long long keys[KC];           // sort keys (score << 32 | ~index)
    f32x4 box[KC];                         // candidate boxes in sorted order
    int aux[KC];                           // sort payload / group ids
    unsigned int hist[256];
    int wsum[32];
    int misc[8];
    unsigned char valid[KC];
};

__device__ __forceinline__ unsigned long long make_key(uint32_t k, uint32_t i) {
    return ((unsigned long long)k << 32) | (unsigned long long)(0xffffffffu - i);
}
__device__ __forceinline__ int key_index(unsigned long long key) {
    return (int)(0xffffffffu - (uint32_t)(key & 0xffffffffull));
}

// Block radix select: T = the K-th largest key among candidates with fkey(i, k) == true.
// misc[1] = number of valid candidates, misc[5] = how many keys == T belong to the top K.
// If valid <= K, returns 0 and misc[5] = 0 (take every valid candidate).
template <int NT, typename F>
__device__ uint32_t radix_select(int n, int K, F fkey, unsigned int* hist, int* misc) {
    if (threadIdx.x == 0) misc[0] = 0;
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < n; i += NT) {
        uint32_t k;
        if (fkey(i, k)) ++cnt;
    }
    atomicAdd(&misc[0], cnt);
    __syncthreads();
    const int nvalid = misc[0];
    if (nvalid <= K) {
        __syncthreads();
        if (threadIdx.x == 0) {
            misc[1] = nvalid;
            misc[5] = 0;
        }
        __syncthreads();
        return 0u;
    }
    uint32_t prefix = 0, pmask = 0;
    int remaining = K;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += NT) {
            uint32_t k;
            if (fkey(i, k) && (k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int acc = 0, d = 255;
            for (; d > 0; --d) {
                if (acc + (int)hist[d] >= remaining) break;
                acc += (int)hist[d];
            }
            misc[2] = d;
            misc[3] = remaining - acc;
        }
        __syncthreads();
        prefix |= (uint32_t)misc[2] << shift;
        pmask |= 255u << shift;
        remaining = misc[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        misc[1] = nvalid;
        misc[5] = remaining;
    }
    __syncthreads();
    return prefix;
}

// Ordered compaction into keys[]: every valid key > T (all valid when take_all) plus the first
// `eq_budget` keys == T in index order; at most `cap` written.  Returns the count.
template <int NT, typename F>
__device__ int compact(int n, uint32_t T, bool take_all, int eq_budget, int cap, F fkey, unsigned long long* keys,
                       int* wsum) {
    int written = 0, eq_taken = 0;
    for (int base = 0; base < n; base += NT) {
        const int i = base + threadIdx.x;
        uint32_t k = 0;
        const bool v = (i < n) && fkey(i, k);
        const bool gt = v && (take_all || k > T);
        const bool eq = v && !take_all && k == T;
        int tot_gt, tot_eq;
        const int pos_gt = BlockScan<NT>::exclusive(gt ? 1 : 0, wsum, tot_gt);
        const int pos_eq = BlockScan<NT>::exclusive(eq ? 1 : 0, wsum, tot_eq);
        const int budget = eq_budget - eq_taken;
        if (gt) {
            const int slot = written + pos_gt;
            if (slot < cap) keys[slot] = make_key(k, (uint32_t)i);
        }
        if (eq && pos_eq < budget) {
            const int slot = written + tot_gt + pos_eq;
            if (slot < cap) keys[slot] = make_key(k, (uint32_t)i);
        }
        const int eq_used = tot_eq < budget ? tot_eq : (budget > 0 ? budget : 0);
        written += tot_gt + eq_used;
        eq_taken += eq_used;
    }
    __syncthreads();
    return written < cap ? written : cap;
}

// Bitonic sort of keys[0..m) descending (padded with 0 sentinels to a power of two); the optional
// payload moves with its key.
template <int NT>
__device__ void bitonic_desc(unsigned long long* keys, int* payload, int m) {
    int p2 = 64;
    while (p2 < m) p2 <<= 1;
    for (int i = m + threadIdx.x; i < p2; i += NT) {
        keys[i] = 0ull;
        if (payload) payload[i] = -1;
    }
    __syncthreads();
    for (int k = 2; k <= p2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < p2 / 2; t += NT) {
                const int i = 2 * t - (t & (j - 1));
                const int l = i + j;
                const bool desc = (i & k) == 0;
                const unsigned long long a = keys[i], b = keys[l];
                if ((a < b) == desc) {
                    keys[i] = b;
                    keys[l] = a;
                    if (payload) {
                        const int pa = payload[i];
                        payload[i] = payload[l];
                        payload[l] = pa;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// IoU test in the op order of torchvision's CPU nms kernel; the float IoU is compared in double.
__device__ __forceinline__ bool iou_gt(f32x4 a, float area_a, f32x4 b, float area_b, double thr) {
    const float xx1 = fmaxf(a.x, b.x), yy1 = fmaxf(a.y, b.y);
    const float xx2 = fminf(a.z, b.z), yy2 = fminf(a.w, b.w);
    float w = xx2 - xx1;
    w = w > 0.f ? w : 0.f;
    float h = yy2 - yy1;
    h = h > 0.f ? h : 0.f;
    const float inter = w * h;
    const float ovr = inter / ((area_a + area_b) - inter);
    return (double)ovr > thr;
}

// Greedy NMS over S.box[0..m) in sorted order.  In: S.valid = candidate may be kept (invalid ones
// neither survive nor suppress).  Out: S.valid = kept.  If `groups`, only pairs with equal
// S.aux[] group ids interact (batched_nms).
template <int NT, int KC>
__device__ void nms_block(SegSmem<KC>& S, int m, double thr, bool groups) {
    constexpr int NWORDS = KC / 64;
    const int nw = (m + 63) >> 6;
    for (int t = threadIdx.x; t < m * nw; t += NT) {
        const int i = t / nw, w = t - (t / nw) * nw;
        unsigned long long bits = 0ull;
        if (w >= (i >> 6)) {
            const f32x4 bi = S.box[i];
            const float ai = (bi.z - bi.x) * (bi.w - bi.y);
            const int gi = groups ? S.aux[i] : 0;
            const int j0 = w * 64;
            const int jend = min(m, j0 + 64);
            for (int j = max(j0, i + 1); j < jend; ++j) {
                if (groups && S.aux[j] != gi) continue;
                const f32x4 bj = S.box[j];
                const float aj = (bj.z - bj.x) * (bj.w - bj.y);
                if (iou_gt(bi, ai, bj, aj, thr)) bits |= 1ull << (j - j0);
            }
        }
        S.mask[i * NWORDS + w] = bits;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        // lane w holds word w of the suppressed set; invalid candidates start suppressed
        unsigned long long removed = 0ull;
        if (lane < nw) {
            for (int jj = 0; jj < 64; ++jj) {
                const int j = lane * 64 + jj;
                if (j >= m || !S.valid[j]) removed |= 1ull << jj;
            }
        }
        for (int blk = 0; blk < nw; ++blk) {
            unsigned long long cur =
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(removed >> 32), blk) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(removed & 0xffffffffu), blk);
            const int row = blk * 64 + lane;
            const unsigned long long diag = row < m ? S.mask[row * NWORDS + blk] : 0ull;
            unsigned long long kept = 0ull;
            unsigned long long avail = ~cur;
            while (avail) {
                const int l = __builtin_ctzll(avail);  // earliest candidate still alive
                kept |= 1ull << l;
                const unsigned long long d =
                    ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(diag >> 32), l) << 32) |
                    (uint32_t)__builtin_amdgcn_readlane((int)(diag & 0xffffffffu), l);
                cur |= d | (1ull << l);
                if (l == 63) break;
                avail = ~cur & ~((2ull << l) - 1ull);
            }
            if (lane > blk && lane < nw) {
                unsigned long long kk = kept, acc = 0ull;
                while (kk) {
                    const int l = __builtin_ctzll(kk);
                    kk &= kk - 1ull;
                    acc |= S.mask[(blk * 64 + l) * NWORDS + lane];
                }
                removed |= acc;
            }
            if (row < m) S.valid[row] = (unsigned char)((kept >> lane) & 1ull);
        }
    }
    __syncthreads();
}

// Per-segment kept lists (records) consumed by merge_topk.

// Write the kept candidates of a segment in sorted order.  rec(t, slot_offset) writes one record.
template <int NT, int KC, typename W>
__device__ void write_kept(SegSmem<KC>& S, int m, int seg, const SegOut& out, W rec) {
    int written = 0;
    for (int base = 0; base < m; base += NT) {
        const int t = base + threadIdx.x;
        const bool kf = t < m && S.valid[t];
        int tot;
        const int pos = BlockScan<NT>::exclusive(kf ? 1 : 0, S.wsum, tot);
        if (kf && written + pos < out.kmax) rec(t, (int64_t)seg * out.kmax + written + pos);
        written += tot;
    }
    if (threadIdx.x == 0) out.count[seg] = written < out.kmax ? written : out.kmax;
}

// ================================================================ SSD per-class selection
// grid (NC-1, B): candidates = anchors with score > score_thresh, top `topk`, NMS.
template <int NT, int KC>
__global__ void __launch_bounds__(NT) ssd_class_nms_kernel(const float* __restrict__ scores_t,
                                                           const f32x4* __restrict__ boxes, int A, int NC,
                                                           float score_thresh, int topk, double iou, SegOut out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int c = blockIdx.x + 1;  // class 0 is background
    const int b = blockIdx.y;
    const float* sc = scores_t + ((int64_t)b * NC + c) * A;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        const float s = sc[i];
        k = __float_as_uint(s);  // probabilities are >= 0: raw bits are ordered
        return s > score_thresh;
    };
    const uint32_t T = radix_select<NT>(A, topk, fkey, S.hist, S.misc);
    const bool take_all = S.misc[1] <= topk;
    const int m = compact<NT>(A, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
    bitonic_desc<NT>(S.keys, nullptr, m);
    for (int t = threadIdx.x; t < m; t += NT) {
        S.box[t] = boxes[(int64_t)b * A + key_index(S.keys[t])];
        S.valid[t] = 1;
    }
    __syncthreads();
    nms_block<NT, KC>(S, m, iou, false);
    write_kept<NT, KC>(S, m, b * (NC - 1) + (c - 1), out, [&](int t, int64_t o) {
        out.box[o] = S.box[t];
        out.score[o] = __uint_as_float((uint32_t)(S.keys[t] >> 32));
        out.tb[o] = ((uint32_t)c << 16) | (uint32_t)t;  // concatenation order: (class, rank)
        out.label[o] = c;
    });
}

// ================================================================ RPN per-level selection

template <int NT, int KC>
__global__ void __launch_bounds__(NT) rpn_level_nms_kernel(RpnParams P, SegOut out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int l = blockIdx.x, b = blockIdx.y;
    const RpnLevel L = P.lv[l];
    const int HW = L.n / P.A;
    const float* hb = L.head + (int64_t)b * HW * P.ld;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        const int pix = i / P.A, a = i - pix * P.A;
        k = float_key(hb[(int64_t)pix * P.ld + a]);
        return true;
    };
    const uint32_t T = radix_select<NT>(L.n, P.topk, fkey, S.hist, S.misc);
    const bool take_all = S.misc[1] <= P.topk;
    const int m = compact<NT>(L.n, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
    bitonic_desc<NT>(S.keys, nullptr, m);
    for (int t = threadIdx.x; t < m; t += NT) {
        const int i = key_index(S.keys[t]);
        const int pix = i / P.A, a = i - pix * P.A;
        const float* row = hb + (int64_t)pix * P.ld + P.A + 4 * a;
        const f32x4 d = f32x4{row[0], row[1], row[2], row[3]};
        const f32x4 an = *reinterpret_cast<const f32x4*>(L.anchors + (int64_t)i * 4);
        const f32x4 bx = clip_box(decode_box(d, an, 1.f, 1.f, 1.f, 1.f), P.img_h, P.img_w);
        const float logit = key_float((uint32_t)(S.keys[t] >> 32));
        const float score = 1.f / (1.f + expf(-logit));
        S.box[t] = bx;
        S.valid[t] = ((bx.z - bx.x) >= P.min_size && (bx.w - bx.y) >= P.min_size && score >= P.score_thresh) ? 1 : 0;
    }
    __syncthreads();
    nms_block<NT, KC>(S, m, P.iou, false);
    write_kept<NT, KC>(S, m, b * P.nlevels + l, out, [&](int t, int64_t o) {
        const float logit = key_float((uint32_t)(S.keys[t] >> 32));
        out.box[o] = S.box[t];
        out.score[o] = 1.f / (1.f + expf(-logit));
        out.tb[o] = ((uint32_t)l << 16) | (uint32_t)t;  // concatenation order: (level, rank)
        out.label[o] = l;
    });
}

// ================================================================ RoIHeads per-class selection
template <int NT, int KC>
__global__ void __launch_bounds__(NT) box_class_nms_kernel(const float* __restrict__ scores,
                                                           const f32x4* __restrict__ boxes,
                                                           const int* __restrict__ counts, int R, int NC,
                                                           float score_thresh, float min_size, double iou,
                                                           SegOut out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int c = blockIdx.x + 1, b = blockIdx.y;
    const int n = counts[b];
    const float* sc = scores + (int64_t)b * R * NC + c;
    const f32x4* bx = boxes + (int64_t)b * R * NC + c;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        const float s = sc[(int64_t)i * NC];
        k = __float_as_uint(s);
        if (!(s > score_thresh)) return false;
        const f32x4 q = bx[(int64_t)i * NC];
        return (q.z - q.x) >= min_size && (q.w - q.y) >= min_size;
    };
    const int m = compact<NT>(n, 0u, true, 0, KC, fkey, S.keys, S.wsum);
    bitonic_desc<NT>(S.keys, nullptr, m);
    for (int t = threadIdx.x; t < m; t += NT) {
        S.box[t] = bx[(int64_t)key_index(S.keys[t]) * NC];
        S.valid[t] = 1;
    }
    __syncthreads();
    nms_block<NT, KC>(S, m, iou, false);
    write_kept<NT, KC>(S, m, b * (NC - 1) + (c - 1), out, [&](int t, int64_t o) {
        const int i = key_index(S.keys[t]);
        out.box[o] = S.box[t];
        out.score[o] = __uint_as_float((uint32_t)(S.keys[t] >> 32));
        out.tb[o] = ((uint32_t)i << 8) | (uint32_t)c;  // concatenation order: (roi, class)
        out.label[o] = c;
    });
}

// ================================================================ unit (batched) NMS for the C API
template <int NT, int KC>
__global__ void __launch_bounds__(NT) unit_nms_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                                                      const int64_t* __restrict__ idxs, int n, double iou,
                                                      int64_t* __restrict__ keep, int* __restrict__ num_keep) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    auto fkey = [&](int i, uint32_t& k) -> bool {
        k = float_key(scores[i]);
        return true;
    };
    const int m = compact<NT>(n, 0u, true, 0, KC, fkey, S.keys, S.wsum);
    bitonic_desc<NT>(S.keys, nullptr, m);
    for (int t = threadIdx.x; t < m; t += NT) {
        const int i = key_index(S.keys[t]);
        S.box[t] = *reinterpret_cast<const f32x4*>(boxes + (int64_t)i * 4);
        S.valid[t] = 1;
        S.aux[t] = idxs ? (int)idxs[i] : 0;
    }
    __syncthreads();
    nms_block<NT, KC>(S, m, iou, idxs != nullptr);
    int written = 0;
    for (int base = 0; base < m; base += NT) {
        const int t = base + threadIdx.x;
        const bool kf = t < m && S.valid[t];
        int tot;
        const int pos = BlockScan<NT>::exclusive(kf ? 1 : 0, S.wsum, tot);
        if (kf) keep[written + pos] = (int64_t)key_index(S.keys[t]);
        written += tot;
    }
    if (threadIdx.x == 0) *num_keep = written;
}

// ================================================================ per-image merge
// Kept lists [B][S][kmax] -> top N by (score desc, tiebreak asc), boxes rescaled by ratio.

template <int NT, int KC>
__global__ void __launch_bounds__(NT) merge_topk_kernel(MergeParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int b = blockIdx.x;
    const int n = P.S * P.kmax;
    const int* cnt = P.count + (int64_t)b * P.S;
    const int64_t base_off = (int64_t)b * P.S * P.kmax;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        const int s = i / P.kmax, slot = i - s * P.kmax;
        if (slot >= cnt[s]) return false;
        k = __float_as_uint(P.score[base_off + i]);  // scores >= 0
        return true;
    };
    const uint32_t T = radix_select<NT>(n, P.N, fkey, S.hist, S.misc);
    const bool take_all = S.misc[1] <= P.N;
    // every key > T plus all ties (up to capacity); ties are ordered by tiebreak in the sort
    const int m0 = compact<NT>(n, T, take_all, KC, KC, fkey, S.keys, S.wsum);
    for (int t = threadIdx.x; t < m0; t += NT) {
        const int i = key_index(S.keys[t]);
        S.aux[t] = i;
        S.keys[t] = make_key(__float_as_uint(P.score[base_off + i]), P.tb[base_off + i]);
    }
    __syncthreads();
    bitonic_desc<NT>(S.keys, S.aux, m0);
    const int m = m0 < P.N ? m0 : P.N;
    float rw = 1.f, rh = 1.f;
    if (P.ratio) {
        rw = P.ratio[2 * b];
        rh = P.ratio[2 * b + 1];
    }
    for (int t = threadIdx.x; t < m; t += NT) {
        const int i = S.aux[t];
        const f32x4 bx = P.box[base_off + i];
        const int64_t o = (int64_t)b * P.N + t;
        float* ob = P.out_box + o * 4;
        ob[0] = bx.x * rw;
        ob[1] = bx.y * rh;
        ob[2] = bx.z * rw;
        ob[3] = bx.w * rh;
        P.out_score[o] = P.score[base_off + i];
        if (P.out_label) P.out_label[o] = (int64_t)P.label[base_off + i];
    }
    if (threadIdx.x == 0) P.out_count[b] = m;
}

// ================================================================ host launchers
template <int KC>
static size_t seg_smem() {
    return sizeof(SegSmem<KC>);
}

// Opt a kernel into > 64 KiB of dynamic LDS once per process (not a stream operation, so it is
// also legal while a graph is being captured).
template <typename K>
static int set_lds(K kernel, size_t bytes) {
    static std::mutex mu;
    static std::vector<std::pair<const void*, size_t>> done;
    std::lock_guard<std::mutex> lk(mu);
    for (auto& d : done)
        if (d.first == (const void*)kernel && d.second >= bytes) return 0;
    EDGEDET_CHECK_HIP(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    done.emplace_back((const void*)kernel, bytes);
    return 0;
}

static bool seg_ok(const SegOut& o) { return o.box && o.score && o.tb && o.label && o.count && o.kmax > 0; }

int ssd_scores_launch(const float* logits, const float* reg, const float* anchors, float* scores_t, float* boxes,
                      int B, int A, int NC, float img_h, float img_w, hipStream_t s) {
    EDGEDET_REQUIRE(logits && reg && anchors && scores_t && boxes, "ssd_scores: null pointer");
    const int64_t total = (int64_t)B * A;
    hipLaunchKernelGGL(ssd_scores_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, logits, reg, anchors,
                       scores_t, boxes, B, A, NC, img_h, img_w);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int box_scores_launch(const float* pred, int ld, int cls_off, int delta_off, const float* props, const int* counts,
                      float* scores, float* boxes, int B, int R, int NC, float img_h, float img_w, hipStream_t s) {
    EDGEDET_REQUIRE(pred && props && counts && scores && boxes, "box_scores: null pointer");
    EDGEDET_REQUIRE(ld >= 5 * NC && ld % 4 == 0 && delta_off % 4 == 0, "box_scores: bad predictor layout");
    const int64_t total = (int64_t)B * R;
    hipLaunchKernelGGL(box_scores_kernel, dim3((unsigned)cdiv(total, 4)), dim3(256), 0, s, pred, ld, cls_off,
                       delta_off, props, counts, scores, boxes, B, R, NC, img_h, img_w);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int ssd_class_nms_launch(const float* scores_t, const float* boxes, int B, int A, int NC, float score_thresh,
                         int topk, double iou, SegOut out, hipStream_t s) {
    EDGEDET_REQUIRE(scores_t && boxes && seg_ok(out), "ssd_class_nms: null pointer");
    EDGEDET_REQUIRE(topk <= 512 && out.kmax >= topk, "ssd_class_nms: topk must be <= 512 and <= kmax");
    constexpr int KC = 512, NT = 256;
    auto k = ssd_class_nms_kernel<NT, KC>;
    if (set_lds(k, seg_smem<KC>())) return -2;
    hipLaunchKernelGGL(k, dim3(NC - 1, B), dim3(NT), seg_smem<KC>(), s, scores_t, (const f32x4*)boxes, A, NC,
                       score_thresh, topk, iou, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int rpn_level_nms_launch(const RpnParams& P, SegOut out, hipStream_t s) {
    EDGEDET_REQUIRE(P.topk <= 1024 && out.kmax >= P.topk, "rpn: topk must be <= 1024 and <= kmax");
    EDGEDET_REQUIRE(P.nlevels >= 1 && P.nlevels <= 5, "rpn: 1..5 levels");
    EDGEDET_REQUIRE(seg_ok(out), "rpn: null output records");
    for (int l = 0; l < P.nlevels; ++l)
        EDGEDET_REQUIRE(P.lv[l].head && P.lv[l].anchors && P.lv[l].n > 0, "rpn: null/empty level");
    constexpr int KC = 1024, NT = 512;
    auto k = rpn_level_nms_kernel<NT, KC>;
    if (set_lds(k, seg_smem<KC>())) return -2;
    hipLaunchKernelGGL(k, dim3(P.nlevels, P.B), dim3(NT), seg_smem<KC>(), s, P, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int box_class_nms_launch(const float* scores, const float* boxes, const int* counts, int B, int R, int NC,
                         float score_thresh, float min_size, double iou, SegOut out, hipStream_t s) {
    EDGEDET_REQUIRE(scores && boxes && counts && seg_ok(out), "box_class_nms: null pointer");
    EDGEDET_REQUIRE(R <= 1024 && out.kmax >= R, "box_class_nms: R must be <= 1024 and <= kmax");
    constexpr int KC = 1024, NT = 512;
    auto k = box_class_nms_kernel<NT, KC>;
    if (set_lds(k, seg_smem<KC>())) return -2;
    hipLaunchKernelGGL(k, dim3(NC - 1, B), dim3(NT), seg_smem<KC>(), s, scores, (const f32x4*)boxes, counts, R, NC,
                       score_thresh, min_size, iou, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int merge_topk_launch(const MergeParams& P, int B, hipStream_t s) {
    EDGEDET_REQUIRE(P.box && P.score && P.tb && P.label && P.count && P.out_box && P.out_score && P.out_count,
                    "merge_topk: null pointer");
    EDGEDET_REQUIRE(P.N <= 1024 && P.N > 0 && P.S > 0 && P.kmax > 0, "merge_topk: bad sizes");
    constexpr int KC = 1024, NT = 512;
    auto k = merge_topk_kernel<NT, KC>;
    if (set_lds(k, seg_smem<KC>())) return -2;
    hipLaunchKernelGGL(k, dim3(B), dim3(NT), seg_smem<KC>(), s, P);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

}  // namespace edgedet

using namespace edgedet;

extern "C" int edgedet_batched_nms(const float* boxes, const float* scores, const int64_t* idxs, int64_t n,
                                   double iou_threshold, int64_t* keep, int32_t* d_num_keep, void* stream) {
    EDGEDET_REQUIRE(n >= 0 && n <= 1024, "batched_nms: n must be in [0, 1024]");
    EDGEDET_REQUIRE(d_num_keep && (n == 0 || (boxes && scores && keep)), "batched_nms: null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        EDGEDET_CHECK_HIP(hipMemsetAsync(d_num_keep, 0, sizeof(int32_t), s));
        return 0;
    }
    constexpr int KC = 1024, NT = 512;
    auto k = unit_nms_kernel<NT, KC>;
    const size_t lds = seg_smem<KC>();
    if (set_lds(k, lds)) return -2;
    hipLaunchKernelGGL(k, dim3(1), dim3(NT), lds, s, boxes, scores, idxs, (int)n, iou_threshold, keep, d_num_keep);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

extern "C" int edgedet_nms(const float* boxes, const float* scores, int64_t n, double iou_threshold, int64_t* keep,
                           int32_t* d_num_keep, void* stream) {
    return edgedet_batched_nms(boxes, scores, nullptr, n, iou_threshold, keep, d_num_keep, stream);
}
