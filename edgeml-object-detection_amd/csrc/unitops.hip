// Unit operators of the C-ABI beyond the plan executor (SURVEY.md §8(b) "unit kernels for testing"):
//   edgedet_nms / edgedet_batched_nms for any n   torchvision::nms / ops.batched_nms (no size cap)
//   edgedet_topk_segments                         torch.topk per segment (RPN pre_nms_top_n, SSD per-class
//                                                 topk), values descending, ties lower index first
//   edgedet_box_decode                            BoxCoder.decode_single (+ clip_boxes_to_image)
// Same arithmetic as the plan's kernels (csrc/detect.hip: decode_box, clip_box, iou_gt, the tie rules),
// so the units and the model path agree bit for bit.
//
// Large-n NMS (n > 1024; smaller n take the single-workgroup kernel of detect.hip):
//   1. keys: float_key(score) (orderable uint32) + index, sorted descending by a stable device radix sort
//      (hipCUB): equal scores keep ascending index order, the reference's tie rule;
//   2. gather: boxes (and group ids) in sorted order;
//   3. mask: one wave per (64-row block, 64-column block) of the upper triangle writes, for each row i,
//      the 64-bit word of columns j > i it suppresses (iou_gt; groups must match for batched_nms);
//   4. scan: one workgroup walks the 64-row blocks in order: wave 0 resolves a block's greedy decisions
//      from the diagonal words (readlane, no memory traffic), then every thread ORs the kept rows' words
//      into the "removed" bitset (LDS) for the blocks to its right.  Kept indices go out in sorted
//      order (score descending, ties lower index), as torchvision returns them.
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <limits>

#include "kernels.hpp"

namespace edgedet {

// ---------------------------------------------------------------------------------------- shared math
constexpr float UNIT_BBOX_CLIP = 4.135166556742356f;  // log(1000/16) as float (detect.hip BBOX_CLIP)

__device__ __forceinline__ uint32_t unit_float_key(float x) {
    uint32_t u = __float_as_uint(x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// BoxCoder.decode_single, op order as torchvision (== detect.hip decode_box with a given clamp)
__device__ __forceinline__ f32x4 unit_decode(f32x4 d, f32x4 a, float wx, float wy, float ww, float wh, float clampv) {
    const float width = a.z - a.x;
    const float height = a.w - a.y;
    const float ctr_x = a.x + 0.5f * width;
    const float ctr_y = a.y + 0.5f * height;
    const float dx = d.x / wx;
    const float dy = d.y / wy;
    float dw = d.z / ww;
    float dh = d.w / wh;
    dw = fminf(dw, clampv);
    dh = fminf(dh, clampv);
    const float pcx = dx * width + ctr_x;
    const float pcy = dy * height + ctr_y;
    const float pw = expf(dw) * width;
    const float ph = expf(dh) * height;
    const float hw = 0.5f * pw;
    const float hh = 0.5f * ph;
    return f32x4{pcx - hw, pcy - hh, pcx + hw, pcy + hh};
}

// detect.hip iou_gt: `(double)RN_f32(inter / uni) > thr` evaluated exactly
__device__ __forceinline__ bool unit_iou_gt(f32x4 a, float area_a, f32x4 b, float area_b, const IouThr& t) {
    const float xx1 = fmaxf(a.x, b.x), yy1 = fmaxf(a.y, b.y);
    const float xx2 = fminf(a.z, b.z), yy2 = fminf(a.w, b.w);
    float w = xx2 - xx1;
    w = w > 0.f ? w : 0.f;
    float h = yy2 - yy1;
    h = h > 0.f ? h : 0.f;
    const float inter = w * h;
    const float uni = (area_a + area_b) - inter;
    if (uni > 0.f) {
        const double dl = (double)inter, dr = t.mid * (double)uni;
        return dl > dr || (dl == dr && t.tie_up);
    }
    return (double)(inter / uni) > t.thr;
}

// ---------------------------------------------------------------------------------------- large NMS
__global__ void nms_keys_kernel(const float* __restrict__ scores, int n, uint32_t* __restrict__ keys,
                                int* __restrict__ idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        keys[i] = unit_float_key(scores[i]);
        idx[i] = i;
    }
}

__global__ void nms_gather_kernel(const float* __restrict__ boxes, const int64_t* __restrict__ groups,
                                  const int* __restrict__ order, int n, f32x4* __restrict__ sbox,
                                  int64_t* __restrict__ sgrp) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) {
        const int i = order[t];
        sbox[t] = *reinterpret_cast<const f32x4*>(boxes + (int64_t)i * 4);
        if (groups) sgrp[t] = groups[i];
    }
}

// One workgroup per upper-triangle block (row block rb, column block cb >= rb): a 1-D grid of
// nw * (nw + 1) / 2 blocks, row-major over the triangle (row rb starts at S(rb) = rb * nw - rb * (rb - 1) / 2).
// One wave: lane = row rb*64 + lane.  (The lower triangle is never read: the scan uses words w >= b.)
__device__ __forceinline__ void tri_block(int64_t t, int nw, int& rb, int& cb) {
    const double a = 2.0 * nw + 1.0;
    int64_t r = (int64_t)((a - sqrt(a * a - 8.0 * (double)t)) * 0.5);
    auto S = [nw](int64_t q) { return q * nw - q * (q - 1) / 2; };
    while (r > 0 && S(r) > t) --r;        // the double root can be off by one either way
    while (r + 1 < nw && S(r + 1) <= t) ++r;
    rb = (int)r;
    cb = (int)(r + (t - S(r)));
}

__global__ void __launch_bounds__(64) nms_mask_kernel(const f32x4* __restrict__ sbox, const int64_t* __restrict__ sgrp,
                                                      int n, int nw, IouThr thr, unsigned long long* __restrict__ mask) {
    int rb, cb;
    tri_block((int64_t)blockIdx.x, nw, rb, cb);
    __shared__ f32x4 cbox[64];
    __shared__ float carea[64];
    __shared__ int64_t cgrp[64];
    const int lane = threadIdx.x;
    const int j = cb * 64 + lane;
    if (j < n) {
        const f32x4 b = sbox[j];
        cbox[lane] = b;
        carea[lane] = (b.z - b.x) * (b.w - b.y);
        cgrp[lane] = sgrp ? sgrp[j] : 0;
    }
    __syncthreads();
    const int i = rb * 64 + lane;
    if (i >= n) return;
    const f32x4 bi = sbox[i];
    const float ai = (bi.z - bi.x) * (bi.w - bi.y);
    const int64_t gi = sgrp ? sgrp[i] : 0;
    const int jend = min(64, n - cb * 64);
    unsigned long long bits = 0ull;
    for (int c = (cb == rb ? lane + 1 : 0); c < jend; ++c) {
        if (sgrp && cgrp[c] != gi) continue;
        if (unit_iou_gt(bi, ai, cbox[c], carea[c], thr)) bits |= 1ull << c;
    }
    mask[(int64_t)i * nw + cb] = bits;
}

constexpr int NMS_SCAN_NT = 1024;
constexpr int NMS_MAX_WORDS = 8192;  // removed bitset in LDS: n <= 524288

__global__ void __launch_bounds__(NMS_SCAN_NT) nms_scan_kernel(const unsigned long long* __restrict__ mask,
                                                               const int* __restrict__ order, int n, int nw,
                                                               int64_t* __restrict__ keep, int* __restrict__ num_keep) {
    __shared__ unsigned long long removed[NMS_MAX_WORDS];
    __shared__ unsigned long long kept_bits;
    __shared__ int kept_total;
    for (int w = threadIdx.x; w < nw; w += NMS_SCAN_NT) removed[w] = 0ull;
    if (threadIdx.x == 0) kept_total = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int b = 0; b < nw; ++b) {
        if (wid == 0) {
            const int r = b * 64 + lane;
            const unsigned long long diag = r < n ? mask[(int64_t)r * nw + b] : 0ull;
            const int rows = min(64, n - b * 64);
            unsigned long long rem = removed[b], kb = 0ull;
            for (int l = 0; l < rows; ++l) {  // uniform loop: every lane tracks the same state
                const unsigned long long d = ((unsigned long long)__shfl((int)(diag >> 32), l) << 32) |
                                             (unsigned int)__shfl((int)(diag & 0xffffffffull), l);
                if (!((rem >> l) & 1ull)) {
                    kb |= 1ull << l;
                    rem |= d;
                }
            }
            const int base = kept_total;
            if ((kb >> lane) & 1ull) {
                const int pos = base + __popcll(kb & ((1ull << lane) - 1ull));
                keep[pos] = (int64_t)order[r];
            }
            if (lane == 0) {
                kept_bits = kb;
                kept_total = base + __popcll(kb);
            }
        }
        __syncthreads();
        const unsigned long long kb = kept_bits;
        if (kb) {
            for (int w = b + 1 + (int)threadIdx.x; w < nw; w += NMS_SCAN_NT) {
                unsigned long long acc = removed[w];
                unsigned long long k = kb;
                while (k) {
                    const int l = __ffsll((long long)k) - 1;
                    k &= k - 1ull;
                    acc |= mask[(int64_t)(b * 64 + l) * nw + w];
                }
                removed[w] = acc;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *num_keep = kept_total;
}

struct NmsLayout {
    size_t keys_in, keys_out, idx_in, idx_out, sbox, sgrp, mask, temp, temp_bytes, total;
};

static size_t align256(size_t x) { return (x + 255) / 256 * 256; }

static int nms_layout(int64_t n, NmsLayout& L) {
    EDGEDET_REQUIRE(n >= 0 && n <= (int64_t)NMS_MAX_WORDS * 64, "nms: n must be in [0, 524288]");
    const int nw = (int)((n + 63) / 64);
    size_t tb = 0;
    EDGEDET_CHECK_HIP(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                                   (const int*)nullptr, (int*)nullptr, (int)n));
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = align256(off + bytes);
        return o;
    };
    L.keys_in = take(4 * (size_t)n);
    L.keys_out = take(4 * (size_t)n);
    L.idx_in = take(4 * (size_t)n);
    L.idx_out = take(4 * (size_t)n);
    L.sbox = take(16 * (size_t)n);
    L.sgrp = take(8 * (size_t)n);
    L.mask = take(8 * (size_t)n * nw);
    L.temp = take(tb);
    L.temp_bytes = tb;
    L.total = off;
    return 0;
}

static int large_nms(const float* boxes, const float* scores, const int64_t* idxs, int64_t n, double iou,
                     int64_t* keep, int32_t* d_num_keep, void* ws, int64_t ws_bytes, hipStream_t s) {
    NmsLayout L;
    if (int rc = nms_layout(n, L)) return rc;
    EDGEDET_REQUIRE(ws && ws_bytes >= (int64_t)L.total, "nms: workspace too small (edgedet_nms_workspace_size)");
    char* base = (char*)ws;
    uint32_t* kin = (uint32_t*)(base + L.keys_in);
    uint32_t* kout = (uint32_t*)(base + L.keys_out);
    int* iin = (int*)(base + L.idx_in);
    int* iout = (int*)(base + L.idx_out);
    f32x4* sbox = (f32x4*)(base + L.sbox);
    int64_t* sgrp = idxs ? (int64_t*)(base + L.sgrp) : nullptr;
    unsigned long long* mask = (unsigned long long*)(base + L.mask);
    const int N = (int)n, nw = (N + 63) / 64;
    hipLaunchKernelGGL(nms_keys_kernel, dim3((unsigned)cdiv(N, 256)), dim3(256), 0, s, scores, N, kin, iin);
    EDGEDET_LAUNCH_CHECK();
    size_t tb = L.temp_bytes;
    EDGEDET_CHECK_HIP(hipcub::DeviceRadixSort::SortPairsDescending(base + L.temp, tb, kin, kout, iin, iout, N, 0, 32, s));
    hipLaunchKernelGGL(nms_gather_kernel, dim3((unsigned)cdiv(N, 256)), dim3(256), 0, s, boxes, idxs, iout, N, sbox, sgrp);
    EDGEDET_LAUNCH_CHECK();
    hipLaunchKernelGGL(nms_mask_kernel, dim3((unsigned)((int64_t)nw * (nw + 1) / 2)), dim3(64), 0, s, sbox, sgrp, N, nw,
                       make_iou_thr(iou), mask);
    EDGEDET_LAUNCH_CHECK();
    hipLaunchKernelGGL(nms_scan_kernel, dim3(1), dim3(NMS_SCAN_NT), 0, s, mask, iout, N, nw, keep, d_num_keep);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------------------------------- top-k
// One workgroup per segment: repeated block-wide max extraction is too slow for k ~ 1000, so the
// segment's k-th largest key is found by a 4 x 8-bit radix select over the (key, index) space held in
// global memory, then the selected (key > T, plus ties == T in index order up to k) are sorted in LDS.
constexpr int TOPK_NT = 512, TOPK_CAP = 1024;

__global__ void __launch_bounds__(TOPK_NT) topk_segments_kernel(const float* __restrict__ values,
                                                                const int64_t* __restrict__ seg_off, int k,
                                                                float* __restrict__ out_val,
                                                                int64_t* __restrict__ out_idx, int* __restrict__ out_count) {
    __shared__ unsigned int hist[256];
    __shared__ int misc[4];
    __shared__ unsigned long long keys[TOPK_CAP];
    __shared__ int wsum[TOPK_NT / 64];
    const int seg = blockIdx.x;
    const int64_t lo = seg_off[seg], n64 = seg_off[seg + 1] - lo;
    const int n = (int)n64;
    const float* v = values + lo;
    const int K = k < n ? k : n;
    // 1. radix select of the K-th largest key
    uint32_t prefix = 0, pmask = 0;
    int remaining = K;
    const bool all = K == n;
    if (!all) {
        for (int shift = 24; shift >= 0; shift -= 8) {
            for (int i = threadIdx.x; i < 256; i += TOPK_NT) hist[i] = 0;
            __syncthreads();
            for (int i = threadIdx.x; i < n; i += TOPK_NT) {
                const uint32_t key = unit_float_key(v[i]);
                if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                int acc = 0, d = 255;
                for (; d > 0; --d) {
                    if (acc + (int)hist[d] >= remaining) break;
                    acc += (int)hist[d];
                }
                misc[0] = d;
                misc[1] = remaining - acc;
            }
            __syncthreads();
            prefix |= (uint32_t)misc[0] << shift;
            pmask |= 255u << shift;
            remaining = misc[1];
            __syncthreads();
        }
    }
    const uint32_t T = prefix;
    // 2. ordered compaction: keys > T, then the first `remaining` ties == T in index order
    int written = 0, eq_taken = 0;
    for (int base = 0; base < n; base += TOPK_NT) {
        const int i = base + (int)threadIdx.x;
        const uint32_t key = i < n ? unit_float_key(v[i]) : 0u;
        const bool gt = i < n && (all || key > T);
        const bool eq = i < n && !all && key == T;
        const unsigned long long bg = __ballot(gt), be = __ballot(eq);
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        if (lane == 0) wsum[wid] = __popcll(bg) | (__popcll(be) << 16);
        __syncthreads();
        int pg = 0, pe = 0, tg = 0, te = 0;
        for (int w = 0; w < TOPK_NT / 64; ++w) {
            const int c = wsum[w];
            if (w < wid) {
                pg += c & 0xffff;
                pe += c >> 16;
            }
            tg += c & 0xffff;
            te += c >> 16;
        }
        const unsigned long long below = (1ull << lane) - 1ull;
        pg += __popcll(bg & below);
        pe += __popcll(be & below);
        if (gt && written + pg < TOPK_CAP) keys[written + pg] = ((unsigned long long)key << 32) | (0xffffffffu - (uint32_t)i);
        const int budget = all ? 0 : remaining - eq_taken;
        if (eq && pe < budget && written + tg + pe < TOPK_CAP)
            keys[written + tg + pe] = ((unsigned long long)key << 32) | (0xffffffffu - (uint32_t)i);
        const int used = te < budget ? te : (budget > 0 ? budget : 0);
        written += tg + used;
        eq_taken += used;
        __syncthreads();
    }
    const int m = written < K ? written : K;
    // 3. bitonic sort descending (key desc, index asc)
    int p2 = 64;
    while (p2 < m) p2 <<= 1;
    for (int i = m + threadIdx.x; i < p2; i += TOPK_NT) keys[i] = 0ull;
    __syncthreads();
    for (int kk = 2; kk <= p2; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < p2 / 2; t += TOPK_NT) {
                const int i = 2 * t - (t & (j - 1));
                const int l = i + j;
                const bool desc = (i & kk) == 0;
                const unsigned long long a = keys[i], b = keys[l];
                if ((a < b) == desc) {
                    keys[i] = b;
                    keys[l] = a;
                }
            }
            __syncthreads();
        }
    for (int t = threadIdx.x; t < m; t += TOPK_NT) {
        const int i = (int)(0xffffffffu - (uint32_t)(keys[t] & 0xffffffffull));
        out_val[(int64_t)seg * k + t] = v[i];
        out_idx[(int64_t)seg * k + t] = i;
    }
    if (threadIdx.x == 0) out_count[seg] = m;
}

// ---------------------------------------------------------------------------------------- decode
__global__ void box_decode_kernel(const float* __restrict__ deltas, const float* __restrict__ refs, int64_t n,
                                  float wx, float wy, float ww, float wh, float clampv, float img_h, float img_w,
                                  float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f32x4 d = *reinterpret_cast<const f32x4*>(deltas + 4 * i);
    const f32x4 a = *reinterpret_cast<const f32x4*>(refs + 4 * i);
    f32x4 b = unit_decode(d, a, wx, wy, ww, wh, clampv);
    if (img_h > 0.f && img_w > 0.f) {
        b.x = fminf(fmaxf(b.x, 0.f), img_w);
        b.y = fminf(fmaxf(b.y, 0.f), img_h);
        b.z = fminf(fmaxf(b.z, 0.f), img_w);
        b.w = fminf(fmaxf(b.w, 0.f), img_h);
    }
    *reinterpret_cast<f32x4*>(out + 4 * i) = b;
}

int unit_small_nms(const float* boxes, const float* scores, const int64_t* idxs, int64_t n, double iou, int64_t* keep,
                   int32_t* d_num_keep, hipStream_t s);  // detect.hip (n <= 1024)

}  // namespace edgedet

using namespace edgedet;

extern "C" int64_t edgedet_nms_workspace_size(int64_t n) {
    if (n <= 1024) return 0;
    NmsLayout L;
    if (nms_layout(n, L)) return -1;
    return (int64_t)L.total;
}

extern "C" int edgedet_batched_nms_ws(const float* boxes, const float* scores, const int64_t* idxs, int64_t n,
                                      double iou_threshold, int64_t* keep, int32_t* d_num_keep, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
    EDGEDET_REQUIRE(n >= 0, "batched_nms: n must be >= 0");
    EDGEDET_REQUIRE(d_num_keep && (n == 0 || (boxes && scores && keep)), "batched_nms: null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (n <= 1024) return unit_small_nms(boxes, scores, idxs, n, iou_threshold, keep, d_num_keep, s);
    return large_nms(boxes, scores, idxs, n, iou_threshold, keep, d_num_keep, workspace, workspace_bytes, s);
}

extern "C" int edgedet_nms_ws(const float* boxes, const float* scores, int64_t n, double iou_threshold, int64_t* keep,
                              int32_t* d_num_keep, void* workspace, int64_t workspace_bytes, void* stream) {
    return edgedet_batched_nms_ws(boxes, scores, nullptr, n, iou_threshold, keep, d_num_keep, workspace,
                                  workspace_bytes, stream);
}

// torchvision::nms's signature: above 1024 boxes the scratch comes from the stream-ordered allocator
// (hipMallocAsync / hipFreeAsync on `stream`, no device synchronisation).
extern "C" int edgedet_batched_nms(const float* boxes, const float* scores, const int64_t* idxs, int64_t n,
                                   double iou_threshold, int64_t* keep, int32_t* d_num_keep, void* stream) {
    EDGEDET_REQUIRE(n >= 0, "batched_nms: n must be >= 0");
    if (n <= 1024)
        return edgedet_batched_nms_ws(boxes, scores, idxs, n, iou_threshold, keep, d_num_keep, nullptr, 0, stream);
    const int64_t bytes = edgedet_nms_workspace_size(n);
    if (bytes < 0) return -1;
    hipStream_t s = (hipStream_t)stream;
    void* ws = nullptr;
    EDGEDET_CHECK_HIP(hipMallocAsync(&ws, (size_t)bytes, s));
    const int rc = edgedet_batched_nms_ws(boxes, scores, idxs, n, iou_threshold, keep, d_num_keep, ws, bytes, stream);
    const hipError_t e = hipFreeAsync(ws, s);
    if (rc) return rc;
    EDGEDET_CHECK_HIP(e);
    return 0;
}

extern "C" int edgedet_nms(const float* boxes, const float* scores, int64_t n, double iou_threshold, int64_t* keep,
                           int32_t* d_num_keep, void* stream) {
    return edgedet_batched_nms(boxes, scores, nullptr, n, iou_threshold, keep, d_num_keep, stream);
}

extern "C" int edgedet_topk_segments(const float* values, const int64_t* seg_off, int64_t nseg, int32_t k,
                                     float* out_values, int64_t* out_index, int32_t* out_count, void* stream) {
    EDGEDET_REQUIRE(nseg >= 0 && nseg < (1ll << 31), "topk_segments: bad segment count");
    EDGEDET_REQUIRE(k >= 1 && k <= TOPK_CAP, "topk_segments: k must be in [1, 1024]");
    if (nseg == 0) return 0;
    EDGEDET_REQUIRE(values && seg_off && out_values && out_index && out_count, "topk_segments: null pointer");
    hipLaunchKernelGGL(topk_segments_kernel, dim3((unsigned)nseg), dim3(TOPK_NT), 0, (hipStream_t)stream, values, seg_off,
                       k, out_values, out_index, out_count);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

extern "C" int edgedet_box_decode(const float* deltas, const float* ref_boxes, int64_t n, float wx, float wy, float ww,
                                  float wh, float clamp, float img_h, float img_w, float* out, void* stream) {
    EDGEDET_REQUIRE(n >= 0, "box_decode: n must be >= 0");
    if (n == 0) return 0;
    EDGEDET_REQUIRE(deltas && ref_boxes && out, "box_decode: null pointer");
    EDGEDET_REQUIRE(((uintptr_t)deltas | (uintptr_t)ref_boxes | (uintptr_t)out) % 16 == 0, "box_decode: 16-byte rows");
    hipLaunchKernelGGL(box_decode_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, deltas,
                       ref_boxes, n, wx, wy, ww, wh, clamp, img_h, img_w, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}
