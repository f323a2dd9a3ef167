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
#include <cmath>
#include <cstring>
#include <limits>
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
// Block = 64 consecutive anchors x 4 waves.  The 64 x NC logits tile is one contiguous span: it is
// loaded coalesced into LDS (odd row pitch: conflict-free column reads); wave q reduces classes
// c = q (mod 4) of all 64 anchors, and writes them class-major (scores_t [B][NC][A]: 64 consecutive
// anchors per store, coalesced) for the per-class selection.  reg [B][A][4] + anchors [A][4] ->
// boxes [B][A][4] (decode + clip) by wave 0.
constexpr int SSD_MAXNC = 128;

__global__ void __launch_bounds__(256) ssd_scores_kernel(const float* __restrict__ logits, const float* __restrict__ reg,
                                                         const float* __restrict__ anchors, float* __restrict__ scores_t,
                                                         float* __restrict__ boxes, int B, int A, int NC, float img_h,
                                                         float img_w) {
    __shared__ float tile[64 * (SSD_MAXNC + 1)];
    __shared__ float red[4][64];
    const int b = blockIdx.y;
    const int a0 = blockIdx.x * 64;
    const int na = min(64, A - a0);
    const int ld = (NC & 1) ? NC : NC + 1;
    const float* src = logits + ((int64_t)b * A + a0) * NC;
    if (ld == NC) {
        stage_lds<256, 8>(tile, na * NC, [&](int e) { return src[e]; });
    } else {
        for (int e = threadIdx.x; e < na * NC; e += 256) {
            const int a = e / NC, c = e - a * NC;
            tile[a * ld + c] = src[e];
        }
    }
    __syncthreads();
    const int a = threadIdx.x & 63, q = threadIdx.x >> 6;
    const float* row = tile + a * ld;
    float mx = -__builtin_inff();
    for (int c = q; c < NC; c += 4) mx = fmaxf(mx, row[c]);
    red[q][a] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0][a], red[1][a]), fmaxf(red[2][a], red[3][a]));
    __syncthreads();
    float sum = 0.f;
    float* rw = tile + a * ld;  // each exponential computed once: (a, c) belongs to this thread alone
    for (int c = q; c < NC; c += 4) {
        const float e = expf(rw[c] - mx);
        rw[c] = e;
        sum += e;
    }
    red[q][a] = sum;
    __syncthreads();
    sum = ((red[0][a] + red[1][a]) + red[2][a]) + red[3][a];
    const float inv = 1.f / sum;
    if (a < na) {
        float* st = scores_t + (int64_t)b * NC * A + a0 + a;
        for (int c = q; c < NC; c += 4) st[(int64_t)c * A] = rw[c] * inv;
        if (q == 0) {
            const int64_t idx = (int64_t)b * A + a0 + a;
            const f32x4 d = *reinterpret_cast<const f32x4*>(reg + idx * 4);
            const f32x4 an = *reinterpret_cast<const f32x4*>(anchors + (int64_t)(a0 + a) * 4);
            f32x4 bx = decode_box(d, an, 10.f, 10.f, 5.f, 5.f);
            *reinterpret_cast<f32x4*>(boxes + idx * 4) = clip_box(bx, img_h, img_w);
        }
    }
}

// ================================================================ FRCNN RoIHeads: softmax + decode
constexpr int BOX_MAXNC = 128;
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
    float sum = 0.f, ex[BOX_MAXNC / 64];  // each exponential computed once (NC <= BOX_MAXNC)
#pragma unroll
    for (int u = 0; u < BOX_MAXNC / 64; ++u) {
        const int c = lane + 64 * u;
        ex[u] = c < NC ? expf(row[c] - mx) : 0.f;
        if (c < NC) sum += ex[u];
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.f / sum;
    const f32x4 an = *reinterpret_cast<const f32x4*>(props + roi * 4);
#pragma unroll
    for (int u = 0; u < BOX_MAXNC / 64; ++u) {
        const int c = lane + 64 * u;
        if (c >= NC) continue;
        scores[roi * NC + c] = ex[u] * inv;
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
    // exclusive prefix of an integer per thread (thread order); *total = block sum.
    __device__ static int exclusive_sum(int v, int* wsum, int& total) {
        constexpr int NW = NT / 64;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        int inc = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(inc, off);
            if (lane >= off) inc += t;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        int base = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int x = wsum[i];
            base += (i < w) ? x : 0;
            tot += x;
        }
        __syncthreads();
        total = tot;
        return base + inc - v;
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
    int misc[32];
    unsigned char valid[KC];
};

template <int KC>
struct SelSmem {  // selection-only kernels: no mask / box image
    unsigned long long keys[KC];
    unsigned int hist[256];
    int wsum[32];
    int misc[32];
    int red[64];
    unsigned long long run[KC];  // rank_sort_desc
};

__device__ __forceinline__ unsigned long long make_key(uint32_t k, uint32_t i) {
    return ((unsigned long long)k << 32) | (unsigned long long)(0xffffffffu - i);
}
__device__ __forceinline__ int key_index(unsigned long long key) {
    return (int)(0xffffffffu - (uint32_t)(key & 0xffffffffull));
}

// Keys are produced by fkey(i, k) -> valid.  Every pass below evaluates U keys per thread before
// using any of them (indices clamped, loads unconditional and pinned with an empty asm so the
// compiler cannot sink them back under the bounds test): U memory round trips overlap instead of
// one dependent round trip per element.
constexpr int KEY_U = 8;

template <int NT, typename F, typename G>
__device__ __forceinline__ void for_keys(int n, F fkey, G body) {
    for (int base = 0; base < n; base += NT * KEY_U) {
        uint32_t k[KEY_U];
        bool v[KEY_U];
#pragma unroll
        for (int u = 0; u < KEY_U; ++u) {
            const int i = base + u * NT + (int)threadIdx.x;
            v[u] = fkey(i < n ? i : n - 1, k[u]);
        }
#pragma unroll
        for (int u = 0; u < KEY_U; ++u) {
            asm volatile("" : "+v"(k[u]));
            const int i = base + u * NT + (int)threadIdx.x;
            body(v[u] & (i < n), k[u]);
        }
    }
}

// Block radix select: T = the K-th largest key among candidates with fkey(i, k) == true.
// misc[1] = number of valid candidates, misc[5] = how many keys == T belong to the top K.
// If valid <= K, returns 0 and misc[5] = 0 (take every valid candidate).
template <int NT, typename F>
__device__ uint32_t radix_select(int n, int K, F fkey, unsigned int* hist, int* misc) {
    if (threadIdx.x == 0) misc[0] = 0;
    __syncthreads();
    int cnt = 0;
    for_keys<NT>(n, fkey, [&](bool v, uint32_t) { cnt += v ? 1 : 0; });
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
        for_keys<NT>(n, fkey, [&](bool v, uint32_t k) {
            if (v && (k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        });
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

// Register-resident top-K selection (no atomics).  Element i = threadIdx.x + NT*j lives in
// kr[j] (key 0 = invalid; valid keys must be > 0).  The K-th largest key T is found by bisection on
// the key space: each probe counts keys >= t with one ballot + popcount per register (wave totals
// in SGPRs) and one barrier.  Then ordered compaction writes every key > T plus the first ties
// == T in index order (the reference's stable order) into keys[] (at most cap).  Returns the count.
template <int NT>
__device__ __forceinline__ int block_sum_uniform(int wave_val, int* red) {
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wave_val;
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) tot += red[w];
    __syncthreads();
    return tot;
}

// count of keys >= t over one wave: one ballot + popcount per register, the popcounts summed in four
// independent chains (written as one running sum, the compiler emits a serial chain of dependent
// s_add, which then sets a probe's latency)
template <int PER>
__device__ __forceinline__ int wave_count_ge(const uint32_t (&kr)[PER], uint32_t t) {
    int n0 = 0, n1 = 0, n2 = 0, n3 = 0;
#pragma unroll
    for (int j = 0; j < PER; j += 4) {
        n0 += __popcll(__ballot(kr[j] >= t));
        if (j + 1 < PER) n1 += __popcll(__ballot(kr[j + 1] >= t));
        if (j + 2 < PER) n2 += __popcll(__ballot(kr[j + 2] >= t));
        if (j + 3 < PER) n3 += __popcll(__ballot(kr[j + 3] >= t));
        asm volatile("" : "+s"(n0), "+s"(n1), "+s"(n2), "+s"(n3));  // keeps the four chains apart
    }
    return (n0 + n1) + (n2 + n3);
}

// count of keys >= t over the block.  red holds 2 x NW slots used alternately by successive calls
// (`parity`), so one barrier per probe suffices: a wave cannot rewrite a slot set before every wave
// has passed the barrier that follows the next probe's write.
template <int NT, int PER>
__device__ __forceinline__ int count_ge(const uint32_t (&kr)[PER], uint32_t t, int* red, int& parity) {
    constexpr int NW = NT / 64;
    const int c = wave_count_ge<PER>(kr, t);
    int* r = red + parity * NW;
    parity ^= 1;
    if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = c;
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += r[w];
    return tot;
}

// block min of the valid (nonzero) keys and block max, in one exchange (2 x NW slots of red)
template <int NT>
__device__ __forceinline__ void block_minmax_u32(uint32_t& mn, uint32_t& mx, int* red) {
    constexpr int NW = NT / 64;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t a = (uint32_t)__shfl_xor((int)mn, o), b = (uint32_t)__shfl_xor((int)mx, o);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = (int)mn;
        red[NW + (threadIdx.x >> 6)] = (int)mx;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        mn = (uint32_t)red[w] < mn ? (uint32_t)red[w] : mn;
        mx = (uint32_t)red[NW + w] > mx ? (uint32_t)red[NW + w] : mx;
    }
    __syncthreads();
}

// kmin < K relaxes the selection to "some prefix of the order": the bisection stops at the first
// probe t with kmin <= count(>= t) <= K and every key >= t is taken (ties whole), which is all a
// caller that consumes candidates in global order, round by round, needs.
// red: 4 x NT / 64 slots (2 x NW for the double-buffered counts, 2 x NW for block_minmax_u32).
template <int NT, int PER, int NR>
__device__ int select_topk_regs(const uint32_t (&kr)[PER], int K, int cap, unsigned long long* keys, int* wsum,
                                int (&red)[NR], bool all_ties = false, int kmin = -1, int* nvalid_out = nullptr) {
    static_assert(NR >= 4 * (NT / 64), "select_topk_regs: red needs 4 x NT / 64 slots");
    int parity = 0;
    const int nvalid = count_ge<NT, PER>(kr, 1u, red, parity);
    if (nvalid_out) *nvalid_out = nvalid;
    uint32_t T = 1u;
    int need_eq = 0;
    const bool take_all = nvalid <= K;
    if (!take_all) {
        uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            kmn = kr[j] != 0u && kr[j] < kmn ? kr[j] : kmn;
            kmx = kr[j] > kmx ? kr[j] : kmx;
        }
        block_minmax_u32<NT>(kmn, kmx, red + 2 * (NT / 64));  // red: 4 x NW slots
        // bisection on [min, max + 1): count(>= lo) >= K > count(>= hi)  (count(>= min) = nvalid > K)
        uint64_t lo = kmn, hi = (uint64_t)kmx + 1;
        bool prefix = false;
        while (hi - lo > 1) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            const int c = count_ge<NT, PER>(kr, (uint32_t)mid, red, parity);
            if (c >= kmin && c <= K && kmin >= 0) {  // uniform: c is a block total
                lo = mid;
                prefix = true;
                break;
            }
            if (c >= K) lo = mid;
            else hi = mid;
        }
        if (prefix) {
            T = (uint32_t)lo - 1u;  // keys > T are exactly the keys >= the probe; no partial ties
            need_eq = 0;
        } else {
            T = (uint32_t)lo;
            const int greater = (hi >> 32) ? 0 : count_ge<NT, PER>(kr, (uint32_t)hi, red, parity);
            need_eq = all_ties ? cap : K - greater;
        }
    }
    __syncthreads();
    // Compaction.  Callers sort the selected keys, so keys > T go out in any order: one scan of
    // per-thread counts.  Ties == T are taken whole when they fit the budget; otherwise the first
    // need_eq of them in index order (element i = threadIdx.x + NT * j), with per-register scans.
    int ngt = 0, neq = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t k = kr[j];
        ngt += (take_all ? (k >= 1u) : (k > T)) ? 1 : 0;
        neq += (!take_all && k == T) ? 1 : 0;
    }
    int tot_gt, tot_eq;
    int w = BlockScan<NT>::exclusive_sum(ngt, wsum, tot_gt);
    const int pos_eq = BlockScan<NT>::exclusive_sum(neq, wsum, tot_eq);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t k = kr[j];
        if (take_all ? (k >= 1u) : (k > T)) {
            if (w < cap) keys[w] = make_key(k, threadIdx.x + (uint32_t)NT * j);
            ++w;
        }
    }
    int written = tot_gt;
    if (tot_eq <= need_eq) {
        int e = tot_gt + pos_eq;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t k = kr[j];
            if (!take_all && k == T) {
                if (e < cap) keys[e] = make_key(k, threadIdx.x + (uint32_t)NT * j);
                ++e;
            }
        }
        written += tot_eq;
    } else if (need_eq > 0) {
        int eq_taken = 0;
        // unrolled (kr stays in registers: a runtime index into it would move the whole array to
        // scratch); the break is uniform (eq_taken is a block total)
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const bool eq = kr[j] == T;
            int tj;
            const int pe = BlockScan<NT>::exclusive(eq ? 1 : 0, wsum, tj);
            const int budget = need_eq - eq_taken;
            if (eq && pe < budget && written + eq_taken + pe < cap)
                keys[written + eq_taken + pe] = make_key(kr[j], threadIdx.x + (uint32_t)NT * j);
            eq_taken += tj < budget ? tj : (budget > 0 ? budget : 0);
            if (eq_taken >= need_eq) break;
        }
        written += eq_taken;
    }
    __syncthreads();
    return written < cap ? written : cap;
}

// Ordered compaction into keys[]: every valid key > T (all valid when take_all) plus the first
// `eq_budget` keys == T in index order; at most `cap` written.  Returns the count.  Each batch
// gives thread t the KEY_U consecutive indices base + t*KEY_U + u (loads issued together), so one
// block scan of per-thread counts orders the batch.
template <int NT, typename F>
__device__ int compact(int n, uint32_t T, bool take_all, int eq_budget, int cap, F fkey, unsigned long long* keys,
                       int* wsum) {
    int written = 0, eq_taken = 0;
    for (int base = 0; base < n; base += NT * KEY_U) {
        uint32_t k[KEY_U];
        bool v[KEY_U];
#pragma unroll
        for (int u = 0; u < KEY_U; ++u) {
            const int i = base + (int)threadIdx.x * KEY_U + u;
            v[u] = fkey(i < n ? i : n - 1, k[u]);
        }
        int ngt = 0, neq = 0;
#pragma unroll
        for (int u = 0; u < KEY_U; ++u) {
            asm volatile("" : "+v"(k[u]));
            const int i = base + (int)threadIdx.x * KEY_U + u;
            v[u] = v[u] & (i < n);
            ngt += (v[u] && (take_all || k[u] > T)) ? 1 : 0;
            neq += (v[u] && !take_all && k[u] == T) ? 1 : 0;
        }
        int tot_gt, tot_eq;
        int pos_gt = BlockScan<NT>::exclusive_sum(ngt, wsum, tot_gt);
        int pos_eq = BlockScan<NT>::exclusive_sum(neq, wsum, tot_eq);
        const int budget = eq_budget - eq_taken;
#pragma unroll
        for (int u = 0; u < KEY_U; ++u) {
            const uint32_t i = (uint32_t)(base + (int)threadIdx.x * KEY_U + u);
            if (v[u] && (take_all || k[u] > T)) {
                const int slot = written + pos_gt++;
                if (slot < cap) keys[slot] = make_key(k[u], i);
            } else if (v[u] && !take_all && k[u] == T) {
                if (pos_eq < budget) {
                    const int slot = written + tot_gt + pos_eq;
                    if (slot < cap) keys[slot] = make_key(k[u], i);
                }
                ++pos_eq;
            }
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

// Sort of keys[0..m) descending for m <= U * NT (U keys per thread: key tid + NT * u), two barriers:
// each 64-key run (the keys of one wave's slot u) is ranked within itself (a readlane walk: keys
// greater, equal keys at lower lanes first) and written sorted into run[]; a key's final position is
// its rank in its own run plus, for every other run, the number of that run's keys ahead of it
// (binary search; equal keys: the earlier run first).  Keys past m are zeros and sort last.
// Replaces the 45 (512 keys) / 55 (1,024) barrier stages of a bitonic sort.
template <int NT, int U = 1>
__device__ void rank_sort_desc(unsigned long long* keys, unsigned long long* run, int m) {
    constexpr int NR = U * NT / 64;  // runs
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    unsigned long long k[U];
    int r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = tid + NT * u, rid = e >> 6;
        k[u] = e < m ? keys[e] : 0ull;
        r[u] = lane;
        if (64 * rid < m) {  // wave-uniform: runs wholly past m hold zeros in lane order
            const uint32_t klo = (uint32_t)k[u], khi = (uint32_t)(k[u] >> 32);
            int c = 0;
#pragma unroll 16
            for (int j = 0; j < 64; ++j) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)klo, j);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)khi, j);
                const unsigned long long kj = ((unsigned long long)hi << 32) | lo;
                c += (kj > k[u] || (kj == k[u] && j < lane)) ? 1 : 0;
            }
            r[u] = c;
        }
        run[64 * rid + r[u]] = k[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = tid + NT * u, rid = e >> 6;
        int pos = r[u];
        for (int v = 0; v < NR; ++v) {
            if (v == rid || 64 * v >= m) continue;  // a run wholly past m holds only zeros, after every key
            const unsigned long long* rv = run + 64 * v;
            int lo = 0;
#pragma unroll
            for (int st = 64; st >= 1; st >>= 1) {
                if (lo + st <= 64) {
                    const unsigned long long x = rv[lo + st - 1];
                    if (x > k[u] || (x == k[u] && v < rid)) lo += st;
                }
            }
            pos += lo;
        }
        if (e < m) keys[pos] = k[u];
    }
    __syncthreads();
}

// IoU threshold test, bit-exact with torchvision's CPU nms: `(double)RN_f32(inter / uni) > thr`, where
// inter and uni = (area_i + area_j) - inter are computed in float in the reference's op order.  The
// float division is replaced by an exact comparison: with t1 = the smallest float > thr and t0 its
// predecessor, RN(x) > thr <=> x > mid(t0, t1), or x == mid and round-half-even picks t1.  mid has
// <= 25 significant bits, so mid * uni is exact in double and so is the comparison (uni > 0; other
// cases keep the division).  See make_iou_thr.
__device__ __forceinline__ bool iou_gt(f32x4 a, float area_a, f32x4 b, float area_b, const IouThr& t) {
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

// unrolled 8: overlaps the LDS reads of consecutive boxes j (RPN level-0 NMS 758k -> 715k cycles)
// Greedy NMS over S.box[0..m) in sorted order.  In: S.valid = candidate may be kept (invalid ones
// neither survive nor suppress).  Out: S.valid = kept.  If `groups`, only pairs with equal
// S.aux[] group ids interact (batched_nms).
// The greedy scan of a segment's suppression mask (rows of NWORDS 64-bit words, word w of row i: the
// later candidates j in [64w, 64w + 64) that i suppresses; only words w >= i / 64 are read).  In:
// valid[j] = candidate may be kept (invalid ones neither survive nor suppress).  Out: valid = kept.
// Run by one wave (threads 0..63 of the caller).
template <int KC>
__device__ __forceinline__ void nms_scan(const unsigned long long* __restrict__ mask, unsigned char* valid, int m) {
    constexpr int NWORDS = KC / 64;
    const int nw = (m + 63) >> 6;
    const int lane = threadIdx.x;
    // lane w holds word w of the suppressed set; invalid candidates start suppressed
    unsigned long long removed = 0ull;
    if (lane < nw) {
        for (int jj = 0; jj < 64; ++jj) {
            const int j = lane * 64 + jj;
            if (j >= m || !valid[j]) removed |= 1ull << jj;
        }
    }
    for (int blk = 0; blk < nw; ++blk) {
        unsigned long long cur =
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(removed >> 32), blk) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(removed & 0xffffffffu), blk);
        const int row = blk * 64 + lane;
        const unsigned long long diag = row < m ? mask[row * NWORDS + blk] : 0ull;
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
            // the kept rows' words, eight loads in flight at a time (a row taken twice ORs the same bits)
            unsigned long long kk = kept, acc = 0ull;
            while (kk) {
                int ls[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    ls[u] = kk ? __builtin_ctzll(kk) : ls[0];
                    kk &= kk - 1ull;
                }
                unsigned long long v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = mask[(blk * 64 + ls[u]) * NWORDS + lane];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc |= v[u];
            }
            removed |= acc;
        }
        if (row < m) valid[row] = (unsigned char)((kept >> lane) & 1ull);
    }
}

// Word w of mask row i over the candidate boxes bx[0..m) (sorted order): bit j - 64w set when j > i
// overlaps i beyond the threshold (same group only, if groups).
__device__ __forceinline__ unsigned long long nms_mask_word(const f32x4* bx, const int* grp, int m, int i, int w,
                                                            const IouThr& thr) {
    unsigned long long bits = 0ull;
    const f32x4 bi = bx[i];
    const float ai = (bi.z - bi.x) * (bi.w - bi.y);
    const int gi = grp ? grp[i] : 0;
    const int j0 = w * 64;
    const int jend = min(m, j0 + 64);
#pragma unroll 8
    for (int j = max(j0, i + 1); j < jend; ++j) {
        if (grp && grp[j] != gi) continue;
        const f32x4 bj = bx[j];
        const float aj = (bj.z - bj.x) * (bj.w - bj.y);
        if (iou_gt(bi, ai, bj, aj, thr)) bits |= 1ull << (j - j0);
    }
    return bits;
}

// Greedy NMS over S.box[0..m) in sorted order.  In: S.valid = candidate may be kept (invalid ones
// neither survive nor suppress).  Out: S.valid = kept.  If `groups`, only pairs with equal
// S.aux[] group ids interact (batched_nms).
template <int NT, int KC>
__device__ void nms_block(SegSmem<KC>& S, int m, const IouThr& thr, bool groups) {
    constexpr int NWORDS = KC / 64;
    const int nw = (m + 63) >> 6;
    // row i varies fastest across lanes: a wave's lanes read the same S.box[j] (an LDS broadcast)
    // while their own rows are consecutive (w-fastest put 16 lanes on one bank, 1 KiB apart)
    for (int t = threadIdx.x; t < m * nw; t += NT) {
        const int w = t / m, i = t - w * m;
        S.mask[i * NWORDS + w] = w >= (i >> 6) ? nms_mask_word(S.box, groups ? S.aux : nullptr, m, i, w, thr) : 0ull;
    }
    __syncthreads();
    if (threadIdx.x < 64) nms_scan<KC>(S.mask, S.valid, m);
    __syncthreads();
}

// Per-segment kept lists (records) consumed by merge_topk.

// Write the kept candidates of a segment in sorted order.  rec(t, slot_offset) writes one record.
template <int NT, int KC, typename SM, typename W>
__device__ void write_kept(SM& S, int m, int seg, const SegOut& out, W rec) {
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

// ================================================================ SSD per-class selection, wave form
// One wave per (image, class), four independent waves per workgroup and no workgroup barriers:
//   select   scores live in VGPRs (element i = lane + 64*j); the top-k threshold is found by
//            bisection with one ballot + popcount per register per probe;
//   compact  in index order (j-major, then lane) with ballots and lane masks: ties at the threshold
//            are taken lowest index first (the reference's stable order);
//   sort     wave-synchronous bitonic sort of (score, ~index) keys in this wave's LDS slice;
//   NMS      lazy greedy: the earliest candidate still alive is kept and suppresses the alive
//            candidates it overlaps (IoU over register-resident boxes, 64 lanes x KC/64 each); only
//            kept candidates' rows are ever evaluated, in sorted order, as the reference's loop does.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-class candidate set of one wave: score > thresh, then the top-k by (score desc, index asc),
// emitted in index order as emit(slot, key, anchor).  Returns the number emitted (<= topk).
template <int PER, typename E>
__device__ __forceinline__ int wave_select_topk(const float* __restrict__ sc, int A, float score_thresh, int topk,
                                                E emit) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    uint32_t kr[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        // unconditional (clamped) loads: no branch between them, so all PER are in flight at once
        const int i = lane + 64 * j;
        const float v = sc[i < A ? i : A - 1];
        kr[j] = (i < A && v > score_thresh) ? __float_as_uint(v) : 0u;  // probabilities >= 0: bits ordered
    }
    auto count_ge = [&](uint32_t t) -> int { return wave_count_ge<PER>(kr, t); };
    const int nvalid = count_ge(1u);
    const bool take_all = nvalid <= topk;
    uint32_t T = 1u;
    int need_eq = 0;
    if (!take_all) {
        // bisection on [min key, max key + 1): count(>= lo) >= topk > count(>= hi), then T = lo, the
        // topk-th largest key.  (Interpolating the probes between the two counts measured slower:
        // 52 against 42 us per 16-image chain.)
        uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            kmn = kr[j] != 0u && kr[j] < kmn ? kr[j] : kmn;
            kmx = kr[j] > kmx ? kr[j] : kmx;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t a = (uint32_t)__shfl_xor((int)kmn, o), b = (uint32_t)__shfl_xor((int)kmx, o);
            kmn = a < kmn ? a : kmn;
            kmx = b > kmx ? b : kmx;
        }
        uint64_t lo = kmn, hi = (uint64_t)kmx + 1;
        int chi = 0;
        while (hi - lo > 1) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            const int c = count_ge((uint32_t)mid);
            if (c >= topk) {
                lo = mid;
            } else {
                hi = mid;
                chi = c;
            }
        }
        T = (uint32_t)lo;
        need_eq = topk - chi;
    }
    int written = 0, eq_taken = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t k = kr[j];
        const bool gt = take_all ? (k != 0u) : (k > T);
        const bool eq = !take_all && k == T;
        const unsigned long long mg = __ballot(gt), me = __ballot(eq);
        const int ng = __popcll(mg), ne = __popcll(me);
        const int budget = need_eq - eq_taken;
        const int i = lane + 64 * j;
        if (gt) emit(written + __popcll(mg & lt_mask), k, i);
        if (eq) {
            const int pe = __popcll(me & lt_mask);
            if (pe < budget) emit(written + ng + pe, k, i);
        }
        const int used = ne < budget ? ne : (budget > 0 ? budget : 0);
        written += ng + used;
        eq_taken += used;
    }
    return written;
}

template <int PER, int KC>
__global__ void __launch_bounds__(256) ssd_class_nms_wave_kernel(const float* __restrict__ scores_t,
                                                                 const f32x4* __restrict__ boxes, int A, int NC,
                                                                 float score_thresh, int topk, IouThr iou,
                                                                 SegOut out) {
    constexpr int NQ = KC / 64;
    __shared__ unsigned long long keys_s[4][KC];
    __shared__ f32x4 box_s[4][KC];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 4 + w + 1;  // class 0 is background
    const int b = blockIdx.y;
    if (c >= NC) return;                   // whole wave leaves; nothing below waits on other waves
    unsigned long long* keys = keys_s[w];
    f32x4* bs = box_s[w];
    const float* sc = scores_t + ((int64_t)b * NC + c) * A;
    const int written = wave_select_topk<PER>(sc, A, score_thresh, topk, [&](int slot, uint32_t k, int i) {
        if (slot < KC) keys[slot] = make_key(k, (uint32_t)i);
    });
    const int m = written < KC ? written : KC;
    int p2 = 64;
    while (p2 < m) p2 <<= 1;
    for (int i = m + lane; i < p2; i += 64) keys[i] = 0ull;
    wave_sync();
    for (int k = 2; k <= p2; k <<= 1) {
        for (int jd = k >> 1; jd > 0; jd >>= 1) {
            for (int t = lane; t < p2 / 2; t += 64) {
                const int i = 2 * t - (t & (jd - 1));
                const int l = i + jd;
                const bool desc = (i & k) == 0;
                const unsigned long long x = keys[i], y = keys[l];
                if ((x < y) == desc) {
                    keys[i] = y;
                    keys[l] = x;
                }
            }
            wave_sync();
        }
    }
    for (int t = lane; t < m; t += 64) bs[t] = boxes[(int64_t)b * A + key_index(keys[t])];
    wave_sync();
    f32x4 bq[NQ];
    float aq[NQ];
    uint32_t alive = 0u;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int j = lane + 64 * q;
        bq[q] = j < m ? bs[j] : f32x4{0.f, 0.f, 0.f, 0.f};
        aq[q] = (bq[q].z - bq[q].x) * (bq[q].w - bq[q].y);
        if (j < m) alive |= 1u << q;
    }
    const int seg = b * (NC - 1) + (c - 1);
    int nkept = 0;
    while (true) {
        int i = -1;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const unsigned long long mq = __ballot((alive >> q) & 1u);
            if (i < 0 && mq) i = 64 * q + __builtin_ctzll(mq);
        }
        if (i < 0) break;
        if (lane == (i & 63)) alive &= ~(1u << (i >> 6));
        const f32x4 bi = bs[i];
        const float ai = (bi.z - bi.x) * (bi.w - bi.y);
#pragma unroll
        for (int q = 0; q < NQ; ++q)
            if (((alive >> q) & 1u) && iou_gt(bi, ai, bq[q], aq[q], iou)) alive &= ~(1u << q);
        if (lane == 0 && nkept < out.kmax) {
            const int64_t o = (int64_t)seg * out.kmax + nkept;
            out.box[o] = bi;
            out.score[o] = __uint_as_float((uint32_t)(keys[i] >> 32));
            out.tb[o] = ((uint32_t)c << 16) | (uint32_t)i;  // concatenation order: (class, rank)
            out.label[o] = c;
        }
        ++nkept;
    }
    if (lane == 0) out.count[seg] = nkept < out.kmax ? nkept : out.kmax;
}

// ================================================================ SSD postprocess, image-greedy form
// The reference's tail (per class: score > t, topk; concatenate; batched_nms; [:N]) only ever
// reports the first N kept candidates in (score desc, concatenation position asc) order.  Greedy
// NMS of one class depends only on that class's higher-ranked candidates, so walking the
// concatenated candidates in that global order, class by class greedy, and stopping once N are
// kept yields exactly the reference's output while touching ~N..2N candidates instead of every
// class's full top-k (SSD: 90 x 300).
//
// Stage 1, ssd_class_select_kernel: one wave per (image, class) writes the class's candidate set
// in index order into a fixed-stride pool [B][NC-1][topk] (key = score bits, 0 = empty; ref =
// anchor).  Pool position (class, slot) is the concatenation order among equal scores.
template <int PER>
__global__ void __launch_bounds__(256) ssd_class_select_kernel(const float* __restrict__ scores_t, int A, int NC,
                                                               float score_thresh, int topk,
                                                               uint32_t* __restrict__ pool_key,
                                                               int* __restrict__ pool_ref) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 4 + w + 1;
    const int b = blockIdx.y;
    if (c >= NC) return;
    const int64_t base = ((int64_t)b * (NC - 1) + (c - 1)) * topk;
    uint32_t* pk = pool_key + base;
    int* pr = pool_ref + base;
    const int written = wave_select_topk<PER>(scores_t + ((int64_t)b * NC + c) * A, A, score_thresh, topk,
                                              [&](int slot, uint32_t k, int i) {
                                                  if (slot < topk) {
                                                      pk[slot] = k;
                                                      pr[slot] = i;
                                                  }
                                              });
    for (int t = (written < topk ? written : topk) + lane; t < topk; t += 64) pk[t] = 0u;
}

// Stage 1, block form (the default): NW waves per (image, class), wave w holding elements
// i = lane + 64*(w*PW + j).  The one-wave form above issues ~7,000 dependent instructions per wave
// at ~1.4 waves per SIMD (profiles/r5h_ssd_sq_stall.txt: issue-bound, 34 us); here each bisection
// probe is NW partial ballot counts summed through LDS (double-buffered: one barrier per probe), and
// the compaction offsets each wave by the counts of the waves before it, so the pool is the one the
// wave form writes, slot for slot.
constexpr int SEL_PW = 13;  // 4 waves x 13 registers x 64 lanes = 3,328 anchors, the wave form's limit

template <int NW, int PW>
__global__ void __launch_bounds__(64 * NW) ssd_class_select_block_kernel(const float* __restrict__ scores_t, int A,
                                                                         int NC, float score_thresh, int topk,
                                                                         uint32_t* __restrict__ pool_key,
                                                                         int* __restrict__ pool_ref) {
    __shared__ int red[2][NW];
    __shared__ uint32_t kmn_s[NW], kmx_s[NW];
    __shared__ int ng_s[NW], ne_s[NW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    const int c = blockIdx.x + 1;  // class 0 is background
    const int b = blockIdx.y;
    const int64_t base = ((int64_t)b * (NC - 1) + (c - 1)) * topk;
    uint32_t* pk = pool_key + base;
    int* pr = pool_ref + base;
    const float* sc = scores_t + ((int64_t)b * NC + c) * A;
    uint32_t kr[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) {
        const int i = lane + 64 * (w * PW + j);
        const float v = sc[i < A ? i : A - 1];  // clamped: all PW loads in flight at once
        kr[j] = (i < A && v > score_thresh) ? __float_as_uint(v) : 0u;
    }
    int par = 0;
    auto count_ge = [&](uint32_t t) -> int {
        const int n = wave_count_ge<PW>(kr, t);
        if (lane == 0) red[par][w] = n;
        __syncthreads();
        int s = 0;
#pragma unroll
        for (int v = 0; v < NW; ++v) s += red[par][v];
        par ^= 1;
        return s;
    };
    const int nvalid = count_ge(1u);
    const bool take_all = nvalid <= topk;
    uint32_t T = 1u;
    int need_eq = 0;
    if (!take_all) {
        uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            kmn = kr[j] != 0u && kr[j] < kmn ? kr[j] : kmn;
            kmx = kr[j] > kmx ? kr[j] : kmx;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t a = (uint32_t)__shfl_xor((int)kmn, o), bb = (uint32_t)__shfl_xor((int)kmx, o);
            kmn = a < kmn ? a : kmn;
            kmx = bb > kmx ? bb : kmx;
        }
        if (lane == 0) {
            kmn_s[w] = kmn;
            kmx_s[w] = kmx;
        }
        __syncthreads();
#pragma unroll
        for (int v = 0; v < NW; ++v) {
            kmn = kmn_s[v] < kmn ? kmn_s[v] : kmn;
            kmx = kmx_s[v] > kmx ? kmx_s[v] : kmx;
        }
        // the same bisection as the wave form: count(>= lo) >= topk > count(>= hi)
        uint64_t lo = kmn, hi = (uint64_t)kmx + 1;
        int chi = 0;
        while (hi - lo > 1) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            const int cnt = count_ge((uint32_t)mid);
            if (cnt >= topk) {
                lo = mid;
            } else {
                hi = mid;
                chi = cnt;
            }
        }
        T = (uint32_t)lo;
        need_eq = topk - chi;
    }
    // this wave's candidates above / at the threshold, then its offsets in index order
    int ngw = 0, new_ = 0;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
        const uint32_t k = kr[j];
        ngw += __popcll(__ballot(take_all ? (k != 0u) : (k > T)));
        new_ += __popcll(__ballot(!take_all && k == T));
    }
    if (lane == 0) {
        ng_s[w] = ngw;
        ne_s[w] = new_;
    }
    __syncthreads();
    int pg = 0, pe = 0, tg = 0, te = 0;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
        if (v < w) {
            pg += ng_s[v];
            pe += ne_s[v];
        }
        tg += ng_s[v];
        te += ne_s[v];
    }
    int eq_taken = pe < need_eq ? pe : need_eq;
    int written = pg + eq_taken;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
        const uint32_t k = kr[j];
        const bool gt = take_all ? (k != 0u) : (k > T);
        const bool eq = !take_all && k == T;
        const unsigned long long mg = __ballot(gt), me = __ballot(eq);
        const int ng = __popcll(mg), ne = __popcll(me);
        const int budget = need_eq - eq_taken;
        const int i = lane + 64 * (w * PW + j);
        if (gt) {
            const int slot = written + __popcll(mg & lt_mask);
            pk[slot] = k;
            pr[slot] = i;
        }
        if (eq) {
            const int q = __popcll(me & lt_mask);
            if (q < budget) {
                const int slot = written + ng + q;
                pk[slot] = k;
                pr[slot] = i;
            }
        }
        const int used = ne < budget ? ne : (budget > 0 ? budget : 0);
        written += ng + used;
        eq_taken += used;
    }
    const int total = tg + (te < need_eq ? te : need_eq);
    for (int t = total + threadIdx.x; t < topk; t += 64 * NW) pk[t] = 0u;
}

// Stage 2, ssd_image_nms_kernel: one workgroup per image.  The pool's keys live in VGPRs (element
// i = threadIdx.x + NT*j); each round takes the exact next M candidates in global order
// (register bisection + ordered compaction, ties lowest pool position first), sorts them, and
// runs greedy NMS per class: wave w owns classes w, w+NW, ...; for each 64-candidate chunk of
// sorted order it first drops candidates overlapping the class's already-kept boxes (kept lists
// live in LDS as linked segments), then resolves the chunk lazily (earliest alive is kept and
// suppresses the alive ones it overlaps).  Kept candidates are emitted in sorted order until N.
template <int M, int KCAP, int PW>
struct ImgSmem {
    unsigned long long keys[M];
    f32x4 box[M];
    int cls[M];
    int kflag[M];
    f32x4 kbox[KCAP];
    int seg_base[KCAP], seg_n[KCAP], seg_next[KCAP];
    int head[SSD_MAXNC];
    int hist[SSD_MAXNC];
    int coff[SSD_MAXNC];  // class bucket offsets of the round
    int bucket[M];        // sorted positions grouped by class, score order within a class
    unsigned long long row[M];  // per candidate: later members of its class it suppresses (bit = rank)
    int rank[M];          // rank of the candidate within its class bucket
    unsigned long long run[M];          // rank_sort_desc's sorted 64-key runs
    int wcnt[M / 64][SSD_MAXNC];        // per wave of sorted order: candidates of each class
    uint32_t done[PW];
    int wsum[32];
    int red[32];
    int misc[8];
};

template <int NT, int PER, int M, int KCAP>
__global__ void __launch_bounds__(NT) ssd_image_nms_kernel(const uint32_t* __restrict__ pool_key,
                                                           const int* __restrict__ pool_ref,
                                                           const f32x4* __restrict__ boxes, int A, int NS, int topk,
                                                           int N, IouThr iou, const float* __restrict__ ratio,
                                                           float* __restrict__ out_box, float* __restrict__ out_score,
                                                           int64_t* __restrict__ out_label, int* __restrict__ out_count) {
    static_assert(M == NT, "one sorted candidate per thread");
    constexpr int PW = NT * PER / 32;
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    ImgSmem<M, KCAP, PW>& S = *reinterpret_cast<ImgSmem<M, KCAP, PW>*>(smem_raw);
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    const int n = NS * topk;
    const uint32_t* pk = pool_key + (int64_t)b * n;
    const int* pr = pool_ref + (int64_t)b * n;
    const f32x4* bx = boxes + (int64_t)b * A;

    uint32_t kr[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int i = tid + NT * j;
        const uint32_t k = pk[i < n ? i : n - 1];  // clamped: loads stay independent
        kr[j] = i < n ? k : 0u;
    }
    for (int t = tid; t < PW; t += NT) S.done[t] = 0u;
    for (int t = tid; t < NS; t += NT) S.head[t] = -1;
    if (tid == 0) {
        S.misc[0] = 0;  // kept boxes stored
        S.misc[1] = 0;  // segments stored
    }
    float rw = 1.f, rh = 1.f;
    if (ratio) {
        rw = ratio[2 * b];
        rh = ratio[2 * b + 1];
    }
    int total = 0;
    while (true) {
        // any prefix of the global order between 3M/4 and M candidates serves a round
        int nleft;
        const int m = select_topk_regs<NT, PER>(kr, M, M, S.keys, S.wsum, S.red, false, 3 * M / 4, &nleft);
        if (m == 0) break;
        if (tid < m) {
            const int i = key_index(S.keys[tid]);
            atomicOr(&S.done[i >> 5], 1u << (i & 31));
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = tid + NT * j;
            if (kr[j] && ((S.done[i >> 5] >> (i & 31)) & 1u)) kr[j] = 0u;
        }
        rank_sort_desc<NT>(S.keys, S.run, m);
        // each candidate's class and its rank among the earlier sorted candidates of its class: within
        // the wave by a ballot per distinct class (ordered by lane), across waves by the per-wave class
        // counts; the class histogram is their sum
        for (int t = tid; t < NW * NS; t += NT) S.wcnt[t / NS][t % NS] = 0;
        int c = -1, rin = 0;
        if (tid < m) {
            const int i = key_index(S.keys[tid]);
            c = i / topk;
            S.box[tid] = bx[pr[i]];
            S.cls[tid] = c;
            S.kflag[tid] = 0;
        }
        __syncthreads();
        {
            unsigned long long todo = __ballot(c >= 0);
            while (todo) {
                const int leader = __ffsll((long long)todo) - 1;
                const int cl = __builtin_amdgcn_readlane(c, leader);
                const unsigned long long mm = __ballot(c == cl);
                if (c == cl) rin = __popcll(mm & lt_mask);
                if (lane == leader) S.wcnt[wv][cl] = __popcll(mm);
                todo &= ~mm;
            }
        }
        __syncthreads();
        for (int t = tid; t < NS; t += NT) {
            int h = 0;
            for (int u = 0; u < NW; ++u) h += S.wcnt[u][t];
            S.hist[t] = h;
        }
        __syncthreads();
        // class buckets: offsets (exclusive scan of the histogram) and each candidate's rank among the
        // earlier sorted candidates of its class (a broadcast LDS walk), so a class's members are
        // processed together instead of every class scanning the whole round.
        if (wv == 0) {
            int run = 0;
            for (int c0 = 0; c0 < NS; c0 += 64) {
                const int c = c0 + lane;
                const int h = c < NS ? S.hist[c] : 0;
                int inc = h;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int t2 = __shfl_up(inc, off);
                    if (lane >= off) inc += t2;
                }
                if (c < NS) S.coff[c] = run + inc - h;
                run += __shfl(inc, 63);
            }
        }
        __syncthreads();
        if (tid < m) {
            int r = rin;
            for (int u = 0; u < wv; ++u) r += S.wcnt[u][c];
            S.bucket[S.coff[c] + r] = tid;
            S.rank[tid] = r;
        }
        __syncthreads();
        // Classes with <= 64 members this round: every candidate builds its suppression row against
        // the later members of its class (and its flag against the class's earlier kept boxes) in
        // parallel; then one thread per class runs the greedy scan over those rows.
        if (tid < m) {
            const int c = S.cls[tid];
            const int nc = S.hist[c];
            if (nc <= 64) {
                const f32x4 q = S.box[tid];
                const float aq = (q.z - q.x) * (q.w - q.y);
                bool alive = true;
                for (int sg = S.head[c]; sg >= 0 && alive; sg = S.seg_next[sg]) {
                    const int sb = S.seg_base[sg], sn = S.seg_n[sg];
                    for (int e = 0; e < sn && alive; ++e) {
                        const f32x4 kb = S.kbox[sb + e];
                        const float ka = (kb.z - kb.x) * (kb.w - kb.y);
                        if (iou_gt(kb, ka, q, aq, iou)) alive = false;
                    }
                }
                unsigned long long row = 0ull;
                const int* bk = S.bucket + S.coff[c];
                for (int k2 = S.rank[tid] + 1; k2 < nc; ++k2) {
                    const f32x4 kb = S.box[bk[k2]];
                    const float ka = (kb.z - kb.x) * (kb.w - kb.y);
                    if (iou_gt(q, aq, kb, ka, iou)) row |= 1ull << k2;
                }
                S.row[tid] = row;
                S.kflag[tid] = alive ? 2 : 0;  // 2 = alive candidate, resolved below
            }
        }
        __syncthreads();
        if (tid < NS) {
            const int c = tid;
            const int nc = S.hist[c];
            if (nc > 0 && nc <= 64) {
                const int* bk = S.bucket + S.coff[c];
                unsigned long long removed = 0ull, keptm = 0ull;
                for (int k2 = 0; k2 < nc; ++k2) {
                    const int t = bk[k2];
                    if (S.kflag[t] != 2) removed |= 1ull << k2;
                }
                for (int k2 = 0; k2 < nc; ++k2) {
                    if ((removed >> k2) & 1ull) continue;
                    keptm |= 1ull << k2;
                    removed |= S.row[bk[k2]];
                }
                const int nk = __popcll(keptm);
                if (nk) {
                    const int sb = atomicAdd(&S.misc[0], nk);
                    const int sg = atomicAdd(&S.misc[1], 1);
                    int w = 0;
                    for (int k2 = 0; k2 < nc; ++k2) {
                        const int t = bk[k2];
                        if ((keptm >> k2) & 1ull) {
                            S.kbox[sb + w++] = S.box[t];
                            S.kflag[t] = 1;
                        } else {
                            S.kflag[t] = 0;
                        }
                    }
                    S.seg_base[sg] = sb;
                    S.seg_n[sg] = nk;
                    S.seg_next[sg] = S.head[c];
                    S.head[c] = sg;
                } else {
                    for (int k2 = 0; k2 < nc; ++k2) S.kflag[bk[k2]] = 0;
                }
            }
        }
        __syncthreads();
        // Classes with more than 64 members this round: one wave per class, 64 members at a time.
        for (int c = wv; c < NS; c += NW) {
            if (S.hist[c] <= 64) continue;
            const int nc = S.hist[c];
            for (int base = 0; base < nc; base += 64) {
                const int j = base + lane;
                const bool in = j < nc;
                const int t = in ? S.bucket[S.coff[c] + j] : 0;
                const f32x4 q = in ? S.box[t] : f32x4{0.f, 0.f, 0.f, 0.f};
                const float aq = (q.z - q.x) * (q.w - q.y);
                bool alive = in;
                // boxes of this class kept in earlier rounds / chunks
                for (int sg = S.head[c]; sg >= 0 && __ballot(alive); sg = S.seg_next[sg]) {
                    const int sb = S.seg_base[sg], sn = S.seg_n[sg];
                    for (int e = 0; e < sn; ++e) {
                        const f32x4 kb = S.kbox[sb + e];
                        const float ka = (kb.z - kb.x) * (kb.w - kb.y);
                        if (alive && iou_gt(kb, ka, q, aq, iou)) alive = false;
                    }
                }
                // suppression row of each member against the later members of the chunk
                const int cnt = nc - base < 64 ? nc - base : 64;
                unsigned long long row = 0ull;
                for (int k2 = 0; k2 < cnt; ++k2) {
                    f32x4 kb;
                    kb.x = __shfl(q.x, k2);
                    kb.y = __shfl(q.y, k2);
                    kb.z = __shfl(q.z, k2);
                    kb.w = __shfl(q.w, k2);
                    const float ka = __shfl(aq, k2);
                    if (k2 > lane && in && iou_gt(q, aq, kb, ka, iou)) row |= 1ull << k2;
                }
                // greedy in score order over the chunk (scalar: rows read lane by lane)
                unsigned long long removed = ~__ballot(alive), keptm = 0ull;
                for (int i = 0; i < cnt; ++i) {
                    if ((removed >> i) & 1ull) continue;
                    keptm |= 1ull << i;
                    removed |= ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(row >> 32), i) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(row & 0xffffffffu), i);
                }
                if (keptm) {
                    const int nk = __popcll(keptm);
                    int sb = 0, sg = 0;
                    if (lane == 0) {
                        sb = atomicAdd(&S.misc[0], nk);
                        sg = atomicAdd(&S.misc[1], 1);
                    }
                    sb = __shfl(sb, 0);
                    sg = __shfl(sg, 0);
                    if ((keptm >> lane) & 1ull) {
                        S.kbox[sb + __popcll(keptm & lt_mask)] = q;
                        S.kflag[t] = 1;
                    }
                    if (lane == 0) {
                        S.seg_base[sg] = sb;
                        S.seg_n[sg] = nk;
                        S.seg_next[sg] = S.head[c];
                        S.head[c] = sg;
                    }
                    wave_sync();
                }
            }
        }
        __syncthreads();
        const bool kf = tid < m && S.kflag[tid];
        int tot;
        const int pos = BlockScan<NT>::exclusive(kf ? 1 : 0, S.wsum, tot);
        if (kf && total + pos < N) {
            const f32x4 q = S.box[tid];
            const int64_t o = (int64_t)b * N + total + pos;
            float* ob = out_box + o * 4;
            ob[0] = q.x * rw;
            ob[1] = q.y * rh;
            ob[2] = q.z * rw;
            ob[3] = q.w * rh;
            out_score[o] = __uint_as_float((uint32_t)(S.keys[tid] >> 32));
            if (out_label) out_label[o] = (int64_t)(S.cls[tid] + 1);
        }
        total += tot;
        if (total >= N || m >= nleft) break;  // a round may be a prefix shorter than M
    }
    if (tid == 0) out_count[b] = total < N ? total : N;
}

// ================================================================ RPN per-level selection

// rpn_chunk_select_kernel: one workgroup per (chunk of P.chunk anchors, level, image) keeps the
// chunk's top-k logits (ties at the cut in index order) unsorted, with their level indices.  compact()
// writes the list in two classes -- the keys above the chunk's threshold T first, then the keys equal
// to T -- each in index order, so the list is NOT in index order overall; it is in per-key index order:
// keys of one value always fall in one class, so entries of equal value keep their index order.
// Every element of a level's top-k is in its chunk's top-k, so the union of the chunk lists, chunks in
// order, holds the level's top-k, and equal keys in it sit in index order (within a chunk by the rule
// above, across chunks by chunk order): the level kernel's selection, which resolves ties at its cut by
// list position, therefore takes the same elements as over the whole level, from at most nchunk x KC
// entries instead of 120,000 logits per image at P2 through its five radix passes
// (tests/test_gpu_plan_records.py: chunked and unchunked records are equal under heavy ties).
template <int NT, int KC>
__global__ void __launch_bounds__(NT) rpn_chunk_select_kernel(RpnParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SelSmem<KC>& S = *reinterpret_cast<SelSmem<KC>*>(smem_raw);
    const int c = blockIdx.x, l = blockIdx.y, b = blockIdx.z;
    const RpnLevel L = P.lv[l];
    const int64_t slot = ((int64_t)(b * P.nlevels + l) * P.nchunk + c);
    const int start = c * P.chunk;
    if (start >= L.n) {
        if (threadIdx.x == 0) P.ccount[slot] = 0;
        return;
    }
    const int nc = min(P.chunk, L.n - start);
    const float* ob = L.obj + (int64_t)b * L.n + start;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        k = float_key(ob[i]);
        return true;
    };
    const uint32_t T = radix_select<NT>(nc, P.topk, fkey, S.hist, S.misc);
    const bool take_all = S.misc[1] <= P.topk;
    const int m = compact<NT>(nc, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
    for (int t = threadIdx.x; t < m; t += NT) {
        P.ckey[slot * KC + t] = (uint32_t)(S.keys[t] >> 32);
        P.cidx[slot * KC + t] = start + key_index(S.keys[t]);
    }
    if (threadIdx.x == 0) P.ccount[slot] = m;
}

template <int NT, int KC>
__global__ void __launch_bounds__(NT) rpn_level_nms_kernel(RpnParams P, SegOut out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int l = blockIdx.x, b = blockIdx.y;
    const RpnLevel L = P.lv[l];
    const float* ob = L.obj + (int64_t)b * L.n;
    const f32x4* db = reinterpret_cast<const f32x4*>(L.deltas) + (int64_t)b * L.n;
    // candidates: the whole level, or the union of its chunk lists (position i -> level index cidx[i])
    const bool chunked = P.ckey != nullptr;
    const int64_t cbase = (int64_t)(b * P.nlevels + l) * P.nchunk;
    const uint32_t* ck = chunked ? P.ckey + cbase * KC : nullptr;
    const int* ci = chunked ? P.cidx + cbase * KC : nullptr;
    const int* cc = chunked ? P.ccount + cbase : nullptr;
    const int n = chunked ? (L.n + P.chunk - 1) / P.chunk * KC : L.n;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        if (!chunked) {
            k = float_key(ob[i]);
            return true;
        }
        const int ch = i / KC, r = i - ch * KC;
        k = ck[i];
        return r < cc[ch];
    };
    auto level_index = [&](int i) { return chunked ? ci[i] : i; };
    const uint32_t T = radix_select<NT>(n, P.topk, fkey, S.hist, S.misc);
    const bool take_all = S.misc[1] <= P.topk;
    const int m = compact<NT>(n, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
    bitonic_desc<NT>(S.keys, nullptr, m);
    for (int t = threadIdx.x; t < m; t += NT) {
        const int i = level_index(key_index(S.keys[t]));
        const f32x4 d = db[i];
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

// ---------------------------------------------------------------- RPN level NMS, split form
// The level kernel above runs the whole segment (select, sort, decode, the m x m IoU mask, the greedy
// scan) in one workgroup per (level, image): 40 workgroups for FRCNN b = 8, each holding a CU for the
// whole O(m^2) mask.  The split form runs the same arithmetic as three launches -- the selection per
// segment (rpn_level_select_kernel, small LDS), the mask rows in 64-row blocks over KC / 64 x segments
// workgroups (rpn_mask_kernel), the scan and the kept records per segment (rpn_level_scan_kernel, the
// mask staged in LDS) -- with the intermediates in one scratch buffer (RpnSplit).
struct RpnSplit {
    unsigned long long* mask;  // [seg][KC][KC / 64]
    f32x4* box;                // [seg][KC]
    unsigned long long* key;   // [seg][KC]
    unsigned char* valid;      // [seg][KC]
    int* m;                    // [seg]
};
constexpr int RPN_KC = 1024, RPN_PER = 32;  // register path: chunk unions of <= 16 chunks
static inline int64_t rs_align(int64_t x) { return (x + 255) / 256 * 256; }
int64_t rpn_split_bytes(int64_t nseg) {
    return rs_align(nseg * RPN_KC * (RPN_KC / 64) * 8) + rs_align(nseg * RPN_KC * 16) + rs_align(nseg * RPN_KC * 8) +
           rs_align(nseg * RPN_KC) + rs_align(nseg * 4);
}
static RpnSplit rpn_split(void* base, int64_t nseg) {
    unsigned char* q = (unsigned char*)base;
    RpnSplit X;
    X.mask = (unsigned long long*)q;
    q += rs_align(nseg * RPN_KC * (RPN_KC / 64) * 8);
    X.box = (f32x4*)q;
    q += rs_align(nseg * RPN_KC * 16);
    X.key = (unsigned long long*)q;
    q += rs_align(nseg * RPN_KC * 8);
    X.valid = q;
    q += rs_align(nseg * RPN_KC);
    X.m = (int*)q;
    return X;
}

template <int NT, int KC>
__global__ void __launch_bounds__(NT) rpn_level_select_kernel(RpnParams P, RpnSplit X) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SelSmem<KC>& S = *reinterpret_cast<SelSmem<KC>*>(smem_raw);
    const int l = blockIdx.x, b = blockIdx.y;
    const int seg = b * P.nlevels + l;
    const RpnLevel L = P.lv[l];
    const float* ob = L.obj + (int64_t)b * L.n;
    const f32x4* db = reinterpret_cast<const f32x4*>(L.deltas) + (int64_t)b * L.n;
    const bool chunked = P.ckey != nullptr;
    const int64_t cbase = (int64_t)seg * P.nchunk;
    const uint32_t* ck = chunked ? P.ckey + cbase * KC : nullptr;
    const int* ci = chunked ? P.cidx + cbase * KC : nullptr;
    const int* cc = chunked ? P.ccount + cbase : nullptr;
    const int n = chunked ? (L.n + P.chunk - 1) / P.chunk * KC : L.n;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        if (!chunked) {
            k = float_key(ob[i]);
            return true;
        }
        const int ch = i / KC, r = i - ch * KC;
        k = ck[i];
        return r < cc[ch];
    };
    auto level_index = [&](int i) { return chunked ? ci[i] : i; };
    int m;
    if (chunked && n <= NT * RPN_PER) {
        // the chunk union held in registers (element i = threadIdx.x + NT * j, 0 = not a candidate):
        // the bisection top-k of select_topk_regs takes the same set as the radix select + compaction
        // below -- the top-k by (key desc, list position asc) -- with one barrier per probe instead of
        // four streaming passes with LDS histograms
        uint32_t kr[RPN_PER];
#pragma unroll
        for (int j = 0; j < RPN_PER; ++j) {
            const int i = (int)threadIdx.x + NT * j, ic = i < n ? i : n - 1;
            const int ch = ic / KC;
            const uint32_t k = ck[ic];
            kr[j] = (i < n && ic - ch * KC < cc[ch]) ? k : 0u;
        }
        m = select_topk_regs<NT, RPN_PER>(kr, P.topk, KC, S.keys, S.wsum, S.red);
    } else {
        const uint32_t T = radix_select<NT>(n, P.topk, fkey, S.hist, S.misc);
        const bool take_all = S.misc[1] <= P.topk;
        m = compact<NT>(n, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
    }
    rank_sort_desc<NT, KC / NT>(S.keys, S.run, m);
    for (int t = threadIdx.x; t < m; t += NT) {
        const int i = level_index(key_index(S.keys[t]));
        const f32x4 d = db[i];
        const f32x4 an = *reinterpret_cast<const f32x4*>(L.anchors + (int64_t)i * 4);
        const f32x4 bx = clip_box(decode_box(d, an, 1.f, 1.f, 1.f, 1.f), P.img_h, P.img_w);
        const float logit = key_float((uint32_t)(S.keys[t] >> 32));
        const float score = 1.f / (1.f + expf(-logit));
        const int64_t o = (int64_t)seg * KC + t;
        X.box[o] = bx;
        X.key[o] = S.keys[t];
        X.valid[o] = ((bx.z - bx.x) >= P.min_size && (bx.w - bx.y) >= P.min_size && score >= P.score_thresh) ? 1 : 0;
    }
    if (threadIdx.x == 0) X.m[seg] = m;
}

// grid (KC / 64 row blocks, levels, images): mask rows [64 rb, 64 rb + 64) of the segment, words
// w >= rb (the only ones the scan reads), the segment's boxes from 64 rb on staged in LDS
template <int KC>
__global__ void __launch_bounds__(256) rpn_mask_kernel(RpnSplit X, int nlevels, IouThr thr) {
    constexpr int NWORDS = KC / 64;
    __shared__ f32x4 sb[KC];
    const int rb = blockIdx.x, seg = blockIdx.z * nlevels + blockIdx.y;
    const int m = X.m[seg];
    const int nw = (m + 63) >> 6;
    if (rb >= nw) return;
    const f32x4* gb = X.box + (int64_t)seg * KC;
    {  // every load of the thread issued before any store (clamped indices)
        f32x4 v[KC / 256];
#pragma unroll
        for (int u = 0; u < KC / 256; ++u) v[u] = gb[min(64 * rb + (int)threadIdx.x + 256 * u, m - 1)];
#pragma unroll
        for (int u = 0; u < KC / 256; ++u) {
            const int t = 64 * rb + (int)threadIdx.x + 256 * u;
            if (t < m) sb[t] = v[u];
        }
    }
    __syncthreads();
    const int i0 = 64 * rb, ni = min(64, m - i0), ntask = ni * (nw - rb);
    unsigned long long* gm = X.mask + (int64_t)seg * KC * NWORDS;
    for (int t = threadIdx.x; t < ntask; t += 256) {  // row fastest across lanes, as nms_block
        const int w = rb + t / ni, i = i0 + t % ni;
        gm[i * NWORDS + w] = nms_mask_word(sb, nullptr, m, i, w, thr);
    }
}

template <int KC>
struct ScanSmem {
    unsigned long long mask[KC * (KC / 64)];
    unsigned char valid[KC];
    int wsum[32];
};

template <int NT, int KC>
__global__ void __launch_bounds__(NT) rpn_level_scan_kernel(RpnParams P, RpnSplit X, SegOut out) {
    constexpr int NWORDS = KC / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    ScanSmem<KC>& S = *reinterpret_cast<ScanSmem<KC>*>(smem_raw);
    const int l = blockIdx.x, b = blockIdx.y;
    const int seg = b * P.nlevels + l;
    const int m = X.m[seg];
    const unsigned long long* gm = X.mask + (int64_t)seg * KC * NWORDS;
    // exactly the words rpn_mask_kernel wrote: rows i < m, words i / 64 .. nw - 1 (nothing below a
    // row's own 64-row block, nothing past the last block).  Wave k stages row blocks k and
    // 2 NW - 1 - k (17 row-block widths per wave), lane-contiguous within each block's
    // rows x words, every load of the wave in flight before its stores.
    {
        static_assert(NWORDS == 2 * (NT / 64), "two row blocks per wave");
        const int nw = (m + 63) >> 6, wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        unsigned long long v[2][NWORDS];
        int at[2][NWORDS];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int rb = h == 0 ? wv : NWORDS - 1 - wv;  // wave-uniform
            const int i0 = 64 * rb, wn = nw - rb, cnt = rb < nw ? min(64, m - i0) * wn : 0;
            const float inv = 1.f / (float)(wn > 0 ? wn : 1);
#pragma unroll
            for (int u = 0; u < NWORDS; ++u) {
                const int f = ln + 64 * u;
                at[h][u] = -1;
                if (f < cnt) {
                    // f / wn exactly: f < 1024 and wn <= 16 keep (f + 0.5) / wn at least 1/32 from an integer
                    const int r = (int)(((float)f + 0.5f) * inv);
                    at[h][u] = (i0 + r) * NWORDS + rb + (f - r * wn);
                    v[h][u] = gm[at[h][u]];
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int u = 0; u < NWORDS; ++u)
                if (at[h][u] >= 0) S.mask[at[h][u]] = v[h][u];
    }
    for (int t = threadIdx.x; t < m; t += NT) S.valid[t] = X.valid[(int64_t)seg * KC + t];
    __syncthreads();
    if (threadIdx.x < 64) nms_scan<KC>(S.mask, S.valid, m);
    __syncthreads();
    write_kept<NT, KC>(S, m, seg, out, [&](int t, int64_t o) {
        const unsigned long long key = X.key[(int64_t)seg * KC + t];
        const float logit = key_float((uint32_t)(key >> 32));
        out.box[o] = X.box[(int64_t)seg * KC + t];
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
                                                           float score_thresh, float min_size, IouThr iou,
                                                           SegOut out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int c = blockIdx.x + 1, b = blockIdx.y;
    const int n = counts[b];
    const float* sc = scores + (int64_t)b * R * NC + c;
    const f32x4* bx = boxes + (int64_t)b * R * NC + c;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        const float s = sc[(int64_t)i * NC];
        const f32x4 q = bx[(int64_t)i * NC];  // loaded unconditionally (no dependent round trip)
        k = __float_as_uint(s);
        return (s > score_thresh) & ((q.z - q.x) >= min_size) & ((q.w - q.y) >= min_size);
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

// ================================================================ RetinaNet postprocess
// RetinaNet.postprocess_detections (retinanet_resnet50_fpn_v2, detect.py:34-38; oracle/retinanet.py):
// per level: sigmoid over the flattened (anchor, class) logits, score > 0.05, topk(min(1000, n))
// (score desc, flat index asc), decode (1,1,1,1) + clip -> candidate lists [B][L][topk];
// then batched_nms(0.5) by label over the concatenated level lists and [:300].
//
// Two stages, so that a level of ~8M (anchor, class) scores is not one workgroup's work:
// retina_chunk_select_kernel: one workgroup per (chunk of CH flat indices, level, image) keeps the
//     chunk's top-k (score desc, index asc) unsorted in index order; every element of the level's
//     top-k is in its chunk's top-k, so the union of the chunk lists (chunks in order) holds it with
//     index order preserved;
// retina_select_kernel: one workgroup per (level, image) selects the top-k of that union, sorts it,
//     decodes and clips the boxes.
template <int NT, int KC>
__global__ void __launch_bounds__(NT) retina_chunk_select_kernel(RetinaSelParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int c = blockIdx.x, l = blockIdx.y, b = blockIdx.z;
    const int K = P.K;
    const int n = P.na[l] * K;
    const int64_t slot = ((int64_t)(b * P.L + l) * P.nchunk + c);
    const int start = c * P.chunk;
    if (start >= n) {
        if (threadIdx.x == 0) P.ccount[slot] = 0;
        return;
    }
    const int nc = min(P.chunk, n - start);
    const float* lg = P.logits + ((int64_t)b * P.Atot + P.a0[l]) * K + start;
    const float thr = P.score_thresh;
    auto fkey = [&](int i, uint32_t& k) -> bool {
        const float s = 1.f / (1.f + expf(-lg[i]));
        k = __float_as_uint(s);
        return s > thr;
    };
    const uint32_t T = radix_select<NT>(nc, P.topk, fkey, S.hist, S.misc);
    const bool take_all = S.misc[1] <= P.topk;
    const int m = compact<NT>(nc, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
    for (int t = threadIdx.x; t < m; t += NT) {
        P.ckey[slot * KC + t] = (uint32_t)(S.keys[t] >> 32);
        P.cidx[slot * KC + t] = start + key_index(S.keys[t]);
    }
    if (threadIdx.x == 0) P.ccount[slot] = m;
}

template <int NT, int KC>
__global__ void __launch_bounds__(NT) retina_select_kernel(RetinaSelParams P, SegOut out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int l = blockIdx.x, b = blockIdx.y;
    const int K = P.K;
    const int n = P.na[l] * K;
    const int nch = (n + P.chunk - 1) / P.chunk;
    const int64_t base = (int64_t)(b * P.L + l) * P.nchunk;
    const uint32_t* ck = P.ckey + base * KC;
    const int* cc = P.ccount + base;
    auto fkey = [&](int i, uint32_t& k) -> bool {  // i = chunk * KC + rank (index order preserved)
        const int ch = i / KC, r = i - ch * KC;
        k = ck[i];
        return r < cc[ch];
    };
    const int n2 = nch * KC;
    const uint32_t T = radix_select<NT>(n2, P.topk, fkey, S.hist, S.misc);
    const bool take_all = S.misc[1] <= P.topk;
    const int m = compact<NT>(n2, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
    bitonic_desc<NT>(S.keys, nullptr, m);
    const int seg = b * P.L + l;
    for (int t = threadIdx.x; t < m; t += NT) {
        const int i = P.cidx[base * KC + key_index(S.keys[t])];
        const int a = P.a0[l] + i / K;
        const f32x4 d = *reinterpret_cast<const f32x4*>(P.deltas + ((int64_t)b * P.Atot + a) * 4);
        const f32x4 an = *reinterpret_cast<const f32x4*>(P.anchors + (int64_t)a * 4);
        const int64_t o = (int64_t)seg * out.kmax + t;
        out.box[o] = clip_box(decode_box(d, an, 1.f, 1.f, 1.f, 1.f), P.img_h, P.img_w);
        out.score[o] = __uint_as_float((uint32_t)(S.keys[t] >> 32));
        out.label[o] = i % K;
        out.tb[o] = (uint32_t)(l * out.kmax + t);
    }
    if (threadIdx.x == 0) out.count[seg] = m;
}

// retina_class_nms_kernel: one workgroup per (class, image).  The class's candidates, in the
// concatenated (level, rank) order, are taken KC at a time in (score desc, position asc) order (radix
// select + ordered compaction, the next chunk strictly after the last key of the previous one);
// each chunk is first suppressed by every box kept so far, then resolved greedily (nms_block).
// Stops once out.kmax boxes are kept: later ones cannot enter the image's top out.kmax.
template <int NT, int KC, int KEEP>
__global__ void __launch_bounds__(NT) retina_class_nms_kernel(RetinaNmsParams P, SegOut out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    __shared__ f32x4 kept_box[KEEP];
    __shared__ float kept_area[KEEP];
    const int c = blockIdx.x, b = blockIdx.y;
    const int n = P.L * P.kin;
    const int64_t base = (int64_t)b * P.L * P.kin;
    const int* cnt = P.count + b * P.L;
    const int seg = b * P.K + c;
    const int cap = out.kmax < KEEP ? out.kmax : KEEP;
    uint32_t Tp = 0xffffffffu;
    int Ip = -1;
    bool first = true;
    int kept = 0;
    for (;;) {
        auto fkey = [&](int i, uint32_t& k) -> bool {
            const int l = i / P.kin, r = i - l * P.kin;
            const float sc = P.score[base + i];
            const int lb = P.label[base + i];
            k = __float_as_uint(sc);
            const bool after = first || k < Tp || (k == Tp && i > Ip);
            return (r < cnt[l]) & (lb == c) & after;
        };
        const uint32_t T = radix_select<NT>(n, KC, fkey, S.hist, S.misc);
        const bool take_all = S.misc[1] <= KC;
        const int m = compact<NT>(n, T, take_all, S.misc[5], KC, fkey, S.keys, S.wsum);
        if (m == 0) break;
        bitonic_desc<NT>(S.keys, nullptr, m);
        for (int t = threadIdx.x; t < m; t += NT) {
            const f32x4 bx = P.box[base + key_index(S.keys[t])];
            const float ab = (bx.z - bx.x) * (bx.w - bx.y);
            bool alive = true;
            for (int q = 0; q < kept && alive; ++q)
                if (iou_gt(kept_box[q], kept_area[q], bx, ab, P.iou)) alive = false;
            S.box[t] = bx;
            S.valid[t] = alive ? 1 : 0;
        }
        __syncthreads();
        nms_block<NT, KC>(S, m, P.iou, false);
        int written = 0;
        for (int b0 = 0; b0 < m; b0 += NT) {
            const int t = b0 + threadIdx.x;
            const bool kf = t < m && S.valid[t];
            int tot;
            const int pos = BlockScan<NT>::exclusive(kf ? 1 : 0, S.wsum, tot);
            const int slot = kept + written + pos;
            if (kf && slot < cap) {
                const int i = key_index(S.keys[t]);
                const int64_t o = (int64_t)seg * out.kmax + slot;
                out.box[o] = S.box[t];
                out.score[o] = __uint_as_float((uint32_t)(S.keys[t] >> 32));
                out.tb[o] = (uint32_t)i;  // concatenation order (level, rank)
                out.label[o] = c;
                kept_box[slot] = S.box[t];
                kept_area[slot] = (S.box[t].z - S.box[t].x) * (S.box[t].w - S.box[t].y);
            }
            written += tot;
        }
        kept = kept + written < cap ? kept + written : cap;
        const unsigned long long last = S.keys[m - 1];
        __syncthreads();
        if (take_all || kept >= cap) break;
        Tp = (uint32_t)(last >> 32);
        Ip = key_index(last);
        first = false;
    }
    if (threadIdx.x == 0) out.count[seg] = kept;
}

// ================================================================ unit (batched) NMS for the C API
template <int NT, int KC>
__global__ void __launch_bounds__(NT) unit_nms_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                                                      const int64_t* __restrict__ idxs, int n, IouThr iou,
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

template <int NT, int KC, int PER>
__global__ void __launch_bounds__(NT) merge_topk_kernel(MergeParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SegSmem<KC>& S = *reinterpret_cast<SegSmem<KC>*>(smem_raw);
    const int b = blockIdx.x;
    const int* cnt = P.count + (int64_t)b * P.S;
    const int64_t base_off = (int64_t)b * P.S * P.kmax;
    // candidates = the valid prefix [0, count) of every segment, concatenated in segment order
    int* pre = S.aux;  // pre[s] = first candidate of segment s, pre[S] = total
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int q = 0; q < P.S; ++q) {
            pre[q] = acc;
            const int c = cnt[q];
            acc += c < P.kmax ? c : P.kmax;
        }
        pre[P.S] = acc;
    }
    __syncthreads();
    const int n = pre[P.S];
    auto flat = [&](int i) -> int {  // candidate index -> segment * kmax + slot
        int lo = 0, hi = P.S;        // largest q with pre[q] <= i
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (pre[mid] <= i) lo = mid;
            else hi = mid;
        }
        return lo * P.kmax + (i - pre[lo]);
    };
    int m0;
    if (n <= NT * PER) {
        // all record offsets first (LDS searches), then the global loads back to back
        int fo[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = threadIdx.x + NT * j;
            fo[j] = flat(i < n ? i : (n > 0 ? n - 1 : 0));
        }
        float v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) v[j] = P.score[base_off + fo[j]];
        uint32_t kr[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            asm volatile("" : "+v"(v[j]));  // keeps every load unconditional (not sunk into a branch)
            const int i = threadIdx.x + NT * j;
            kr[j] = i < n ? float_key(v[j]) : 0u;
        }
        // every key > T plus all ties (up to capacity); ties are then ordered by tiebreak
        m0 = select_topk_regs<NT, PER>(kr, P.N, KC, S.keys, S.wsum, S.misc, true);
    } else {
        auto fkey = [&](int i, uint32_t& k) -> bool {
            k = float_key(P.score[base_off + flat(i)]);
            return true;
        };
        const uint32_t T = radix_select<NT>(n, P.N, fkey, S.hist, S.misc);
        const bool take_all = S.misc[1] <= P.N;
        m0 = compact<NT>(n, T, take_all, KC, KC, fkey, S.keys, S.wsum);
    }
    // candidate indices must be recovered before pre[] (aliasing aux) is overwritten
    unsigned long long* tmp = S.mask;
    for (int t = threadIdx.x; t < m0; t += NT) tmp[t] = (unsigned long long)flat(key_index(S.keys[t]));
    __syncthreads();
    for (int t = threadIdx.x; t < m0; t += NT) {
        const int f = (int)tmp[t];
        S.aux[t] = f;
        S.keys[t] = make_key(__float_as_uint(P.score[base_off + f]), P.tb[base_off + f]);
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
    EDGEDET_REQUIRE(NC <= SSD_MAXNC, "ssd_scores: at most 128 classes");
    hipLaunchKernelGGL(ssd_scores_kernel, dim3((unsigned)cdiv(A, 64), B), dim3(256), 0, s, logits, reg, anchors,
                       scores_t, boxes, B, A, NC, img_h, img_w);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int box_scores_launch(const float* pred, int ld, int cls_off, int delta_off, const float* props, const int* counts,
                      float* scores, float* boxes, int B, int R, int NC, float img_h, float img_w, hipStream_t s) {
    EDGEDET_REQUIRE(pred && props && counts && scores && boxes, "box_scores: null pointer");
    EDGEDET_REQUIRE(ld >= 5 * NC && ld % 4 == 0 && delta_off % 4 == 0, "box_scores: bad predictor layout");
    EDGEDET_REQUIRE(NC >= 1 && NC <= BOX_MAXNC, "box_scores: 1..128 classes");
    const int64_t total = (int64_t)B * R;
    hipLaunchKernelGGL(box_scores_kernel, dim3((unsigned)cdiv(total, 4)), dim3(256), 0, s, pred, ld, cls_off,
                       delta_off, props, counts, scores, boxes, B, R, NC, img_h, img_w);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

IouThr make_iou_thr(double thr) {
    IouThr t;
    t.thr = thr;
    float t1 = (float)thr;
    if ((double)t1 <= thr) t1 = std::nextafter(t1, std::numeric_limits<float>::infinity());
    const float t0 = std::nextafter(t1, -std::numeric_limits<float>::infinity());
    t.mid = ((double)t0 + (double)t1) * 0.5;
    uint32_t bits;
    std::memcpy(&bits, &t1, 4);
    t.tie_up = (bits & 1u) == 0u;
    return t;
}

int ssd_class_nms_launch(const float* scores_t, const float* boxes, int B, int A, int NC, float score_thresh,
                         int topk, double iou, SegOut out, hipStream_t s) {
    EDGEDET_REQUIRE(scores_t && boxes && seg_ok(out), "ssd_class_nms: null pointer");
    EDGEDET_REQUIRE(topk <= 512 && out.kmax >= topk, "ssd_class_nms: topk must be <= 512 and <= kmax");
    constexpr int KC = 512, PER = 52;
    EDGEDET_REQUIRE(A <= 64 * PER, "ssd_class_nms: at most 3328 anchors per image");
    hipLaunchKernelGGL((ssd_class_nms_wave_kernel<PER, KC>), dim3((unsigned)cdiv(NC - 1, 4), B), dim3(256), 0, s,
                       scores_t, (const f32x4*)boxes, A, NC, score_thresh, topk, make_iou_thr(iou), out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int ssd_postprocess_launch(const SsdPostParams& P, hipStream_t s) {
    EDGEDET_REQUIRE(P.scores_t && P.boxes && P.pool_key && P.pool_ref && P.out_box && P.out_score && P.out_count,
                    "ssd_postprocess: null pointer");
    constexpr int PER_A = 52, NT = 512, PER = 54, M = 512, KCAP = 1536;
    EDGEDET_REQUIRE(P.A > 0 && P.A <= 64 * PER_A, "ssd_postprocess: at most 3328 anchors per image");
    EDGEDET_REQUIRE(P.NC >= 2 && P.NC <= SSD_MAXNC, "ssd_postprocess: 2..128 classes");
    EDGEDET_REQUIRE(P.topk > 0 && (int64_t)(P.NC - 1) * P.topk <= (int64_t)NT * PER,
                    "ssd_postprocess: (classes-1) * topk must be <= 27648");
    EDGEDET_REQUIRE(P.N > 0 && P.N + M <= KCAP, "ssd_postprocess: detections per image must be <= 1024");
    if (P.select_wave) {
        hipLaunchKernelGGL(ssd_class_select_kernel<PER_A>, dim3((unsigned)cdiv(P.NC - 1, 4), P.B), dim3(256), 0, s,
                           P.scores_t, P.A, P.NC, P.score_thresh, P.topk, P.pool_key, P.pool_ref);
    } else {
        constexpr int NWS = 4;
        static_assert(NWS * SEL_PW >= PER_A, "the block form covers the wave form's anchors");
        hipLaunchKernelGGL((ssd_class_select_block_kernel<NWS, SEL_PW>), dim3((unsigned)(P.NC - 1), P.B),
                           dim3(64 * NWS), 0, s, P.scores_t, P.A, P.NC, P.score_thresh, P.topk, P.pool_key,
                           P.pool_ref);
    }
    EDGEDET_LAUNCH_CHECK();
    auto k = ssd_image_nms_kernel<NT, PER, M, KCAP>;
    const size_t lds = sizeof(ImgSmem<M, KCAP, NT * PER / 32>);
    if (set_lds(k, lds)) return -2;
    hipLaunchKernelGGL(k, dim3(P.B), dim3(NT), lds, s, P.pool_key, P.pool_ref, (const f32x4*)P.boxes, P.A, P.NC - 1,
                       P.topk, P.N, make_iou_thr(P.iou), P.ratio, P.out_box, P.out_score, P.out_label, P.out_count);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int rpn_level_nms_launch(const RpnParams& P, SegOut out, hipStream_t s) {
    EDGEDET_REQUIRE(P.topk <= 1024 && out.kmax >= P.topk, "rpn: topk must be <= 1024 and <= kmax");
    EDGEDET_REQUIRE(P.nlevels >= 1 && P.nlevels <= 5, "rpn: 1..5 levels");
    EDGEDET_REQUIRE(seg_ok(out), "rpn: null output records");
    for (int l = 0; l < P.nlevels; ++l)
        EDGEDET_REQUIRE(P.lv[l].obj && P.lv[l].deltas && P.lv[l].anchors && P.lv[l].n > 0, "rpn: null/empty level");
    constexpr int KC = 1024, NT = 512;
    if (P.ckey) {
        EDGEDET_REQUIRE(P.cidx && P.ccount && P.chunk >= P.topk && P.nchunk >= 1, "rpn: chunk scratch");
        for (int l = 0; l < P.nlevels; ++l)
            EDGEDET_REQUIRE((P.lv[l].n + P.chunk - 1) / P.chunk <= P.nchunk, "rpn: a level exceeds nchunk chunks");
        auto k1 = rpn_chunk_select_kernel<NT, KC>;
        if (set_lds(k1, sizeof(SelSmem<KC>))) return -2;
        hipLaunchKernelGGL(k1, dim3(P.nchunk, P.nlevels, P.B), dim3(NT), sizeof(SelSmem<KC>), s, P);
        EDGEDET_LAUNCH_CHECK();
    }
    if (P.split) {
        static_assert(KC == RPN_KC, "split scratch layout");
        const RpnSplit X = rpn_split(P.split, (int64_t)P.B * P.nlevels);
        auto k1 = rpn_level_select_kernel<NT, KC>;
        if (set_lds(k1, sizeof(SelSmem<KC>))) return -2;
        hipLaunchKernelGGL(k1, dim3(P.nlevels, P.B), dim3(NT), sizeof(SelSmem<KC>), s, P, X);
        EDGEDET_LAUNCH_CHECK();
        hipLaunchKernelGGL(rpn_mask_kernel<KC>, dim3(KC / 64, P.nlevels, P.B), dim3(256), 0, s, X, P.nlevels, P.iou);
        EDGEDET_LAUNCH_CHECK();
        auto k3 = rpn_level_scan_kernel<NT, KC>;
        if (set_lds(k3, sizeof(ScanSmem<KC>))) return -2;
        hipLaunchKernelGGL(k3, dim3(P.nlevels, P.B), dim3(NT), sizeof(ScanSmem<KC>), s, P, X, out);
        EDGEDET_LAUNCH_CHECK();
        return 0;
    }
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
                       score_thresh, min_size, make_iou_thr(iou), out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int retina_select_launch(const RetinaSelParams& P, SegOut out, hipStream_t s) {
    EDGEDET_REQUIRE(P.logits && P.deltas && P.anchors && seg_ok(out), "retina_select: null pointer");
    EDGEDET_REQUIRE(P.L >= 1 && P.L <= 5 && P.topk > 0 && P.topk <= 1024 && out.kmax >= P.topk,
                    "retina_select: 1..5 levels, topk <= 1024 <= kmax");
    for (int l = 0; l < P.L; ++l)
        EDGEDET_REQUIRE(P.na[l] > 0 && (int64_t)P.na[l] * P.K < (1ll << 31) && P.a0[l] + P.na[l] <= P.Atot,
                        "retina_select: bad level extent");
    EDGEDET_REQUIRE(P.ckey && P.cidx && P.ccount && P.chunk > 0 && P.nchunk > 0, "retina_select: null scratch");
    for (int l = 0; l < P.L; ++l)
        EDGEDET_REQUIRE(((int64_t)P.na[l] * P.K + P.chunk - 1) / P.chunk <= P.nchunk, "retina_select: scratch too small");
    constexpr int KC = 1024, NT = 512;
    auto k1 = retina_chunk_select_kernel<NT, KC>;
    if (set_lds(k1, seg_smem<KC>())) return -2;
    hipLaunchKernelGGL(k1, dim3(P.nchunk, P.L, P.B), dim3(NT), seg_smem<KC>(), s, P);
    EDGEDET_LAUNCH_CHECK();
    auto k2 = retina_select_kernel<NT, KC>;
    if (set_lds(k2, seg_smem<KC>())) return -2;
    hipLaunchKernelGGL(k2, dim3(P.L, P.B), dim3(NT), seg_smem<KC>(), s, P, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int retina_class_nms_launch(const RetinaNmsParams& P, int B, SegOut out, hipStream_t s) {
    EDGEDET_REQUIRE(P.box && P.score && P.label && P.count && seg_ok(out), "retina_class_nms: null pointer");
    EDGEDET_REQUIRE(P.L >= 1 && P.kin > 0 && P.K > 0 && out.kmax > 0 && out.kmax <= 512,
                    "retina_class_nms: bad sizes (kmax <= 512)");
    constexpr int KC = 512, NT = 512, KEEP = 512;
    auto k = retina_class_nms_kernel<NT, KC, KEEP>;
    const size_t lds = seg_smem<KC>();
    if (set_lds(k, lds + KEEP * 20)) return -2;
    hipLaunchKernelGGL(k, dim3(P.K, B), dim3(NT), lds, s, P, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int merge_topk_launch(const MergeParams& P, int B, hipStream_t s) {
    EDGEDET_REQUIRE(P.box && P.score && P.tb && P.label && P.count && P.out_box && P.out_score && P.out_count,
                    "merge_topk: null pointer");
    EDGEDET_REQUIRE(P.N <= 1024 && P.N > 0 && P.S > 0 && P.kmax > 0, "merge_topk: bad sizes");
    EDGEDET_REQUIRE(P.S < 1024, "merge_topk: at most 1023 segments");
    // PER = 16 register slots per thread (8,192 candidates on the register path, the radix path above
    // that): at 64 the kernel took 202 VGPRs and 272 B of scratch per lane
    constexpr int KC = 1024, NT = 512, PER = 16;
    auto k = merge_topk_kernel<NT, KC, PER>;
    if (set_lds(k, seg_smem<KC>())) return -2;
    hipLaunchKernelGGL(k, dim3(B), dim3(NT), seg_smem<KC>(), s, P);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// the single-workgroup path of the unit NMS (csrc/unitops.hip: edgedet_nms / edgedet_batched_nms)
int unit_small_nms(const float* boxes, const float* scores, const int64_t* idxs, int64_t n, double iou_threshold,
                   int64_t* keep, int32_t* d_num_keep, hipStream_t s) {
    EDGEDET_REQUIRE(n >= 0 && n <= 1024, "batched_nms: single-workgroup path takes n <= 1024");
    EDGEDET_REQUIRE(d_num_keep && (n == 0 || (boxes && scores && keep)), "batched_nms: null pointer");
    if (n == 0) {
        EDGEDET_CHECK_HIP(hipMemsetAsync(d_num_keep, 0, sizeof(int32_t), s));
        return 0;
    }
    constexpr int KC = 1024, NT = 512;
    auto k = unit_nms_kernel<NT, KC>;
    const size_t lds = seg_smem<KC>();
    if (set_lds(k, lds)) return -2;
    hipLaunchKernelGGL(k, dim3(1), dim3(NT), lds, s, boxes, scores, idxs, (int)n, make_iou_thr(iou_threshold), keep,
                       d_num_keep);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

}  // namespace edgedet
