// Memory-bound layers of the two detectors (NHWC fp32, one thread per pixel x 4 channels).
//
//   preprocess   GeneralizedRCNNTransform eval: (x - mean) / std, bilinear resize
//                (align_corners=False), zero pad to the batch size        SURVEY.md App. A.0, row a6
//   dwconv       depthwise conv + folded BN + act (MobileNetV3 / SSDLite)  App. A.1, rows a7/a8
//   channel_mean adaptive_avg_pool2d(1) of SqueezeExcitation               App. A.1 step 2
//   se_fc        SE fc1 -> ReLU -> fc2 -> Hardsigmoid (batched GEMVs)       App. A.1 step 2
//   maxpool      ResNet stem max_pool2d(3,2,1); FPN LastLevelMaxPool(1,2,0) App. A.2 steps 2-3
//   roi_align    MultiScaleRoIAlign: LevelMapper + roi_align(7x7, sr=2, aligned=False)
//                                                                          App. A.2 step 5, row a13
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "kernels.hpp"

namespace edgedet {


// ------------------------------------------------------------------------------ preprocess

// ObjectDetectionDataset.__getitem__'s `image / 255` (detect.py:55-58) on the device for a uint8
// input: an IEEE float division (correctly rounded, as torch's CPU true_divide), so the value equals
// the host's float image bit for bit and the rest of the transform is unchanged.
//
// FAST (uint8 input only): both divisions of the transform -- x / 255 and (v - mean) / std -- as a
// multiply by the rounded reciprocal and one fma residual correction, q = RN(a r); q += RN(a - q b) r,
// 3 instructions instead of the ~10 of a correctly rounded division.  That form is not correctly
// rounded for every float a, but a uint8 image gives each division only 256 operands per channel, and
// the launcher (u8_fast_div) checks all of them on the host against the IEEE division for the actual
// mean / std, taking this path only when every one is bit-identical.
__device__ __forceinline__ float div_fast(float a, float b, float rb) {
    const float q = a * rb;
    return fmaf(fmaf(-q, b, a), rb, q);
}

template <typename T, bool FAST = false>
__device__ __forceinline__ float pre_load(const T* src, int64_t i) {
    if constexpr (sizeof(T) == 1) return FAST ? div_fast((float)src[i], 255.f, 1.f / 255.f) : (float)src[i] / 255.f;
    else return src[i];
}

// One output pixel of the transform (normalise, then bilinear resize with align_corners=False; ATen
// area_pixel_compute_source_index) from image plane base xb [3][H][W]: the three channels and a zero
// fourth.  Shared by the transform kernel and the SSD stem that folds the transform in, so both
// produce the same bits.
template <typename T, bool FAST = false>
__device__ __forceinline__ f32x4 pre_pixel(const T* __restrict__ xb, int H, int W, float sh, float sw,
                                           const float* mean, const float* stdv, const float* rstd, int oy, int ox) {
    // ATen's CPU upsample_bilinear2d as built (contracted): src = fma(scale, dst + 0.5, -0.5), clamped
    // at 0; index = min(floor(src), size - 1); lambda = clamp(src - index, 0, 1); each linear step
    // fma(t0, lambda0, t1 * lambda1), width first (bit-identical to F.interpolate on the CPU oracle,
    // tests/test_resize_rule.py)
    float ry = __builtin_fmaf(sh, (float)oy + 0.5f, -0.5f);
    float rx = __builtin_fmaf(sw, (float)ox + 0.5f, -0.5f);
    ry = ry < 0.f ? 0.f : ry;
    rx = rx < 0.f ? 0.f : rx;
    const int y0 = min((int)ry, H - 1), x0 = min((int)rx, W - 1);
    const int y1 = y0 + ((y0 < H - 1) ? 1 : 0);
    const int x1 = x0 + ((x0 < W - 1) ? 1 : 0);
    const float ly = fminf(fmaxf(ry - (float)y0, 0.f), 1.f), lx = fminf(fmaxf(rx - (float)x0, 0.f), 1.f);
    const float hy = 1.f - ly, hx = 1.f - lx;
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const T* src = xb + (int64_t)c * H * W;
        auto norm = [&](int64_t i) {
            const float a = pre_load<T, FAST>(src, i) - mean[c];
            return FAST ? div_fast(a, stdv[c], rstd[c]) : a / stdv[c];
        };
        const float a00 = norm((int64_t)y0 * W + x0);
        const float a01 = norm((int64_t)y0 * W + x1);
        const float a10 = norm((int64_t)y1 * W + x0);
        const float a11 = norm((int64_t)y1 * W + x1);
        v[c] = __builtin_fmaf(__builtin_fmaf(a00, hx, a01 * lx), hy, __builtin_fmaf(a10, hx, a11 * lx) * ly);
    }
    return f32x4{v[0], v[1], v[2], 0.f};
}

// Host: may the uint8 transform use div_fast?  Every operand a uint8 image can give either division
// (x = 0..255; then (x / 255 - mean_c) for each channel) is checked against the IEEE division; rstd
// receives RN(1 / std_c).  (Host float arithmetic is IEEE single with -ffp-contract=off, fmaf exact.)
static bool u8_fast_div(const float mean[3], const float stdv[3], float rstd[3]) {
    const float r255 = 1.f / 255.f;
    for (int c = 0; c < 3; ++c) rstd[c] = 1.f / stdv[c];
    auto same = [](float a, float b) { return __builtin_memcmp(&a, &b, sizeof(float)) == 0; };
    auto fast = [](float a, float b, float rb) {
        const float q = a * rb;
        return std::fma(std::fma(-q, b, a), rb, q);
    };
    for (int x = 0; x < 256; ++x) {
        const float xf = (float)x, t = xf / 255.f;
        if (!same(fast(xf, 255.f, r255), t)) return false;
        for (int c = 0; c < 3; ++c) {
            const float a = t - mean[c];
            if (!same(fast(a, stdv[c], rstd[c]), a / stdv[c])) return false;
        }
    }
    return true;
}

template <typename T, bool FAST>
__global__ void preprocess_kernel(PreParams p, const T* __restrict__ x) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)p.B * p.Hp * p.Wp;
    if (idx >= total) return;
    const int ox = (int)(idx % p.Wp);
    const int oy = (int)((idx / p.Wp) % p.Hp);
    const int b = (int)(idx / ((int64_t)p.Wp * p.Hp));
    f32x4 out = {0.f, 0.f, 0.f, 0.f};
    if (oy < p.Ho && ox < p.Wo) out = pre_pixel<T, FAST>(x + (int64_t)b * 3 * p.H * p.W, p.H, p.W, p.sh, p.sw, p.mean, p.stdv, p.rstd, oy, ox);
    *reinterpret_cast<f32x4*>(p.y + idx * 4) = out;
}

int preprocess_launch(const PreParams& p0, hipStream_t s) {
    PreParams p = p0;
    EDGEDET_REQUIRE(p.y && ((p.x != nullptr) != (p.xu8 != nullptr)), "preprocess: null y, or not exactly one of x (f32) / x (u8)");
    EDGEDET_REQUIRE(p.Hp >= p.Ho && p.Wp >= p.Wo && p.Ho > 0 && p.Wo > 0, "preprocess: bad sizes");
    p.sh = (float)p.H / (float)p.Ho;
    p.sw = (float)p.W / (float)p.Wo;
    const int64_t total = (int64_t)p.B * p.Hp * p.Wp;
    p.fastdiv = p.xu8 && u8_fast_div(p.mean, p.stdv, p.rstd);
    if (p.xu8) {
        void (*k)(PreParams, const uint8_t*) = p.fastdiv ? preprocess_kernel<uint8_t, true> : preprocess_kernel<uint8_t, false>;
        hipLaunchKernelGGL(k, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p, p.xu8);
    } else {
        void (*k)(PreParams, const float*) = preprocess_kernel<float, false>;
        hipLaunchKernelGGL(k, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p, p.x);
    }
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ depthwise

__global__ void dwconv_kernel(DwParams p) {
    const int C4 = p.C >> 2;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)p.B * p.Ho * p.Wo * C4;
    if (idx >= total) return;
    const int c = (int)(idx % C4) * 4;
    const int64_t pix = idx / C4;
    const int ow = (int)(pix % p.Wo);
    const int oh = (int)((pix / p.Wo) % p.Ho);
    const int b = (int)(pix / ((int64_t)p.Wo * p.Ho));
    const float* xb = p.x + (int64_t)b * p.H * p.W * p.C + c;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int ih0 = oh * p.stride - p.pad, iw0 = ow * p.stride - p.pad;
    for (int kh = 0; kh < p.K; ++kh) {
        const int ih = ih0 + kh;
        if ((unsigned)ih >= (unsigned)p.H) continue;
        for (int kw = 0; kw < p.K; ++kw) {
            const int iw = iw0 + kw;
            if ((unsigned)iw >= (unsigned)p.W) continue;
            const f32x4 xv = *reinterpret_cast<const f32x4*>(xb + ((int64_t)ih * p.W + iw) * p.C);
            const f32x4 wv = *reinterpret_cast<const f32x4*>(p.w + (kh * p.K + kw) * p.C + c);
            acc.x = fmaf(xv.x, wv.x, acc.x);
            acc.y = fmaf(xv.y, wv.y, acc.y);
            acc.z = fmaf(xv.z, wv.z, acc.z);
            acc.w = fmaf(xv.w, wv.w, acc.w);
        }
    }
    const f32x4 bv = *reinterpret_cast<const f32x4*>(p.bias + c);
    f32x4 o;
    o.x = apply_act(acc.x + bv.x, p.act);
    o.y = apply_act(acc.y + bv.y, p.act);
    o.z = apply_act(acc.z + bv.z, p.act);
    o.w = apply_act(acc.w + bv.w, p.act);
    *reinterpret_cast<f32x4*>(p.y + pix * p.C + c) = o;
}

// Depthwise conv + folded BN + act that also emits the SqueezeExcitation squeeze: partial channel
// sums part[b][s][c] over pixel split s (p.parts <= SE_PARTS splits, reduced in fixed order by
// se_fc1_kernel).
// grid (cdiv(C, 64), SE_PARTS, B); block 256 = 16 channel quads x 16 pixel lanes, so one wave
// writes 4 pixels x 256 contiguous bytes.
__global__ void __launch_bounds__(256) dwconv_se_kernel(DwParams p) {
    __shared__ f32x4 red[16][16];
    const int cq = threadIdx.x & 15, pl = threadIdx.x >> 4;
    const int c = blockIdx.x * 64 + cq * 4;
    const int sidx = blockIdx.y, b = blockIdx.z;
    const int HWo = p.Ho * p.Wo;
    const int p0 = (int)((int64_t)sidx * HWo / p.parts), p1 = (int)((int64_t)(sidx + 1) * HWo / p.parts);
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    if (c < p.C) {
        const float* xb = p.x + (int64_t)b * p.H * p.W * p.C + c;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(p.bias + c);
        for (int pix = p0 + pl; pix < p1; pix += 16) {
            const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
            const int ih0 = oh * p.stride - p.pad, iw0 = ow * p.stride - p.pad;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            for (int kh = 0; kh < p.K; ++kh) {
                const int ih = ih0 + kh;
                if ((unsigned)ih >= (unsigned)p.H) continue;
                for (int kw = 0; kw < p.K; ++kw) {
                    const int iw = iw0 + kw;
                    if ((unsigned)iw >= (unsigned)p.W) continue;
                    const f32x4 xv = *reinterpret_cast<const f32x4*>(xb + ((int64_t)ih * p.W + iw) * p.C);
                    const f32x4 wv = *reinterpret_cast<const f32x4*>(p.w + (kh * p.K + kw) * p.C + c);
                    acc.x = fmaf(xv.x, wv.x, acc.x);
                    acc.y = fmaf(xv.y, wv.y, acc.y);
                    acc.z = fmaf(xv.z, wv.z, acc.z);
                    acc.w = fmaf(xv.w, wv.w, acc.w);
                }
            }
            f32x4 o;
            o.x = apply_act(acc.x + bv.x, p.act);
            o.y = apply_act(acc.y + bv.y, p.act);
            o.z = apply_act(acc.z + bv.z, p.act);
            o.w = apply_act(acc.w + bv.w, p.act);
            *reinterpret_cast<f32x4*>(p.y + ((int64_t)b * HWo + pix) * p.C + c) = o;
            sum += o;
        }
    }
    red[pl][cq] = sum;
    __syncthreads();
    if (pl == 0 && c < p.C) {
        f32x4 t = red[0][cq];
        for (int q = 1; q < 16; ++q) t += red[q][cq];
        *reinterpret_cast<f32x4*>(p.part + ((int64_t)b * p.parts + sidx) * p.C + c) = t;
    }
}

// Register-blocked depthwise conv for the MobileNetV3 shapes (K in {3,5}, stride in {1,2}): a
// thread computes PW horizontally adjacent outputs of one channel quad, loading each input row
// segment once into registers ((PW-1)*S+K f32x4 per kernel row instead of PW*K), so L1/TA traffic
// per output drops by ~K/(1+(K-1)/PW).  Accumulation order per output is (kh, kw) as in the
// scalar kernel.  SE variant: grid (cdiv(C/4,16), SE_PARTS, B), block = 16 quads x 16 group lanes,
// partial sums per pixel-group split (see dwconv_se_kernel).
template <int K, int S, int PW>
__device__ __forceinline__ void dw_group(const DwParams& p, const float* __restrict__ xb, int oh, int ow0, int c,
                                         f32x4 (&acc)[PW]) {
    constexpr int IW = (PW - 1) * S + K;
#pragma unroll
    for (int o = 0; o < PW; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ih0 = oh * S - p.pad, iw0 = ow0 * S - p.pad;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
        const int ih = ih0 + kh;
        if ((unsigned)ih >= (unsigned)p.H) continue;
        const float* row = xb + (int64_t)ih * p.W * p.C;
        f32x4 xin[IW];
#pragma unroll
        for (int j = 0; j < IW; ++j) {
            const int iw = iw0 + j;
            xin[j] = (unsigned)iw < (unsigned)p.W ? *reinterpret_cast<const f32x4*>(row + (int64_t)iw * p.C)
                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
            const f32x4 wv = *reinterpret_cast<const f32x4*>(p.w + (kh * K + kw) * p.C + c);
#pragma unroll
            for (int o = 0; o < PW; ++o) {
                const f32x4 xv = xin[o * S + kw];
                acc[o].x = fmaf(xv.x, wv.x, acc[o].x);
                acc[o].y = fmaf(xv.y, wv.y, acc[o].y);
                acc[o].z = fmaf(xv.z, wv.z, acc[o].z);
                acc[o].w = fmaf(xv.w, wv.w, acc[o].w);
            }
        }
    }
}

template <int K, int S, int PW>
__device__ __forceinline__ void dwconv_rb_body(const DwParams& p, int nq, int nwg, int64_t idx) {
    const int64_t total = (int64_t)p.B * p.Ho * nwg * nq;
    if (idx >= total) return;
    const int q = (int)(idx % nq);
    int64_t r = idx / nq;
    const int wg = (int)(r % nwg);
    r /= nwg;
    const int oh = (int)(r % p.Ho);
    const int b = (int)(r / p.Ho);
    const int c = q * 4, ow0 = wg * PW;
    f32x4 acc[PW];
    dw_group<K, S, PW>(p, p.x + (int64_t)b * p.H * p.W * p.C + c, oh, ow0, c, acc);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(p.bias + c);
    float* yb = p.y + (((int64_t)b * p.Ho + oh) * p.Wo + ow0) * p.C + c;
    const int act = p.act;
#pragma unroll
    for (int o = 0; o < PW; ++o) {
        if (ow0 + o < p.Wo) {
            f32x4 v;
            v.x = apply_act(acc[o].x + bv.x, act);
            v.y = apply_act(acc[o].y + bv.y, act);
            v.z = apply_act(acc[o].z + bv.z, act);
            v.w = apply_act(acc[o].w + bv.w, act);
            *reinterpret_cast<f32x4*>(yb + (int64_t)o * p.C) = v;
        }
    }
}

template <int K, int S, int PW>
__global__ void __launch_bounds__(256) dwconv_rb_kernel(DwParams p, int nq, int nwg) {
    dwconv_rb_body<K, S, PW>(p, nq, nwg, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// Grouped form (csrc/exec.hip EDGEDET_OP_GROUP): up to EDGEDET_MAX_GROUP depthwise problems of one
// (K, stride) in one launch (the twelve SSDLite head depthwise convs); workgroups [start[k], start[k+1])
// run problem k.
template <int K, int S, int PW>
__global__ void __launch_bounds__(256) dwconv_rb_group_kernel(DwGroup g) {
    const int bx = (int)blockIdx.x;
    int k = 0;
    while (k + 1 < g.n && bx >= g.start[k + 1]) ++k;
    dwconv_rb_body<K, S, PW>(g.p[k], g.nq[k], g.nwg[k], (int64_t)(bx - g.start[k]) * blockDim.x + threadIdx.x);
}

template <int K, int S, int PW, int QL = 16>
__global__ void __launch_bounds__(256) dwconv_rb_se_kernel(DwParams p, int nq, int nwg) {
    constexpr int GL = 256 / QL;  // group lanes per channel quad (QL quads per workgroup)
    __shared__ f32x4 red[GL][QL];
    const int ql = threadIdx.x % QL, gl = threadIdx.x / QL;
    const int q = blockIdx.x * QL + ql;
    const int c = q * 4;
    const int sidx = blockIdx.y, b = blockIdx.z;
    const int G = p.Ho * nwg;
    const int g0 = (int)((int64_t)sidx * G / p.parts), g1 = (int)((int64_t)(sidx + 1) * G / p.parts);
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    if (q < nq) {
        const float* xb = p.x + (int64_t)b * p.H * p.W * p.C + c;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(p.bias + c);
        const int act = p.act;
        for (int g = g0 + gl; g < g1; g += GL) {
            const int oh = g / nwg, ow0 = (g - oh * nwg) * PW;
            f32x4 acc[PW];
            dw_group<K, S, PW>(p, xb, oh, ow0, c, acc);
            float* yb = p.y + (((int64_t)b * p.Ho + oh) * p.Wo + ow0) * p.C + c;
#pragma unroll
            for (int o = 0; o < PW; ++o) {
                if (ow0 + o < p.Wo) {
                    f32x4 v;
                    v.x = apply_act(acc[o].x + bv.x, act);
                    v.y = apply_act(acc[o].y + bv.y, act);
                    v.z = apply_act(acc[o].z + bv.z, act);
                    v.w = apply_act(acc[o].w + bv.w, act);
                    *reinterpret_cast<f32x4*>(yb + (int64_t)o * p.C) = v;
                    sum += v;
                }
            }
        }
    }
    red[gl][ql] = sum;
    __syncthreads();
    if (gl == 0 && q < nq) {
        f32x4 t = red[0][ql];
        for (int k = 1; k < GL; ++k) t += red[k][ql];
        *reinterpret_cast<f32x4*>(p.part + ((int64_t)b * p.parts + sidx) * p.C + c) = t;
    }
}

template <int K, int S>
static int dwconv_rb_launch(const DwParams& p, hipStream_t s) {
    constexpr int PW = 4;
    const int nq = p.C / 4, nwg = cdiv(p.Wo, PW);
    if (p.part) {
        // 16 channel quads x 16 group lanes per workgroup, 4 outputs per thread: against 8 x 32 and
        // 2 outputs per thread, alternated SSD runs 31.59k / 31.48k vs 31.34k / 31.29k (8 x 32),
        // 30.98k / 31.00k and 30.90k / 30.99k (2 outputs) (profiles/r4h_ab_dwse.txt)
        hipLaunchKernelGGL((dwconv_rb_se_kernel<K, S, PW>), dim3((unsigned)cdiv(nq, 16), p.parts, p.B), dim3(256), 0,
                           s, p, nq, nwg);
    } else {
        const int64_t total = (int64_t)p.B * p.Ho * nwg * nq;
        hipLaunchKernelGGL((dwconv_rb_kernel<K, S, PW>), dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p, nq,
                           nwg);
    }
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ SSDLite stem
// features.0.0 (conv 3x3 s2, 3(+1 pad) -> 16, folded BN, hardswish) and features.0.1 (depthwise 3x3
// 16 + BN + ReLU, projection 1x1 16 -> 16 + BN, + the stem output) in one pass: the two 16-channel
// 160x160 tensors between them never reach HBM.  Block = one image, a 16 x 16 output tile:
//   1. the 37 x 37 x 4 input tile (stride-2 receptive field of the 18 x 18 stem halo) into LDS;
//   2. stem outputs on the 18 x 18 halo (zero outside the map: the depthwise pads them) as a GEMM on
//      the matrix cores, [324 halo pixels] x [36 = 9 taps x 4 channels] x [16], one
//      v_mfma_f32_16x16x4_f32 per tap (exact fp32 products);
//   3. per output pixel: depthwise on the vector ALUs (taps (kh, kw) as dw_group), then the projection
//      as a [256 pixels] x [16] x [16] MFMA GEMM, + bias, + residual.
// The matrix-core form replaced one pixel x 16 channels per thread on the vector ALUs for phases 2 and
// 3 (SSD 30.63k / 30.63k -> 30.87k / 30.95k img/s in ABBA-ordered runs, profiles/r4c_ab.txt).  The
// weights (1024 floats) are staged in LDS with the input tile, in the same memory round trip (as
// scalar loads they did not fit the SGPRs and were re-fetched per pixel).
constexpr int STEM_T = 16, STEM_SH = STEM_T + 2, STEM_XH = 2 * STEM_SH + 1, STEM_SS = 20;
// LDS weight image: w0 [16][36] (taps (kh, kw, ci)), b0 [16], wd [9][16], bd [16], w1 [16][16], b1 [16]
constexpr int STEM_W0 = 0, STEM_B0 = 576, STEM_WD = 592, STEM_BD = 736, STEM_W1 = 752, STEM_B1 = 1008, STEM_NW = 1024;

// T = float: the transform's NHWC4 output (p.x); T = float / uint8_t with FUSED: the source image
// (p.src / p.src8, [B][3][H0][W0]) and the transform computed per input pixel of the tile (pre_pixel,
// the same bits as the transform kernel): no transform launch and no NHWC4 round trip through HBM.
template <typename T, bool FUSED, bool FAST = false>
__global__ void __launch_bounds__(256) ssd_stem_kernel(StemParams p, int tiles_w) {
    __shared__ __attribute__((aligned(16))) float xs[STEM_XH * STEM_XH * 4];
    __shared__ __attribute__((aligned(16))) float ss[STEM_SH * STEM_SH * STEM_SS];
    __shared__ __attribute__((aligned(16))) float ws[STEM_NW];
    const int tid = threadIdx.x, b = blockIdx.y;
    const int oh0 = (blockIdx.x / tiles_w) * STEM_T, ow0 = (blockIdx.x % tiles_w) * STEM_T;
    const int sh0 = oh0 - 1, sw0 = ow0 - 1;          // stem-output halo origin
    const int xh0 = 2 * sh0 - 1, xw0 = 2 * sw0 - 1;  // input tile origin (stem pad 1, stride 2)
    const float* xb = FUSED ? nullptr : p.x + (int64_t)b * p.H * p.W * 4;
    {  // all of a thread's input pixels and weights in flight at once (one memory round trip)
        float wv[STEM_NW / 256];
#pragma unroll
        for (int r = 0; r < STEM_NW / 256; ++r) {
            const int e = tid + 256 * r;
            const float* src = e < STEM_B0   ? p.w0 + (e / 36) * p.ld0 + e % 36
                               : e < STEM_WD ? p.b0 + (e - STEM_B0)
                               : e < STEM_BD ? p.wd + (e - STEM_WD)
                               : e < STEM_W1 ? p.bd + (e - STEM_BD)
                               : e < STEM_B1 ? p.w1 + ((e - STEM_W1) / 16) * p.ld1 + (e - STEM_W1) % 16
                                             : p.b1 + (e - STEM_B1);
            wv[r] = *src;
        }
        constexpr int R = (STEM_XH * STEM_XH + 255) / 256;
        f32x4 xv[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int v = tid + 256 * r;
            const int ih = xh0 + v / STEM_XH, iw = xw0 + v % STEM_XH;
            const bool in = v < STEM_XH * STEM_XH && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
            if constexpr (FUSED) {
                const T* img = (const T*)(sizeof(T) == 1 ? (const void*)p.src8 : (const void*)p.src) +
                               (int64_t)b * 3 * p.H0 * p.W0;
                xv[r] = in ? pre_pixel<T, FAST>(img, p.H0, p.W0, p.sh, p.sw, p.mean, p.stdv, p.rstd, ih, iw)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
            } else {
                const float* src = xb + (in ? ((int64_t)ih * p.W + iw) * 4 : 0);  // clamped: loads stay unconditional
                xv[r] = *reinterpret_cast<const f32x4*>(src);
                if (!in) xv[r] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (tid + 256 * r < STEM_XH * STEM_XH) *reinterpret_cast<f32x4*>(xs + 4 * (tid + 256 * r)) = xv[r];
#pragma unroll
        for (int r = 0; r < STEM_NW / 256; ++r) ws[tid + 256 * r] = wv[r];
    }
    __syncthreads();
    const int lane = tid & 63, wid = tid >> 6, l16 = lane & 15, q4 = lane >> 4;
    // stem conv as a GEMM on the matrix cores (v_mfma_f32_16x16x4_f32, exact fp32 products): rows =
    // the 324 halo pixels in 21 tiles of 16 (wave w takes tiles w, w + 4, ...), columns = the 16
    // output channels, K = 9 taps x 4 channels in the packed (kh, kw, ci) order (one MFMA per tap)
    float wb[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wb[t] = ws[STEM_W0 + l16 * 36 + 4 * t + q4];
    const float b0v = ws[STEM_B0 + l16];
    constexpr int NV = STEM_SH * STEM_SH, NTL = (NV + 15) / 16;
    for (int tl = wid; tl < NTL; tl += 4) {
        const int va = min(16 * tl + l16, NV - 1);  // this lane's A row (pad rows repeat the last pixel)
        const int lh = va / STEM_SH, lw = va - lh * STEM_SH;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const float av = xs[4 * ((2 * lh + t / 3) * STEM_XH + 2 * lw + t % 3) + q4];
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wb[t], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int v = 16 * tl + 4 * q4 + i;
            if (v < NV) {
                const int vh = v / STEM_SH, vw = v - vh * STEM_SH;
                const bool in = (unsigned)(sh0 + vh) < (unsigned)p.Ho && (unsigned)(sw0 + vw) < (unsigned)p.Wo;
                ss[v * STEM_SS + l16] = in ? apply_act(acc[i] + b0v, ACT_HSWISH) : 0.f;
            }
        }
    }
    __syncthreads();
    const int lh = tid / STEM_T, lw = tid % STEM_T;
    const int oh = oh0 + lh, ow = ow0 + lw;
    // depthwise on the vector ALUs (one output pixel x 16 channels per thread, taps (kh, kw)), its
    // outputs through LDS (the input tile's space, free now) into the projection GEMM on the matrix
    // cores: rows = the wave's 64 pixels in 4 tiles, columns = 16 channels, K = 16 in 4 steps
    float dv[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) dv[c] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
        if ((unsigned)(oh - 1 + kh) >= (unsigned)p.Ho) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const float* sv = ss + ((lh + kh) * STEM_SH + lw + kw) * STEM_SS;
            const float* wv = ws + STEM_WD + (kh * 3 + kw) * 16;
#pragma unroll
            for (int c = 0; c < 16; ++c) dv[c] = fmaf(sv[c], wv[c], dv[c]);
        }
    }
    constexpr int DS = 17;  // odd pitch
    float* dsm = xs;        // [256][DS]
#pragma unroll
    for (int c = 0; c < 16; ++c) dsm[tid * DS + c] = apply_act(dv[c] + ws[STEM_BD + c], ACT_RELU);
    float w1v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w1v[k] = ws[STEM_W1 + l16 * 16 + 4 * k + q4];
    const float b1v = ws[STEM_B1 + l16];
    __syncthreads();
#pragma unroll
    for (int tl = 0; tl < 4; ++tl) {
        const int row0 = 64 * wid + 16 * tl;  // the tile's first output pixel (= thread index)
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dsm[(row0 + l16) * DS + 4 * k + q4], w1v[k], acc, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int px = row0 + 4 * q4 + i, ph = px / STEM_T, pw = px % STEM_T;
            const int yh = oh0 + ph, yw = ow0 + pw;
            if (yh < p.Ho && yw < p.Wo) {
                const float r = ss[((ph + 1) * STEM_SH + pw + 1) * STEM_SS + l16];
                p.y[(((int64_t)b * p.Ho + yh) * p.Wo + yw) * 16 + l16] = (acc[i] + b1v) + r;
            }
        }
    }
}

int ssd_stem_launch(const StemParams& p0, hipStream_t s) {
    StemParams p = p0;
    const bool fused = p.src || p.src8;
    EDGEDET_REQUIRE((p.x || fused) && p.w0 && p.b0 && p.wd && p.bd && p.w1 && p.b1 && p.y, "ssd_stem: null pointer");
    EDGEDET_REQUIRE(!(p.src && p.src8), "ssd_stem: one source image (float or uint8)");
    if (fused) {
        EDGEDET_REQUIRE(p.H0 >= 1 && p.W0 >= 1, "ssd_stem: source image size");
        p.sh = (float)p.H0 / (float)p.H;  // as the transform kernel's input / output scales
        p.sw = (float)p.W0 / (float)p.W;
    }
    EDGEDET_REQUIRE(p.Ho == (p.H - 1) / 2 + 1 && p.Wo == (p.W - 1) / 2 + 1, "ssd_stem: 3x3 stride 2 pad 1 shape");
    EDGEDET_REQUIRE(p.ld0 >= 36 && p.ld1 >= 16, "ssd_stem: weight row strides");
    const int tiles_w = cdiv(p.Wo, STEM_T);
    const dim3 grid((unsigned)(cdiv(p.Ho, STEM_T) * tiles_w), (unsigned)p.B);
    p.fastdiv = p.src8 && u8_fast_div(p.mean, p.stdv, p.rstd);
    void (*k)(StemParams, int) = p.src8 ? (p.fastdiv ? ssd_stem_kernel<uint8_t, true, true> : ssd_stem_kernel<uint8_t, true>)
                                 : p.src ? ssd_stem_kernel<float, true> : ssd_stem_kernel<float, false>;
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, p, tiles_w);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

extern "C" int edgedet_ssd_stem(const float* x, int64_t B, int64_t H, int64_t W, const float* w0, int64_t ld0,
                                const float* b0, const float* wd, const float* bd, const float* w1, int64_t ld1,
                                const float* b1, float* y, void* stream) {
    StemParams p{};
    p.x = x;
    p.w0 = w0;
    p.b0 = b0;
    p.wd = wd;
    p.bd = bd;
    p.w1 = w1;
    p.b1 = b1;
    p.y = y;
    p.B = (int)B;
    p.H = (int)H;
    p.W = (int)W;
    p.Ho = (int)((H - 1) / 2 + 1);
    p.Wo = (int)((W - 1) / 2 + 1);
    p.ld0 = (int)ld0;
    p.ld1 = (int)ld1;
    return ssd_stem_launch(p, (hipStream_t)stream);
}

// ------------------------------------------------------------------------------ fused MBConv
// A whole torchvision InvertedResidual without SqueezeExcitation (SSDLite blocks
// 0.2 / 0.3 at 160^2 / 80^2): expand 1x1 (+ folded BN, act), depthwise KxK stride S (+ folded BN, act),
// project 1x1 (+ folded BN), + the block input when S == 1 and Cin == Cout.  Neither the 3-4x-wide
// expanded tensor nor the depthwise output reaches HBM.
// Block = one image's TH x TW output tile (8 x 8 at stride 1, 4 x 8 at stride 2); one wave per 16
// expanded channels (Cexp <= 128: up to 8 waves).  The input halo is staged in LDS once (the only
// barrier before the final reduction); after it each wave runs its own chunk start to end with no
// workgroup barrier — the round-2 / early round-3 forms shared 32-channel chunks between the waves and
// paid four barriers per chunk, and measured at 15-20 TFLOP/s with half the wave time waiting:
//   expand   v_mfma_f32_16x16x4_f32 (exact fp32): [halo pixels] x [Cin] x [the wave's 16 channels],
//            two independent accumulation chains at a time; + bias, act; halo pixels outside the image
//            are zero (the depthwise conv pads the expanded tensor with zeros); into the wave's LDS;
//   depthwise lane = (channel, row group), a K x K register window slid along the row (3 or 6 new
//            LDS reads per output instead of 9), taps in (kh, kw) order, + bias, act; into LDS;
//   project  v_mfma_f32_16x16x4_f32: [tile pixels] x [the wave's 16 channels] x [Cout <= 32];
// then the waves' partial projections are added in wave order ((w0 + w1) + w2 ...), + bias (+ the
// input pixel), and stored.  All weights live in registers, loaded before the halo.
constexpr int MBW_C = 16;    // expanded channels per wave
constexpr int MBW_MAXW = 8;  // waves per workgroup (Cexp <= 128)

template <int K, int S, int CINP, int TH, int TW>
struct MbwGeom {
    static constexpr int IHh = (TH - 1) * S + K, IWh = (TW - 1) * S + K;  // halo rows, columns
    static constexpr int NPX = IHh * IWh, NPXP = (NPX + 15) / 16 * 16;
    static constexpr int P = TH * TW;                                       // output pixels (16k)
    static constexpr int XS = CINP + 1;                                     // odd pitches: spread banks
    static constexpr int ES = MBW_C + 1;
    static constexpr int PS = 33;                                           // partial sums: 32 + 1
    static constexpr int EW = NPXP * ES > P * PS ? NPXP * ES : P * PS;      // per wave: chunk, then partials
    static size_t smem(int nw) { return 4 * ((size_t)NPXP * (XS + 1) + (size_t)nw * (EW + P * ES)); }
};

// A workgroup barrier for LDS traffic only: __syncthreads' workgroup fence also waits for every
// outstanding global load and store (vmcnt(0)), which would land the next tile's halo prefetch and the
// previous tile's output stores on each barrier; the waves of this kernel exchange data through LDS
// only.
__device__ __forceinline__ void mbw_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void mbw_wave_sync() {  // this wave's LDS writes visible to its own lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int K, int S, int ACT, int CINP, int TH, int TW>
__global__ void __launch_bounds__(64 * MBW_MAXW, 4) mbconv_kernel(MbParams p, int tiles_w, int tiles_img, int ntiles) {
    using G = MbwGeom<K, S, CINP, TH, TW>;
    constexpr int IWh = G::IWh, NPX = G::NPX, NPXP = G::NPXP, P = G::P;
    constexpr int XS = G::XS, ES = G::ES, PS = G::PS, EW = G::EW;
    constexpr int NT = NPXP / 16, KS = CINP / 4, PT = P / 16, Q4 = CINP / 4;
    constexpr int HR = (NPXP * Q4 + 255) / 256;  // halo float4s per thread (at least four waves)
    static_assert(P % 16 == 0 && TW % 4 == 0 && NPXP <= 256, "mbconv: tile shape");
    extern __shared__ __attribute__((aligned(16))) float mb_smem[];
    const int nt = (int)blockDim.x, nw = nt >> 6;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l16 = lane & 15, q = lane >> 4;
    float* xs = mb_smem;                                        // [NPXP][XS] input halo
    float* es = mb_smem + NPXP * XS + wid * EW;                 // [NPXP][ES] expanded chunk; later [P][PS]
    float* ds = mb_smem + NPXP * XS + nw * EW + wid * P * ES;   // [P][ES] depthwise outputs
    float* xm = mb_smem + NPXP * XS + nw * (EW + P * ES);       // [NPXP] 1 inside the image, else 0
    const int Cin = p.Cin, Cexp = p.Cexp, Cout = p.Cout;
    const int ch = wid * MBW_C + l16;  // this lane's expanded channel
    const bool chv = ch < Cexp;
    // weights in registers for the workgroup's lifetime; every load issued unconditionally (a clamped
    // index, the value masked) so they are all in flight together
    float w1r[KS], w2r[4][2], wdr[K * K];
    const int chc = chv ? ch : 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const bool ok = chv && 4 * s + q < Cin;
        const float v = p.w1[(int64_t)chc * p.ld1 + (ok ? 4 * s + q : 0)];
        w1r[s] = ok ? v : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const int co = 16 * n + l16, k = wid * MBW_C + 4 * s + q;
            const bool ok = co < Cout && k < Cexp;
            const float v = p.w2[ok ? (int64_t)co * p.ld2 + k : 0];
            w2r[s][n] = ok ? v : 0.f;
        }
#pragma unroll
    for (int t = 0; t < K * K; ++t) {
        const float v = p.wd[(int64_t)t * Cexp + chc];
        wdr[t] = chv ? v : 0.f;
    }
    const float b1 = chv ? p.b1[chc] : 0.f, bd = chv ? p.bd[chc] : 0.f;
    // the output channel of this thread in the final sum (the element stride is a multiple of 32), its
    // bias loaded once: a load in that loop would sit behind the previous iteration's output store
    // (the compiler cannot prove p.b2 and p.y apart) and cost a memory round trip per element
    const int co_t = tid & 31;
    const float b2v = p.b2[co_t < Cout ? co_t : 0];
    // the halo of a tile: [NPX][Cin] as 16-byte loads (Cin % 4 == 0), zero outside the image / past Cin;
    // the next tile's halo is in flight in registers while the current tile is computed.  A thread's
    // halo slots (pixel row / column, channel quad) are the same for every tile: decomposed once.
    f32x4 hv[HR];
    int hr[HR], hc[HR], hoff[HR], hdst[HR];
#pragma unroll
    for (int u = 0; u < HR; ++u) {
        const int t = tid + nt * u, px = t / Q4, c4 = t - px * Q4;
        const bool live = t < NPXP * Q4 && px < NPX && 4 * c4 < Cin;
        hr[u] = live ? px / IWh : -(1 << 20);  // a dead slot never passes the bounds test
        hc[u] = px % IWh;
        hoff[u] = 4 * c4;
        hdst[u] = t < NPXP * Q4 ? px * XS + 4 * c4 : -1;
    }
    const int mr = tid < NPXP ? tid / IWh : 0, mc = tid % IWh;  // this thread's mask pixel (tid < NPXP)
    uint32_t hok = 0;
    auto load_halo = [&](int tile) {
        const int b = tile / tiles_img, r = tile - b * tiles_img, th = r / tiles_w, tw = r - th * tiles_w;
        const int ih0 = th * TH * S - p.pad, iw0 = tw * TW * S - p.pad;
        const float* xb = p.x + (int64_t)b * p.H * p.W * Cin;
#pragma unroll
        for (int u = 0; u < HR; ++u) {
            const int ih = ih0 + hr[u], iw = iw0 + hc[u];
            const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
            // one load path: the offset is zeroed (not selected) outside the image, and the value is
            // kept raw with an in-image bit; the select happens where it is stored, a tile later, so
            // nothing waits on these loads until then (a select or a conditional address here made the
            // compiler branch around the load and wait for every prefetch right after issuing it)
            const int off = ((ih * p.W + iw) * Cin + hoff[u]) * (int)ok;
            hv[u] = *reinterpret_cast<const f32x4*>(xb + off);
            hok = (hok & ~(1u << u)) | ((uint32_t)ok << u);
        }
    };
    int tile = blockIdx.x;
    if (tile < ntiles) load_halo(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        const int b = tile / tiles_img, r = tile - b * tiles_img, th = r / tiles_w, tw = r - th * tiles_w;
        const int oh0 = th * TH, ow0 = tw * TW, ih0 = oh0 * S - p.pad, iw0 = ow0 * S - p.pad;
        mbw_lds_barrier();  // the previous tile's reads of xs and of the partials are done
#pragma unroll
        for (int u = 0; u < HR; ++u) {
            if (hdst[u] >= 0) {
                const f32x4 v = (hok >> u) & 1 ? hv[u] : f32x4{0.f, 0.f, 0.f, 0.f};
                float* d = xs + hdst[u];
                d[0] = v.x;
                d[1] = v.y;
                d[2] = v.z;
                d[3] = v.w;
            }
        }
        if (tid < NPXP) {  // NPXP <= 4 waves of threads (the launcher's minimum)
            const int ih = ih0 + mr, iw = iw0 + mc;
            xm[tid] = tid < NPX && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W ? 1.f : 0.f;
        }
        if (tile + (int)gridDim.x < ntiles) load_halo(tile + gridDim.x);
        mbw_lds_barrier();
        // expand: the wave's 16 channels over every halo pixel, two accumulation chains at a time
        // (x 0 outside the image: the depthwise conv zero-pads the expanded tensor)
        auto expand_store = [&](const f32x4& a, int t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = 16 * t + 4 * q + i;
                es[m * ES + l16] = apply_act(a[i] + b1, ACT) * xm[m];
            }
        };
#pragma unroll 1
        for (int t = 0; t < NT; t += 2) {
            f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
            const float* r0 = xs + (16 * t + l16) * XS + q;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(r0[4 * s], w1r[s], a0, 0, 0, 0);
                if (t + 1 < NT) a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(r0[16 * XS + 4 * s], w1r[s], a1, 0, 0, 0);
            }
            expand_store(a0, t);
            if (t + 1 < NT) expand_store(a1, t + 1);
        }
        mbw_wave_sync();
        // depthwise: lane = (channel l16, output rows q, q + 4, ...), a K x K window slid along the row
#pragma unroll 1
        for (int oy = q; oy < TH; oy += 4) {
            float win[K][K];
#pragma unroll
            for (int kh = 0; kh < K; ++kh)
#pragma unroll
                for (int kw = 0; kw < K; ++kw) win[kh][kw] = es[((oy * S + kh) * IWh + kw) * ES + l16];
#pragma unroll
            for (int ox = 0; ox < TW; ++ox) {
                if (ox > 0) {
#pragma unroll
                    for (int kh = 0; kh < K; ++kh) {
#pragma unroll
                        for (int kw = 0; kw < K - S; ++kw) win[kh][kw] = win[kh][kw + S];
#pragma unroll
                        for (int kw = K - S; kw < K; ++kw)
                            win[kh][kw] = es[((oy * S + kh) * IWh + ox * S + kw) * ES + l16];
                    }
                }
                float a = 0.f;
#pragma unroll
                for (int kh = 0; kh < K; ++kh)
#pragma unroll
                    for (int kw = 0; kw < K; ++kw) a = fmaf(win[kh][kw], wdr[kh * K + kw], a);
                ds[(oy * TW + ox) * ES + l16] = apply_act(a + bd, ACT);
            }
        }
        mbw_wave_sync();
        // project the wave's 16 channels: acc[pixel tile][Cout half]
        f32x4 acc[PT][2];
#pragma unroll
        for (int t = 0; t < PT; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < PT; ++t) {
                const float a = ds[(16 * t + l16) * ES + 4 * s + q];
                acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w2r[s][0], acc[t][0], 0, 0, 0);
                acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w2r[s][1], acc[t][1], 0, 0, 0);
            }
        // the partials replace the expanded chunk in this wave's region (its last reads were above)
#pragma unroll
        for (int t = 0; t < PT; ++t)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int i = 0; i < 4; ++i) es[(16 * t + 4 * q + i) * PS + 16 * n + l16] = acc[t][n][i];
        mbw_lds_barrier();
        // partials added in wave order, bias, residual (S == 1: the input pixel at the tap centre), store
        const float* part = mb_smem + NPXP * XS;
        for (int e = tid; e < P * 32; e += nt) {
            const int px = e >> 5, co = e & 31;
            const int ly = px / TW, lx = px - ly * TW, oh = oh0 + ly, ow = ow0 + lx;
            if (co >= Cout || oh >= p.Ho || ow >= p.Wo) continue;
            float v = part[px * PS + co];
            for (int w = 1; w < nw; ++w) v += part[w * EW + px * PS + co];
            v += b2v;
            if (p.residual) v += xs[((ly + p.pad) * IWh + lx + p.pad) * XS + co];
            p.y[(((int64_t)b * p.Ho + oh) * p.Wo + ow) * Cout + co] = v;
        }
    }
}

// Opt an instantiation into its dynamic LDS once per process (not a stream operation: legal while a
// graph is being captured).
template <typename KF>
static int mbw_set_lds(KF kernel, size_t bytes) {
    static std::mutex mu;
    static std::vector<std::pair<const void*, size_t>> done;
    std::lock_guard<std::mutex> lk(mu);
    for (auto& d : done)
        if (d.first == (const void*)kernel && d.second >= bytes) return 0;
    EDGEDET_CHECK_HIP(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    done.emplace_back((const void*)kernel, bytes);
    return 0;
}

template <int K, int S, int ACT, int CINP>
static int mbconv_launch_t(const MbParams& p, hipStream_t s) {
    constexpr int TH = S == 1 ? 8 : 4, TW = 8;
    using G = MbwGeom<K, S, CINP, TH, TW>;
    // at least four waves (the halo loader's stride); waves past Cexp carry zero weights
    const int nw = std::max(4, (int)cdiv(p.Cexp, MBW_C)), tiles_w = (int)cdiv(p.Wo, TW);
    const int tiles_img = (int)cdiv(p.Ho, TH) * tiles_w, ntiles = p.B * tiles_img;
    const size_t lds = G::smem(nw);
    EDGEDET_REQUIRE(lds <= 160 * 1024, "mbconv: tile exceeds the LDS");
    auto kern = mbconv_kernel<K, S, ACT, CINP, TH, TW>;
    if (int rc = mbw_set_lds(kern, lds)) return rc;
    // a resident grid (the workgroups that fit the CUs at once) looping over the tiles, each tile's
    // halo loaded under the previous tile's compute
    const int per_cu = std::max(1, (int)((160 * 1024) / lds));
    const int grid = std::min(ntiles, 256 * per_cu);
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * nw), lds, s, p, tiles_w, tiles_img, ntiles);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

template <int K, int S, int ACT>
static int mbconv_launch_a(const MbParams& p, hipStream_t s) {
    if (p.Cin <= 16) return mbconv_launch_t<K, S, ACT, 16>(p, s);
    if (p.Cin <= 24) return mbconv_launch_t<K, S, ACT, 24>(p, s);
    return mbconv_launch_t<K, S, ACT, 32>(p, s);
}

template <int K, int S>
static int mbconv_launch_ks(const MbParams& p, hipStream_t s) {
    switch (p.act) {
        case ACT_RELU: return mbconv_launch_a<K, S, ACT_RELU>(p, s);
        case ACT_RELU6: return mbconv_launch_a<K, S, ACT_RELU6>(p, s);
        case ACT_HSWISH: return mbconv_launch_a<K, S, ACT_HSWISH>(p, s);
        default: EDGEDET_REQUIRE(false, "mbconv: activation RE / R6 / HS");
    }
}

int mbconv_launch(const MbParams& p, hipStream_t s) {
    EDGEDET_REQUIRE(p.x && p.w1 && p.b1 && p.wd && p.bd && p.w2 && p.b2 && p.y, "mbconv: null pointer");
    EDGEDET_REQUIRE(p.Cin >= 1 && p.Cin <= 32 && p.Cin % 4 == 0 && p.Cout >= 1 && p.Cout <= 32 && p.Cexp >= 1 &&
                        p.Cexp <= MBW_C * MBW_MAXW,
                    "mbconv: Cin <= 32 (a multiple of 4), Cout <= 32, Cexp <= 128");
    EDGEDET_REQUIRE(((uintptr_t)p.x & 15) == 0, "mbconv: input 16-byte aligned");
    EDGEDET_REQUIRE(p.ld1 >= p.Cin && p.ld2 >= p.Cexp, "mbconv: weight row strides");
    EDGEDET_REQUIRE(p.pad == (p.K - 1) / 2 && p.Ho == (p.H + 2 * p.pad - p.K) / p.stride + 1 &&
                    p.Wo == (p.W + 2 * p.pad - p.K) / p.stride + 1, "mbconv: 'same' padding shape");
    EDGEDET_REQUIRE(!p.residual || (p.stride == 1 && p.Cin == p.Cout), "mbconv: residual needs stride 1, Cin == Cout");
    if (p.K == 3 && p.stride == 1) return mbconv_launch_ks<3, 1>(p, s);
    if (p.K == 3 && p.stride == 2) return mbconv_launch_ks<3, 2>(p, s);
    if (p.K == 5 && p.stride == 1) return mbconv_launch_ks<5, 1>(p, s);
    if (p.K == 5 && p.stride == 2) return mbconv_launch_ks<5, 2>(p, s);
    EDGEDET_REQUIRE(false, "mbconv: K in {3, 5}, stride in {1, 2}");
}

// Grouped launch of depthwise problems (exec.hip EDGEDET_OP_GROUP): every member a register-blocked
// shape (K 3 / 5, stride 1 / 2) of one (K, stride), no SE squeeze; returns 1 without launching when
// they are not, and the caller issues them one by one.
int dwconv_group_launch(const DwParams* ps, int n, hipStream_t s) {
    EDGEDET_REQUIRE(n >= 1 && n <= EDGEDET_MAX_GROUP, "dwconv group: 1..EDGEDET_MAX_GROUP members");
    constexpr int PW = 4;
    DwGroup g;
    g.n = n;
    const int K = ps[0].K, S = ps[0].stride;
    int64_t total = 0;
    for (int k = 0; k < n; ++k) {
        const DwParams& p = ps[k];
        EDGEDET_REQUIRE(p.x && p.w && p.bias && p.y && p.C % 4 == 0, "dwconv group: null pointer or C % 4 != 0");
        if (p.K != K || p.stride != S || p.part || !((K == 3 || K == 5) && (S == 1 || S == 2))) return 1;
        g.p[k] = p;
        g.nq[k] = p.C / 4;
        g.nwg[k] = cdiv(p.Wo, PW);
        g.start[k] = (int)total;
        total += cdiv((int64_t)p.B * p.Ho * g.nwg[k] * g.nq[k], 256);
        EDGEDET_REQUIRE(total < (1ll << 31), "dwconv group grid too large");
    }
    g.start[n] = (int)total;
    auto kern = K == 3 ? (S == 1 ? dwconv_rb_group_kernel<3, 1, PW> : dwconv_rb_group_kernel<3, 2, PW>)
                       : (S == 1 ? dwconv_rb_group_kernel<5, 1, PW> : dwconv_rb_group_kernel<5, 2, PW>);
    hipLaunchKernelGGL(kern, dim3((unsigned)total), dim3(256), 0, s, g);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

int dwconv_launch(const DwParams& p, hipStream_t s) {
    EDGEDET_REQUIRE(p.x && p.w && p.bias && p.y, "dwconv: null x/w/bias/y");
    EDGEDET_REQUIRE(p.C % 4 == 0, "dwconv: C must be a multiple of 4");
    if (p.part) EDGEDET_REQUIRE(p.parts >= 1 && p.parts <= SE_PARTS, "dwconv: 1..16 SE partial sums");
    if (p.K == 3 && p.stride == 1) return dwconv_rb_launch<3, 1>(p, s);
    if (p.K == 3 && p.stride == 2) return dwconv_rb_launch<3, 2>(p, s);
    if (p.K == 5 && p.stride == 1) return dwconv_rb_launch<5, 1>(p, s);
    if (p.K == 5 && p.stride == 2) return dwconv_rb_launch<5, 2>(p, s);
    if (p.part) {
        hipLaunchKernelGGL(dwconv_se_kernel, dim3((unsigned)cdiv(p.C, 64), p.parts, p.B), dim3(256), 0, s, p);
        EDGEDET_LAUNCH_CHECK();
        return 0;
    }
    const int64_t total = (int64_t)p.B * p.Ho * p.Wo * (p.C / 4);
    hipLaunchKernelGGL(dwconv_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ SE squeeze
// Standalone adaptive_avg_pool2d(1) for an SE whose producer is not a depthwise conv: grid
// (cdiv(C, 64), B), block 256 = 64 channels x 4 pixel groups, fixed-order reduction.  (The SSDLite
// blocks use the squeeze fused into dwconv_se_kernel instead.)
__global__ void channel_mean_kernel(const float* __restrict__ x, float* __restrict__ mean, int HW, int C) {
    __shared__ float red[4][64];
    const int b = blockIdx.y;
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    float acc = 0.f;
    if (c < C) {
        const float* xb = x + (int64_t)b * HW * C + c;
        for (int i = g; i < HW; i += 4) acc += xb[(int64_t)i * C];
    }
    red[g][cl] = acc;
    __syncthreads();
    if (g == 0 && c < C)
        mean[(int64_t)b * C + c] = (((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl]) / (float)HW;
}

int channel_mean_launch(const float* x, float* out, int B, int HW, int C, hipStream_t s) {
    EDGEDET_REQUIRE(x && out, "channel_mean: null pointer");
    hipLaunchKernelGGL(channel_mean_kernel, dim3((unsigned)cdiv(C, 64), B), dim3(256), 0, s, x, out, HW, C);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ SE excitation
// All B images share the SE weights, so the excitation runs as two small batched GEMVs tiled over
// many workgroups; each workgroup stages its operands in LDS with independent loads (one or two
// memory round trips instead of a dependent chain per element):
//   se_fc1: tile 8 images x 8 squeeze outputs.  mean[b][c] = (sum of the SE_PARTS partial sums in
//           fixed order) / HW for its 8 images, w1 rows [8][C]; hidden = relu(b1 + w1 . mean),
//           each output reduced over C quarters by 4 threads (fixed order).
//   se_fc2: tile 8 images x 64 channels.  hidden[8][S] and w2t [128-row chunks][64] in LDS;
//           scale = hardsigmoid(b2 + w2 . hidden), 2 outputs per thread.
constexpr int SE1_BB = 8, SE1_SB = 8, SE2_BB = 8, SE2_SCH = 128;
constexpr int SE_CMAX = 1024, SE_SMAX = 512;

// LDS staging with SE_U independent 16-byte loads in flight per thread (a plain strided loop waits for
// every load before issuing the next: one memory round trip per element, which dominated these
// latency-bound kernels).  dst (16-byte aligned) as f32x4 [t] = src4(t) for t < n4.
constexpr int SE_U = 8;
template <typename F>
__device__ __forceinline__ void se_stage4(float* dst, int n4, F src4) {
    for (int base = threadIdx.x; base < n4; base += 256 * SE_U) {
        f32x4 v[SE_U];
#pragma unroll
        for (int u = 0; u < SE_U; ++u) {
            const int t = base + 256 * u;
            v[u] = t < n4 ? src4(t) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < SE_U; ++u) {
            const int t = base + 256 * u;
            if (t < n4) reinterpret_cast<f32x4*>(dst)[t] = v[u];
        }
    }
}

// ms[bl * C + c] = mean over the squeeze partial sums of image b0 + bl, summed in part order; each
// thread takes four channels (C % 4 == 0), and the loads of SE_U quads x 4 parts are issued together.
__device__ __forceinline__ void se_stage_means(float* ms, const float* __restrict__ part, int b0, int nb, int C,
                                               int parts, float inv) {
    const int C4 = C >> 2, n4 = nb * C4;
    for (int base = threadIdx.x; base < n4; base += 256 * SE_U) {
        const float* src[SE_U];
        f32x4 acc[SE_U];
#pragma unroll
        for (int u = 0; u < SE_U; ++u) {
            const int t = min(base + 256 * u, n4 - 1);
            const int bl = t / C4, c4 = t - bl * C4;
            src[u] = part + (int64_t)(b0 + bl) * parts * C + 4 * c4;
            acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        for (int k0 = 0; k0 < parts; k0 += 4) {
            f32x4 v[SE_U][4];
#pragma unroll
            for (int u = 0; u < SE_U; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    v[u][q] = *reinterpret_cast<const f32x4*>(src[u] + (int64_t)min(k0 + q, parts - 1) * C);
#pragma unroll
            for (int u = 0; u < SE_U; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (k0 + q < parts) acc[u] += v[u][q];
        }
#pragma unroll
        for (int u = 0; u < SE_U; ++u) {
            const int t = base + 256 * u;
            if (t < n4) reinterpret_cast<f32x4*>(ms)[t] = acc[u] * inv;
        }
    }
}

__global__ void __launch_bounds__(256) se_fc1_kernel(const float* __restrict__ part, const float* __restrict__ w1,
                                                     const float* __restrict__ b1, float* __restrict__ hidden, int B,
                                                     int C, int S, int HW, int parts) {
    __shared__ __attribute__((aligned(16))) float ms[SE1_BB * SE_CMAX];
    __shared__ __attribute__((aligned(16))) float ws[SE1_SB * SE_CMAX];
    const int s0 = blockIdx.x * SE1_SB, b0 = blockIdx.y * SE1_BB;
    const int nb = min(SE1_BB, B - b0), ns = min(SE1_SB, S - s0);
    const float inv = 1.f / (float)HW;
    se_stage_means(ms, part, b0, nb, C, parts, inv);  // each thread rewrites only its own elements
    se_stage4(ws, ns * C / 4, [&](int t) { return *reinterpret_cast<const f32x4*>(w1 + (int64_t)s0 * C + 4 * t); });
    __syncthreads();
    // 64 outputs (bl = o & 7, sl = o >> 3), 4 threads each over C quarters
    const int o = threadIdx.x >> 2, h = threadIdx.x & 3;
    const int bl = o & 7, sl = o >> 3;
    const int ch = (C + 3) >> 2;
    const int c0 = h * ch, c1 = min(C, c0 + ch);
    float acc = 0.f;
    if (bl < nb && sl < ns) {
        const float* mr = ms + bl * C;
        const float* wr = ws + sl * C;
#pragma unroll 8
        for (int c = c0; c < c1; ++c) acc = fmaf(wr[c], mr[c], acc);  // unrolled: the loads issue together
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (h == 0 && bl < nb && sl < ns) {
        const float t = acc + b1[s0 + sl];
        hidden[(int64_t)(b0 + bl) * S + s0 + sl] = t > 0.f ? t : 0.f;
    }
}

__global__ void __launch_bounds__(256) se_fc2_kernel(const float* __restrict__ hidden, const float* __restrict__ w2t,
                                                     const float* __restrict__ b2, float* __restrict__ scale, int B,
                                                     int C, int S) {
    __shared__ __attribute__((aligned(16))) float hs[SE2_BB * SE_SMAX];
    __shared__ __attribute__((aligned(16))) float ws[SE2_SCH * 64];
    const int c0 = blockIdx.x * 64, b0 = blockIdx.y * SE2_BB;
    const int nb = min(SE2_BB, B - b0), nc = min(64, C - c0);
    se_stage4(hs, nb * S / 4, [&](int t) { return *reinterpret_cast<const f32x4*>(hidden + (int64_t)b0 * S + 4 * t); });
    const int cl = threadIdx.x & 63, bp = threadIdx.x >> 6;  // images bp and bp + 4
    float a0 = 0.f, a1 = 0.f;
    const float* h0 = hs + bp * S;
    const float* h1 = hs + (bp + 4) * S;
    for (int j0 = 0; j0 < S; j0 += SE2_SCH) {
        const int nj = min(SE2_SCH, S - j0);
        se_stage4(ws, nj * 16, [&](int t) {  // 16 quads per 64-channel row; quads past C read as zero
            const int j = t >> 4, c = 4 * (t & 15);
            return c < nc ? *reinterpret_cast<const f32x4*>(w2t + (int64_t)(j0 + j) * C + c0 + c)
                          : f32x4{0.f, 0.f, 0.f, 0.f};
        });
        __syncthreads();
#pragma unroll 8
        for (int j = 0; j < nj; ++j) {
            const float wv = ws[j * 64 + cl];
            a0 = fmaf(wv, h0[j0 + j], a0);
            a1 = fmaf(wv, h1[j0 + j], a1);
        }
        __syncthreads();
    }
    if (cl < nc) {
        const float bias = b2[c0 + cl];
        if (bp < nb) scale[(int64_t)(b0 + bp) * C + c0 + cl] = apply_act(a0 + bias, ACT_HSIGMOID);
        if (bp + 4 < nb) scale[(int64_t)(b0 + bp + 4) * C + c0 + cl] = apply_act(a1 + bias, ACT_HSIGMOID);
    }
}

// Both excitation GEMVs in one launch: one workgroup per SE_FB images does squeeze (mean of the
// partial sums) -> fc1 + ReLU -> fc2 + Hardsigmoid, so a SqueezeExcitation costs one launch (the
// latency of the small SSDLite layers, not their bytes, sets their cost).  Used for C * S <= 8192:
// larger layers read too many weight bytes per workgroup and keep the two-kernel form.
constexpr int SE_FB = 4;
__global__ void __launch_bounds__(512) se_fused_kernel(const float* __restrict__ part, const float* __restrict__ w1,
                                                      const float* __restrict__ b1, const float* __restrict__ w2t,
                                                      const float* __restrict__ b2, float* __restrict__ hidden,
                                                      float* __restrict__ scale, int B, int C, int S, int HW,
                                                      int parts) {
    __shared__ float ms[SE_FB * SE_CMAX];
    __shared__ float hs[SE_FB * SE_SMAX];
    const int b0 = blockIdx.x * SE_FB;
    const int nb = min(SE_FB, B - b0);
    const float inv = 1.f / (float)HW;
    for (int t = threadIdx.x; t < nb * C; t += 512) {  // nb * C <= 4 * 1024: at most 8 rounds
        const int bl = t / C, c = t - bl * C;
        const float* pp = part + ((int64_t)(b0 + bl) * parts) * C + c;
        float acc = 0.f;
        for (int k = 0; k < parts; ++k) acc += pp[(int64_t)k * C];
        ms[t] = acc * inv;
    }
    __syncthreads();
    // fc1: output (s, b) by a group of 4 lanes over C quarters (same order as se_fc1_kernel)
    const int ch = (C + 3) >> 2;
    for (int o = threadIdx.x >> 2; o < nb * S; o += 128) {
        const int sl = o / nb, bl = o - sl * nb;
        const int h = threadIdx.x & 3;
        const int c0 = h * ch, c1 = min(C, c0 + ch);
        const float* wr = w1 + (int64_t)sl * C;
        const float* mr = ms + bl * C;
        float acc = 0.f;
#pragma unroll 8
        for (int c = c0; c < c1; ++c) acc = fmaf(wr[c], mr[c], acc);  // unrolled: the loads issue together
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        if (h == 0) {
            const float t = acc + b1[sl];
            hs[bl * S + sl] = t > 0.f ? t : 0.f;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nb * S; t += 512) hidden[(int64_t)b0 * S + t] = hs[t];
    // fc2: channel c of every image of the group, sequential over S (same order as se_fc2_kernel)
    for (int c = threadIdx.x; c < C; c += 512) {
        float a[SE_FB];
#pragma unroll
        for (int q = 0; q < SE_FB; ++q) a[q] = 0.f;
#pragma unroll 8
        for (int j = 0; j < S; ++j) {
            const float wv = w2t[(int64_t)j * C + c];
#pragma unroll
            for (int q = 0; q < SE_FB; ++q) a[q] = fmaf(wv, hs[q * S + j], a[q]);
        }
        const float bias = b2[c];
#pragma unroll
        for (int q = 0; q < SE_FB; ++q)
            if (q < nb) scale[(int64_t)(b0 + q) * C + c] = apply_act(a[q] + bias, ACT_HSIGMOID);
    }
}

int se_fc_launch(const float* part, const float* w1, const float* b1, const float* w2t, const float* b2,
                 float* hidden, float* scale, int B, int C, int S, int HW, int parts, hipStream_t s) {
    if ((int64_t)C * S <= 8192 && parts >= 1 && parts <= SE_PARTS && S >= 1 && S <= SE_SMAX && C >= 1 && C <= SE_CMAX) {
        EDGEDET_REQUIRE(part && w1 && b1 && w2t && b2 && hidden && scale, "se_fc: null pointer");
        hipLaunchKernelGGL(se_fused_kernel, dim3((unsigned)cdiv(B, SE_FB)), dim3(512), 0, s, part, w1, b1, w2t, b2,
                           hidden, scale, B, C, S, HW, parts);
        EDGEDET_LAUNCH_CHECK();
        return 0;
    }
    EDGEDET_REQUIRE(parts >= 1 && parts <= SE_PARTS, "se_fc: 1..16 squeeze partial sums");
    EDGEDET_REQUIRE(part && w1 && b1 && w2t && b2 && hidden && scale, "se_fc: null pointer");
    EDGEDET_REQUIRE(S >= 1 && S <= SE_SMAX && C >= 1 && C <= SE_CMAX && HW >= 1, "se_fc: C <= 1024, S <= 512");
    EDGEDET_REQUIRE(C % 4 == 0 && S % 4 == 0 && ((uintptr_t)part & 15) == 0 && ((uintptr_t)w1 & 15) == 0 &&
                        ((uintptr_t)w2t & 15) == 0 && ((uintptr_t)hidden & 15) == 0,
                    "se_fc: C % 4, S % 4 and 16-byte aligned partial sums / weights / hidden (16-byte staging)");
    hipLaunchKernelGGL(se_fc1_kernel, dim3((unsigned)cdiv(S, SE1_SB), (unsigned)cdiv(B, SE1_BB)), dim3(256), 0, s,
                       part, w1, b1, hidden, B, C, S, HW, parts);
    EDGEDET_LAUNCH_CHECK();
    hipLaunchKernelGGL(se_fc2_kernel, dim3((unsigned)cdiv(C, 64), (unsigned)cdiv(B, SE2_BB)), dim3(256), 0, s,
                       hidden, w2t, b2, scale, B, C, S);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ max pool

__global__ void maxpool_kernel(PoolParams p) {
    const int C4 = p.C >> 2;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)p.B * p.Ho * p.Wo * C4;
    if (idx >= total) return;
    const int c = (int)(idx % C4) * 4;
    const int64_t pix = idx / C4;
    const int ow = (int)(pix % p.Wo);
    const int oh = (int)((pix / p.Wo) % p.Ho);
    const int b = (int)(pix / ((int64_t)p.Wo * p.Ho));
    const float* xb = p.x + (int64_t)b * p.H * p.W * p.C + c;
    const float ninf = -__builtin_inff();
    f32x4 m = {ninf, ninf, ninf, ninf};
    for (int kh = 0; kh < p.K; ++kh) {
        const int ih = oh * p.stride - p.pad + kh;
        if ((unsigned)ih >= (unsigned)p.H) continue;
        for (int kw = 0; kw < p.K; ++kw) {
            const int iw = ow * p.stride - p.pad + kw;
            if ((unsigned)iw >= (unsigned)p.W) continue;
            const f32x4 v = *reinterpret_cast<const f32x4*>(xb + ((int64_t)ih * p.W + iw) * p.C);
            // ATen max_pool2d: NaN propagates, otherwise max
            m.x = (v.x > m.x || isnan(v.x)) ? v.x : m.x;
            m.y = (v.y > m.y || isnan(v.y)) ? v.y : m.y;
            m.z = (v.z > m.z || isnan(v.z)) ? v.z : m.z;
            m.w = (v.w > m.w || isnan(v.w)) ? v.w : m.w;
        }
    }
    *reinterpret_cast<f32x4*>(p.y + pix * p.C + c) = m;
}

int maxpool_launch(const PoolParams& p, hipStream_t s) {
    EDGEDET_REQUIRE(p.x && p.y, "maxpool: null x/y");
    EDGEDET_REQUIRE(p.C % 4 == 0, "maxpool: C must be a multiple of 4");
    const int64_t total = (int64_t)p.B * p.Ho * p.Wo * (p.C / 4);
    hipLaunchKernelGGL(maxpool_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ RoIAlign
// torchvision roi_align (aligned=False) bilinear_interpolate, restated for NHWC features.
__host__ __device__ inline void bilinear_setup(float y, float x, int H, int W, int& o1, int& o2, int& o3, int& o4,
                                               float& w1, float& w2, float& w3, float& w4) {
    if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) {
        o1 = o2 = o3 = o4 = 0;
        w1 = w2 = w3 = w4 = 0.f;
        return;
    }
    if (y <= 0.f) y = 0.f;
    if (x <= 0.f) x = 0.f;
    int y_low = (int)y, x_low = (int)x, y_high, x_high;
    if (y_low >= H - 1) {
        y_high = y_low = H - 1;
        y = (float)y_low;
    } else {
        y_high = y_low + 1;
    }
    if (x_low >= W - 1) {
        x_high = x_low = W - 1;
        x = (float)x_low;
    } else {
        x_high = x_low + 1;
    }
    const float ly = y - (float)y_low, lx = x - (float)x_low;
    const float hy = 1.f - ly, hx = 1.f - lx;
    o1 = y_low * W + x_low;
    o2 = y_low * W + x_high;
    o3 = y_high * W + x_low;
    o4 = y_high * W + x_high;
    w1 = hy * hx;
    w2 = hy * lx;
    w3 = ly * hx;
    w4 = ly * lx;
}


// One output element group (4 channels of one bin of one RoI).  __host__ __device__ so the exact
// kernel body also runs in the host-side debug harness (tools/roi_align_host_check.cpp, ASan).
__host__ __device__ inline void roi_align_thread(const RoiParams& p, int r, int j) {
    // j = (ph * PW + pw) * C4 + c/4 within RoI r: 32-bit index math (int64 division is a long
    // software sequence on the GPU and used to dominate the kernel)
    const int C4 = p.C >> 2;
    const int bin = j / C4;
    const int c = (j - bin * C4) * 4;
    const int ph = bin / p.PW;
    const int pw = bin - ph * p.PW;
    const int64_t idx = (int64_t)r * (p.PH * p.PW * C4) + j;
    float* o = p.out + idx * 4;
    int b, lvl = 0;
    float x1, y1, x2, y2;
    if (p.mode == 0) {
        const float* rr = p.rois + (int64_t)r * 5;
        b = (int)rr[0];
        x1 = rr[1];
        y1 = rr[2];
        x2 = rr[3];
        y2 = rr[4];
    } else {
        b = r / p.RMAX;
        const int slot = r - b * p.RMAX;
        if (slot >= p.counts[b]) {
            *reinterpret_cast<f32x4*>(o) = f32x4{0.f, 0.f, 0.f, 0.f};
            return;
        }
        const float* bb = p.rois + (int64_t)r * 4;
        x1 = bb[0];
        y1 = bb[1];
        x2 = bb[2];
        y2 = bb[3];
        // LevelMapper (canonical scale 224, level 4, eps 1e-6)
        const float area = (x2 - x1) * (y2 - y1);
        const float s = sqrtf(area);
        float tl = floorf((4.0f + log2f(s / 224.0f)) + 1e-6f);
        tl = fminf(fmaxf(tl, (float)p.k_min), (float)p.k_max);
        lvl = (int)tl - p.k_min;
    }
    const float* f = p.feat[lvl];
    const int H = p.H[lvl], W = p.W[lvl];
    const float scale = p.scale[lvl];
    const float rsw = x1 * scale, rsh = y1 * scale;
    const float rew = x2 * scale, reh = y2 * scale;
    float rw = rew - rsw, rh = reh - rsh;
    rw = rw > 1.f ? rw : 1.f;
    rh = rh > 1.f ? rh : 1.f;
    const float bin_h = rh / (float)p.PH, bin_w = rw / (float)p.PW;
    const int gh = p.sr > 0 ? p.sr : (int)ceilf(rh / (float)p.PH);
    const int gw = p.sr > 0 ? p.sr : (int)ceilf(rw / (float)p.PW);
    const int cnt = gh * gw;
    const float count = (float)(cnt > 1 ? cnt : 1);
    const float* fb = f + (int64_t)b * H * W * p.C + c;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int iy = 0; iy < gh; ++iy) {
        const float yy = (rsh + (float)ph * bin_h) + ((float)iy + .5f) * bin_h / (float)gh;
        for (int ix = 0; ix < gw; ++ix) {
            const float xx = (rsw + (float)pw * bin_w) + ((float)ix + .5f) * bin_w / (float)gw;
            int o1, o2, o3, o4;
            float w1, w2, w3, w4;
            bilinear_setup(yy, xx, H, W, o1, o2, o3, o4, w1, w2, w3, w4);
            const f32x4 v1 = *reinterpret_cast<const f32x4*>(fb + (int64_t)o1 * p.C);
            const f32x4 v2 = *reinterpret_cast<const f32x4*>(fb + (int64_t)o2 * p.C);
            const f32x4 v3 = *reinterpret_cast<const f32x4*>(fb + (int64_t)o3 * p.C);
            const f32x4 v4 = *reinterpret_cast<const f32x4*>(fb + (int64_t)o4 * p.C);
            acc.x += ((w1 * v1.x + w2 * v2.x) + w3 * v3.x) + w4 * v4.x;
            acc.y += ((w1 * v1.y + w2 * v2.y) + w3 * v3.y) + w4 * v4.y;
            acc.z += ((w1 * v1.z + w2 * v2.z) + w3 * v3.z) + w4 * v4.z;
            acc.w += ((w1 * v1.w + w2 * v2.w) + w3 * v3.w) + w4 * v4.w;
        }
    }
    *reinterpret_cast<f32x4*>(o) = f32x4{acc.x / count, acc.y / count, acc.z / count, acc.w / count};
}

// grid (R, bins x channel groups of one RoI / 256): the RoI, its level and sampling grid are
// uniform across the workgroup
__global__ void __launch_bounds__(256) roi_align_kernel(RoiParams p) {
    const int j = blockIdx.y * 256 + threadIdx.x;
    if (j >= p.PH * p.PW * (p.C >> 2)) return;
    roi_align_thread(p, blockIdx.x, j);
}

int roi_align_launch(const RoiParams& p, hipStream_t s) {
    EDGEDET_REQUIRE(p.C % 4 == 0, "roi_align: C must be a multiple of 4");
    EDGEDET_REQUIRE(p.out != nullptr && p.rois != nullptr && p.feat[0] != nullptr, "roi_align: null pointer");
    EDGEDET_REQUIRE(p.mode == 0 || (p.counts != nullptr && p.RMAX > 0), "roi_align: mode 1 needs counts/RMAX");
    EDGEDET_REQUIRE(p.nlevels >= 1 && p.nlevels <= 4, "roi_align: 1..4 levels");
    const int64_t total = (int64_t)p.R * p.PH * p.PW * (p.C / 4);
    if (total == 0) return 0;
    EDGEDET_REQUIRE((int64_t)p.PH * p.PW * (p.C / 4) <= 65535 * 256, "roi_align: too many bins x channels");
    hipLaunchKernelGGL(roi_align_kernel, dim3((unsigned)p.R, (unsigned)cdiv(p.PH * p.PW * (p.C / 4), 256)), dim3(256),
                       0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ================================================================ GroupNorm statistics
// RetinaNetHead's GroupNorm(32, 256) (retinanet_resnet50_fpn_v2, detect.py:34-38): per (image,
// group) mean / biased variance over HW x C/G values, in float64 (deterministic fixed-order
// reduction), then ATen's forward form GN(x) = x * scale + shift with scale = rstd * gamma and
// shift = -scale * mean + beta (float).  The consumer conv applies it (+ ReLU) as it loads its A
// operand (conv.hip in_transform), so the normalized tensor never reaches HBM.
__global__ void __launch_bounds__(256) gn_stats_kernel(GnParams p) {
    const int g = blockIdx.x, b = blockIdx.y;
    const int cpg = p.C / p.G;
    const float* xb = p.x + (int64_t)b * p.HW * p.C + g * cpg;
    double s1 = 0.0, s2 = 0.0;
    for (int px = threadIdx.x; px < p.HW; px += 256) {
        const float* r = xb + (int64_t)px * p.C;
        for (int c = 0; c < cpg; c += 4) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(r + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                s1 += (double)v[e];
                s2 += (double)v[e] * (double)v[e];
            }
        }
    }
    __shared__ double red[2][4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_down(s1, o, 64);
        s2 += __shfl_down(s2, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = s1;
        red[1][w] = s2;
    }
    __syncthreads();
    if (threadIdx.x < cpg) {
        const double n = (double)p.HW * cpg;
        const double S1 = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        const double S2 = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
        const double mean = S1 / n;
        double var = S2 / n - mean * mean;
        var = var > 0.0 ? var : 0.0;
        const float meanf = (float)mean;
        const float rstd = 1.f / sqrtf((float)var + p.eps);
        const int c = g * cpg + threadIdx.x;
        const float sc = rstd * p.gamma[c];
        p.scale[(int64_t)b * p.C + c] = sc;
        p.shift[(int64_t)b * p.C + c] = -sc * meanf + p.beta[c];
    }
}

int gn_stats_launch(const GnParams& p, hipStream_t s) {
    EDGEDET_REQUIRE(p.x && p.gamma && p.beta && p.scale && p.shift, "group_norm: null pointer");
    EDGEDET_REQUIRE(p.G > 0 && p.C % p.G == 0 && (p.C / p.G) % 4 == 0 && p.C / p.G <= 256,
                    "group_norm: channels per group must be a multiple of 4 (<= 256)");
    EDGEDET_REQUIRE(p.B > 0 && p.HW > 0 && ((uintptr_t)p.x & 15) == 0, "group_norm: bad sizes/alignment");
    hipLaunchKernelGGL(gn_stats_kernel, dim3(p.G, p.B), dim3(256), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

}  // namespace edgedet

using namespace edgedet;

extern "C" int edgedet_roi_align(const float* feat, int64_t B, int64_t H, int64_t W, int64_t C, const float* rois,
                                 int64_t R, float spatial_scale, int32_t pooled_h, int32_t pooled_w,
                                 int32_t sampling_ratio, float* out, void* stream) {
    RoiParams p{};
    p.feat[0] = feat;
    p.H[0] = (int)H;
    p.W[0] = (int)W;
    p.scale[0] = spatial_scale;
    p.nlevels = 1;
    p.rois = rois;
    p.mode = 0;
    p.R = (int)R;
    p.B = (int)B;
    p.C = (int)C;
    p.PH = pooled_h;
    p.PW = pooled_w;
    p.sr = sampling_ratio;
    p.out = out;
    return roi_align_launch(p, (hipStream_t)stream);
}

extern "C" int edgedet_dwconv2d(const float* x, int64_t B, int64_t H, int64_t W, int64_t C, const float* w,
                                const float* bias, int32_t K, int32_t stride, int32_t pad, int32_t act, float* y,
                                void* stream) {
    DwParams p{};
    p.x = x;
    p.w = w;
    p.bias = bias;
    p.y = y;
    p.B = (int)B;
    p.H = (int)H;
    p.W = (int)W;
    p.C = (int)C;
    p.K = K;
    p.stride = stride;
    p.pad = pad;
    p.act = act;
    p.Ho = (int)((H + 2 * pad - K) / stride + 1);
    p.Wo = (int)((W + 2 * pad - K) / stride + 1);
    return dwconv_launch(p, (hipStream_t)stream);
}
