// Memory-bound layers of the two detectors (NHWC fp32, one thread per pixel x 4 channels).
//
//   preprocess   GeneralizedRCNNTransform eval: (x - mean) / std, bilinear resize
//                (align_corners=False), zero pad to the batch size        SURVEY.md App. A.0, row a6
//   dwconv       depthwise conv + folded BN + act (MobileNetV3 / SSDLite)  App. A.1, rows a7/a8
//   channel_mean adaptive_avg_pool2d(1) of SqueezeExcitation               App. A.1 step 2
//   se_fc        SE fc1 -> ReLU -> fc2 -> Hardsigmoid (per image)          App. A.1 step 2
//   maxpool      ResNet stem max_pool2d(3,2,1); FPN LastLevelMaxPool(1,2,0) App. A.2 steps 2-3
//   roi_align    MultiScaleRoIAlign: LevelMapper + roi_align(7x7, sr=2, aligned=False)
//                                                                          App. A.2 step 5, row a13
#include "kernels.hpp"

namespace edgedet {


// ------------------------------------------------------------------------------ preprocess

__global__ void preprocess_kernel(PreParams p) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)p.B * p.Hp * p.Wp;
    if (idx >= total) return;
    const int ox = (int)(idx % p.Wp);
    const int oy = (int)((idx / p.Wp) % p.Hp);
    const int b = (int)(idx / ((int64_t)p.Wp * p.Hp));
    f32x4 out = {0.f, 0.f, 0.f, 0.f};
    if (oy < p.Ho && ox < p.Wo) {
        // ATen area_pixel_compute_source_index (align_corners=False, linear)
        float ry = p.sh * ((float)oy + 0.5f) - 0.5f;
        float rx = p.sw * ((float)ox + 0.5f) - 0.5f;
        ry = ry < 0.f ? 0.f : ry;
        rx = rx < 0.f ? 0.f : rx;
        const int y0 = (int)ry, x0 = (int)rx;
        const int y1 = y0 + ((y0 < p.H - 1) ? 1 : 0);
        const int x1 = x0 + ((x0 < p.W - 1) ? 1 : 0);
        const float ly = ry - (float)y0, lx = rx - (float)x0;
        const float hy = 1.f - ly, hx = 1.f - lx;
        float v[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float* src = p.x + ((int64_t)b * 3 + c) * p.H * p.W;
            const float a00 = (src[(int64_t)y0 * p.W + x0] - p.mean[c]) / p.stdv[c];
            const float a01 = (src[(int64_t)y0 * p.W + x1] - p.mean[c]) / p.stdv[c];
            const float a10 = (src[(int64_t)y1 * p.W + x0] - p.mean[c]) / p.stdv[c];
            const float a11 = (src[(int64_t)y1 * p.W + x1] - p.mean[c]) / p.stdv[c];
            v[c] = (a00 * hx + a01 * lx) * hy + (a10 * hx + a11 * lx) * ly;
        }
        out = f32x4{v[0], v[1], v[2], 0.f};
    }
    *reinterpret_cast<f32x4*>(p.y + idx * 4) = out;
}

int preprocess_launch(const PreParams& p0, hipStream_t s) {
    PreParams p = p0;
    EDGEDET_REQUIRE(p.x && p.y, "preprocess: null x/y");
    EDGEDET_REQUIRE(p.Hp >= p.Ho && p.Wp >= p.Wo && p.Ho > 0 && p.Wo > 0, "preprocess: bad sizes");
    p.sh = (float)p.H / (float)p.Ho;
    p.sw = (float)p.W / (float)p.Wo;
    const int64_t total = (int64_t)p.B * p.Hp * p.Wp;
    hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p);
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

int dwconv_launch(const DwParams& p, hipStream_t s) {
    EDGEDET_REQUIRE(p.x && p.w && p.bias && p.y, "dwconv: null x/w/bias/y");
    EDGEDET_REQUIRE(p.C % 4 == 0, "dwconv: C must be a multiple of 4");
    const int64_t total = (int64_t)p.B * p.Ho * p.Wo * (p.C / 4);
    hipLaunchKernelGGL(dwconv_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ SE squeeze
// Partial channel sums: grid (cdiv(C, 64), B, S) with block 256 = 64 channels x 4 pixel groups; split s
// covers pixels [s*HW/S, (s+1)*HW/S).  part[b][s][c] is reduced in fixed order by se_fc_kernel
// (deterministic, no atomics).

__global__ void channel_sum_kernel(const float* __restrict__ x, float* __restrict__ part, int HW, int C, int S) {
    __shared__ float red[4][64];
    const int b = blockIdx.y, sidx = blockIdx.z;
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int p0 = (int)((int64_t)sidx * HW / S), p1 = (int)((int64_t)(sidx + 1) * HW / S);
    float acc = 0.f;
    if (c < C) {
        const float* xb = x + (int64_t)b * HW * C + c;
        for (int i = p0 + g; i < p1; i += 4) acc += xb[(int64_t)i * C];
    }
    red[g][cl] = acc;
    __syncthreads();
    if (g == 0 && c < C)
        part[((int64_t)b * S + sidx) * C + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

int channel_mean_launch(const float* x, float* out, int B, int HW, int C, hipStream_t s) {
    EDGEDET_REQUIRE(x && out, "channel_mean: null pointer");
    hipLaunchKernelGGL(channel_sum_kernel, dim3((unsigned)cdiv(C, 64), B, SE_PARTS), dim3(256), 0, s, x, out, HW, C,
                       SE_PARTS);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------ SE excitation
// grid (cdiv(C, 64), B): every block recomputes the (small) fc1 of its image from the partial sums
// part [B][SE_PARTS][C] (mean = sum / HW, fixed reduction order), then evaluates fc2 + Hardsigmoid
// for its 64 channels.  w1 [S][C] (fc1 as stored), w2t [S][C] (fc2 transposed).  fc1 splits the C
// reduction over the 64 lanes of a wave; fc2 splits the S reduction over 4 waves.
__global__ void __launch_bounds__(256) se_fc_kernel(const float* __restrict__ part, const float* __restrict__ w1,
                                                    const float* __restrict__ b1, const float* __restrict__ w2t,
                                                    const float* __restrict__ b2, float* __restrict__ scale, int C,
                                                    int S, int HW) {
    extern __shared__ float sm[];
    float* m = sm;             // [C]
    float* s1 = sm + C;        // [S]
    float* red = s1 + S;       // [256]
    const int b = blockIdx.y;
    const int tid = threadIdx.x;
    for (int c = tid; c < C; c += 256) {
        float acc = 0.f;
        for (int k = 0; k < SE_PARTS; ++k) acc += part[((int64_t)b * SE_PARTS + k) * C + c];
        m[c] = acc / (float)HW;
    }
    __syncthreads();
    // fc1: wave w owns outputs j = w, w+4, ...; its 64 lanes split the C reduction (fixed order:
    // lane-strided partial sums, then a butterfly)
    const int lane = tid & 63, wv = tid >> 6;
    for (int j = wv; j < S; j += 4) {
        float a = 0.f;
        for (int c = lane; c < C; c += 64) a = fmaf(w1[(int64_t)j * C + c], m[c], a);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
        if (lane == 0) {
            a += b1[j];
            s1[j] = a > 0.f ? a : 0.f;
        }
    }
    __syncthreads();
    const int cl = tid & 63, g = tid >> 6;
    const int c = blockIdx.x * 64 + cl;
    float a = 0.f;
    if (c < C)
        for (int j = g; j < S; j += 4) a = fmaf(w2t[(int64_t)j * C + c], s1[j], a);
    red[tid] = a;
    __syncthreads();
    if (g == 0 && c < C) {
        const float v = ((red[cl] + red[64 + cl]) + red[128 + cl]) + red[192 + cl];
        scale[(int64_t)b * C + c] = apply_act(v + b2[c], ACT_HSIGMOID);
    }
}

int se_fc_launch(const float* mean, const float* w1, const float* b1, const float* w2t, const float* b2,
                 float* scale, int B, int C, int S, int HW, hipStream_t s) {
    EDGEDET_REQUIRE(mean && w1 && b1 && w2t && b2 && scale, "se_fc: null pointer");
    EDGEDET_REQUIRE(S >= 1 && S <= 256, "se_fc: squeeze width must be in [1, 256]");
    const size_t lds = (size_t)(C + S + 256) * sizeof(float);
    EDGEDET_REQUIRE(lds <= 60 * 1024, "se_fc: too many channels");
    hipLaunchKernelGGL(se_fc_kernel, dim3((unsigned)cdiv(C, 64), B), dim3(256), lds, s, mean, w1, b1, w2t, b2, scale,
                       C, S, HW);
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
__host__ __device__ inline void roi_align_thread(const RoiParams& p, int64_t idx) {
    const int C4 = p.C >> 2;
    const int c = (int)(idx % C4) * 4;
    int64_t t = idx / C4;
    const int pw = (int)(t % p.PW);
    t /= p.PW;
    const int ph = (int)(t % p.PH);
    const int r = (int)(t / p.PH);
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

__global__ void roi_align_kernel(RoiParams p) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)p.R * p.PH * p.PW * (p.C >> 2);
    if (idx >= total) return;
    roi_align_thread(p, idx);
}

int roi_align_launch(const RoiParams& p, hipStream_t s) {
    EDGEDET_REQUIRE(p.C % 4 == 0, "roi_align: C must be a multiple of 4");
    EDGEDET_REQUIRE(p.out != nullptr && p.rois != nullptr && p.feat[0] != nullptr, "roi_align: null pointer");
    EDGEDET_REQUIRE(p.mode == 0 || (p.counts != nullptr && p.RMAX > 0), "roi_align: mode 1 needs counts/RMAX");
    EDGEDET_REQUIRE(p.nlevels >= 1 && p.nlevels <= 4, "roi_align: 1..4 levels");
    const int64_t total = (int64_t)p.R * p.PH * p.PW * (p.C / 4);
    if (total == 0) return 0;
    hipLaunchKernelGGL(roi_align_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, p);
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
