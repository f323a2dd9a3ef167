// Implicit-GEMM convolution on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the ATen conv2d + eval BatchNorm2d (+ activation) layers of the torchvision backbones
// and heads reached from torch_models/detect.py:78.
//
// GEMM view: C[M=B*Ho*Wo][N=Cout] = A[M][K=KH*KW*Cin] * W[N][K]^T, NHWC activations, weights
// packed K-contiguous ([Cout][KH][KW][Cin], K zero-padded to a multiple of 32).  BN is folded
// into W/bias on the host.  The epilogue fuses bias, an optional residual (ResNet identity, FPN
// top-down nearest-upsample add), the activation and a strided store (so SSD head outputs land
// directly in the concatenated [B, anchors, classes] layout).  SqueezeExcitation's channel scale
// is fused into the A-operand load of the projection conv.
//
// Tile: block = WM x WN waves, each wave TM x TN 32x32 MFMA tiles; BK = 32 per LDS stage,
// double-buffered through registers (one barrier per K stage).  In an MFMA step lane-half h of a
// wave contributes k = 16h + 8q + t (q, t loop indices), so both operands are read from LDS as
// contiguous f32x4s (ds_read_b128) from K-contiguous rows padded to 36 floats (conflict-free
// for the b128 lane groups).
#include <algorithm>
#include <cstdlib>

#include "kernels.hpp"

namespace edgedet {

typedef float floatx16 __attribute__((ext_vector_type(16)));


constexpr int BK = 32;
constexpr int LDK = BK + 4;  // padded LDS row (floats)

// Output offset of GEMM row m (an output pixel), for y (is_res = false) or the residual.
__device__ __forceinline__ int64_t conv_row_offset(const ConvParams& p, int m, bool is_res) {
    if (!is_res && p.lin_y) return p.y_off + (int64_t)m * p.y_pstride;
    if (is_res && p.lin_res) return (int64_t)m * p.res_pstride;
    const int b = (int)fdiv((uint32_t)m, p.div_howo);
    const int pix = m - b * p.Ho * p.Wo;
    if (!is_res) return p.y_off + (int64_t)b * p.y_bstride + (int64_t)pix * p.y_pstride;
    int rpix = pix;
    if (p.res_H != p.Ho || p.res_W != p.Wo) {  // FPN top-down: nearest upsample of the residual
        const int oh = (int)fdiv((uint32_t)pix, p.div_wo);
        const int ow = pix - oh * p.Wo;
        int ry = (int)floorf((float)oh * p.res_sh);
        int rx = (int)floorf((float)ow * p.res_sw);
        ry = ry < p.res_H - 1 ? ry : p.res_H - 1;
        rx = rx < p.res_W - 1 ? rx : p.res_W - 1;
        rpix = ry * p.res_W + rx;
    }
    return (int64_t)b * p.res_bstride + (int64_t)rpix * p.res_pstride;
}

// Input transform applied to in-bounds A-operand values (zero padding stays zero, as the reference
// pads the transformed tensor): SqueezeExcitation's channel scale, GroupNorm's x * scale + shift
// (ATen's GroupNorm forward form), and an optional ReLU.
__device__ __forceinline__ f32x4 in_transform(const ConvParams& p, f32x4 v, int b, int ci) {
    if (p.in_scale) v *= *reinterpret_cast<const f32x4*>(p.in_scale + (int64_t)b * p.Cin + ci);
    if (p.in_shift) v += *reinterpret_cast<const f32x4*>(p.in_shift + (int64_t)b * p.Cin + ci);
    if (p.in_relu) {
        v.x = v.x > 0.f ? v.x : 0.f;
        v.y = v.y > 0.f ? v.y : 0.f;
        v.z = v.z > 0.f ? v.z : 0.f;
        v.w = v.w > 0.f ? v.w : 0.f;
    }
    return v;
}

template <int TM, int TN, int ACT>
__device__ __forceinline__ void act_tile(floatx16 (&acc)[TM][TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = apply_act(acc[i][j][r], ACT);
}

// Epilogue shared by both conv kernels.  Row of (i, r) = row0 + 32i + (r&3) + 8(r>>2) + 4h (the
// 32x32 MFMA C layout), column of j = col0 + 32j + (lane & 31).  L16: the 32 x 32 block (i, j) holds
// four 16x16 MFMA C tiles, register r in tile q = r >> 2 (row half q >> 1, column half q & 1): row
// row0 + 32i + 16((r>>3)&1) + 4(lane>>4) + (r&3), column col0 + 32j + 16((r>>2)&1) + (lane&15).
// Pass 1 adds bias and residual, pass 2 applies the activation (one uniform switch outside the
// element loops), pass 3 stores.
template <int TM, int TN, bool L16 = false>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, floatx16 (&acc)[TM][TN], int row0, int col0,
                                              int h, int l32) {
    const int lane = l32 + 32 * h;
    auto row_of = [&](int i, int r) {
        return L16 ? row0 + i * 32 + 16 * ((r >> 3) & 1) + 4 * (lane >> 4) + (r & 3)
                   : row0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    };
    constexpr int NS = L16 ? 2 : 1;  // column halves of a 32-wide block
    auto half_of = [](int r) { return L16 ? (r >> 2) & 1 : 0; };
    // Loads use clamped (always valid) rows/columns so no load sits behind a branch; only the
    // stores are predicated.
    float bj[TN][NS];
    int nc[TN][NS], col[TN][NS];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            col[j][s] = col0 + j * 32 + (L16 ? 16 * s + (lane & 15) : l32);
            nc[j][s] = col[j][s] < p.Cout ? col[j][s] : p.Cout - 1;
            bj[j][s] = p.bias[nc[j][s]];
        }
    if (p.res) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = row_of(i, r);
                const float* rrow = p.res + conv_row_offset(p, m < p.M ? m : p.M - 1, true);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j][r] = (acc[i][j][r] + bj[j][half_of(r)]) + rrow[nc[j][half_of(r)]];
            }
    } else if (p.ksplit > 1) {
        // two K halves meet in y (zeroed by the plan): the first adds the bias; a + b == b + a in
        // IEEE arithmetic, so the result does not depend on which half lands first
        const bool first = (blockIdx.x & 1) == 0;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = row_of(i, r);
                float* yrow = p.y + conv_row_offset(p, m < p.M ? m : p.M - 1, false);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    if (m < p.M && col[j][half_of(r)] < p.Cout)
                        atomicAdd(yrow + nc[j][half_of(r)], first ? acc[i][j][r] + bj[j][half_of(r)] : acc[i][j][r]);
            }
        return;
    } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] += bj[j][half_of(r)];
    }
    switch (p.act) {
        case ACT_RELU: act_tile<TM, TN, ACT_RELU>(acc); break;
        case ACT_RELU6: act_tile<TM, TN, ACT_RELU6>(acc); break;
        case ACT_HSWISH: act_tile<TM, TN, ACT_HSWISH>(acc); break;
        case ACT_HSIGMOID: act_tile<TM, TN, ACT_HSIGMOID>(acc); break;
        case ACT_SIGMOID: act_tile<TM, TN, ACT_SIGMOID>(acc); break;
        default: break;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = row_of(i, r);
            float* yrow = p.y + conv_row_offset(p, m < p.M ? m : p.M - 1, false);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                if (m < p.M && col[j][half_of(r)] < p.Cout) yrow[nc[j][half_of(r)]] = acc[i][j][r];
        }
}


template <int WM, int WN, int TM, int TN>
__global__ void __launch_bounds__(WM* WN * 64) conv_mfma_kernel(ConvParams p) {
    constexpr int NT = WM * WN * 64;
    constexpr int BM = WM * TM * 32;
    constexpr int BN = WN * TN * 32;
    constexpr int AJ = BM * 8 / NT;  // f32x4 A loads per thread per stage
    constexpr int BJ = BN * 8 / NT;
    static_assert(AJ >= 1 && BJ >= 1, "tile too small for block");

    __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * LDK];
    float* As = lds;
    float* Bs = lds + 2 * BM * LDK;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wave_m = wid / WN;
    const int wave_n = wid % WN;

    // XCD-aware, bijective block remap: blocks that share an XCD (bid % 8) get consecutive tiles,
    // which share their A (activation) panel.
    const int nmt = (p.M + BM - 1) / BM;
    const int nnt = (p.Cout + BN - 1) / BN;
    const int nwg = nmt * nnt;
    int bid = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int mt = bid / nnt;
    const int nt = bid % nnt;
    const int m0 = mt * BM;
    const int n0 = nt * BN;

    // ---- per-thread A rows (fixed across K stages)
    const int c4 = tid & 7;  // f32x4 column within the 32-wide stage
    int64_t a_base[AJ];
    int a_ih0[AJ], a_iw0[AJ], a_b[AJ];
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
        const int row = (tid >> 3) + (NT / 8) * j;
        const int m = m0 + row;
        if (m < p.M && p.lin_x) {
            // 1x1 / stride 1 / pad 0 over a dense NHWC tensor: pixel m sits at m * pstride
            a_b[j] = (p.in_scale || p.in_shift) ? (int)fdiv((uint32_t)m, p.div_howo) : 0;
            a_base[j] = (int64_t)m * p.x_pstride;
            a_ih0[j] = 0;
            a_iw0[j] = 0;
        } else if (m < p.M) {
            const int b = (int)fdiv((uint32_t)m, p.div_howo);
            const int rem = m - b * p.Ho * p.Wo;
            const int oh = (int)fdiv((uint32_t)rem, p.div_wo);
            const int ow = rem - oh * p.Wo;
            a_b[j] = b;
            a_base[j] = (int64_t)b * p.x_bstride;
            a_ih0[j] = oh * p.stride - p.pad;
            a_iw0[j] = ow * p.stride - p.pad;
        } else {
            a_b[j] = 0;
            a_base[j] = 0;
            a_ih0[j] = -(1 << 28);  // forces out-of-bounds -> zero
            a_iw0[j] = 0;
        }
    }
    const int KHW = p.KH * p.KW;

    f32x4 ra[AJ], rb[BJ];

    auto load_stage = [&](int k0) {
        const int k = k0 + c4 * 4;
        const int tap = (int)fdiv((uint32_t)k, p.div_cin);
        const int ci = k - tap * p.Cin;
        const int kh = (int)fdiv((uint32_t)tap, p.div_kw);
        const int kw = tap - kh * p.KW;
        const bool kval = tap < KHW;
#pragma unroll
        for (int j = 0; j < AJ; ++j) {
            const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
            f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (kval && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) {
                v = *reinterpret_cast<const f32x4*>(p.x + a_base[j] + (int64_t)(ih * p.W + iw) * p.x_pstride + ci);
                v = in_transform(p, v, a_b[j], ci);
            }
            ra[j] = v;
        }
#pragma unroll
        for (int j = 0; j < BJ; ++j) {
            const int row = (tid >> 3) + (NT / 8) * j;
            const int n = n0 + row;
            f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (n < p.Cout) v = *reinterpret_cast<const f32x4*>(p.w + (int64_t)n * p.Kpad + k0 + c4 * 4);
            rb[j] = v;
        }
    };
    auto store_stage = [&](int buf) {
        float* A = As + buf * BM * LDK;
        float* Bb = Bs + buf * BN * LDK;
#pragma unroll
        for (int j = 0; j < AJ; ++j) {
            const int row = (tid >> 3) + (NT / 8) * j;
            *reinterpret_cast<f32x4*>(A + row * LDK + c4 * 4) = ra[j];
        }
#pragma unroll
        for (int j = 0; j < BJ; ++j) {
            const int row = (tid >> 3) + (NT / 8) * j;
            *reinterpret_cast<f32x4*>(Bb + row * LDK + c4 * 4) = rb[j];
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = p.Kpad / BK;
    load_stage(0);
    store_stage(0);
    __syncthreads();

    const int h = lane >> 5;
    const int l32 = lane & 31;
    for (int kc = 0; kc < nk; ++kc) {
        const int buf = kc & 1;
        if (kc + 1 < nk) load_stage((kc + 1) * BK);
        const float* A = As + buf * BM * LDK;
        const float* Bb = Bs + buf * BN * LDK;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            f32x4 af[TM][2], bf[TN][2];
            const int kofs = 16 * h + 8 * q;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float* src = A + (wave_m * TM * 32 + i * 32 + l32) * LDK + kofs;
                af[i][0] = *reinterpret_cast<const f32x4*>(src);
                af[i][1] = *reinterpret_cast<const f32x4*>(src + 4);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const float* src = Bb + (wave_n * TN * 32 + j * 32 + l32) * LDK + kofs;
                bf[j][0] = *reinterpret_cast<const f32x4*>(src);
                bf[j][1] = *reinterpret_cast<const f32x4*>(src + 4);
            }
            // each tile's 16 K of this half stage into a stage sum from zero, then one add into the
            // running output (the running sum is rounded once per 16 K instead of at every product)
            // (the 2 x 2-tile forms, 128 x 128 and 256 x 128, run only under fp32 conv math and have no
            // registers for four stage sums: they keep the plain fmaf chain, the accuracy reference of
            // tools/accuracy_probe.py)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    floatx16 s{};
                    if constexpr (TM * TN == 4) s = acc[i][j];
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const float a = (t < 4) ? af[i][0][t & 3] : af[i][1][t & 3];
                        const float b = (t < 4) ? bf[j][0][t & 3] : bf[j][1][t & 3];
                        s = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, s, 0, 0, 0);
                    }
                    acc[i][j] = TM * TN == 4 ? s : acc[i][j] + s;
                }
        }
        if (kc + 1 < nk) store_stage(buf ^ 1);
        __syncthreads();
    }

    conv_epilogue<TM, TN>(p, acc, m0 + wave_m * TM * 32, n0 + wave_n * TN * 32, h, l32);
}

// ---------------------------------------------------------------------------------------------
// Pointwise (1x1, stride 1, dense NHWC) conv with operands loaded straight from global memory into
// MFMA fragments: no LDS, no barriers.  A wave owns a (32*TM) x (32*TN) output tile; lane l supplies
// row/column (l & 31) and k = 16*(l >> 5) + t of each 32-deep K chunk (t = MFMA step), which for a
// K-contiguous row is one 64-byte run per lane.  The next chunk's fragments are loaded into a
// second register set before the current chunk's MFMAs issue (one chunk of prefetch), so the
// memory latency of chunk k+1 overlaps the 16*TM*TN MFMAs of chunk k.
//
// pw_splitk_kernel: the same fragments, but the four waves of a workgroup share one 32 x (32*TN)
// output tile and take every fourth K chunk; their partial tiles are summed through LDS in fixed
// wave order before the epilogue.  For narrow outputs over long K (SSDLite regression heads and
// late projections: N <= 96, K >= 256) this gives 4x more waves per tile and 4x shorter chains.
template <int TM, int TN>
struct PwFrag {
    f32x4 a[TM][4], b[TN][4];
};

template <int TM, int TN>
__device__ __forceinline__ void pw_load(const ConvParams& p, PwFrag<TM, TN>& f, const float* const (&arow)[TM],
                                        const int (&ab)[TM], const bool (&aval)[TM], const float* const (&brow)[TN],
                                        const bool (&bval)[TN], int kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = kk + 4 * q;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (aval[i] && k < p.K) {
                v = *reinterpret_cast<const f32x4*>(arow[i] + k);
                v = in_transform(p, v, ab[i], k);
            }
            f.a[i][q] = v;
        }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            f.b[j][q] = bval[j] ? *reinterpret_cast<const f32x4*>(brow[j] + kk + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
}

// One 32-deep K chunk: each tile's chunk sum from zero, then one add into the running output.
template <int TM, int TN>
__device__ __forceinline__ void pw_mma(const PwFrag<TM, TN>& f, floatx16 (&acc)[TM][TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            floatx16 s{};
#pragma unroll
            for (int t = 0; t < 16; ++t)
                s = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[i][t >> 2][t & 3], f.b[j][t >> 2][t & 3], s, 0, 0, 0);
            acc[i][j] = acc[i][j] + s;
        }
}

template <int TM, int TN>
__device__ __forceinline__ void pw_rows(const ConvParams& p, int m0, int n0, int l32, const float* (&arow)[TM],
                                        int (&ab)[TM], bool (&aval)[TM], const float* (&brow)[TN], bool (&bval)[TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + i * 32 + l32;
        aval[i] = m < p.M;
        arow[i] = p.x + (int64_t)(aval[i] ? m : 0) * p.x_pstride;
        ab[i] = ((p.in_scale || p.in_shift) && aval[i]) ? (int)fdiv((uint32_t)m, p.div_howo) : 0;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + j * 32 + l32;
        bval[j] = n < p.Cout;
        brow[j] = p.w + (int64_t)(bval[j] ? n : 0) * p.Kpad;
    }
}

template <int TM, int TN>
__global__ void __launch_bounds__(256) pw_mfma_kernel(ConvParams p) {
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, l32 = lane & 31;
    const int nnt = (p.Cout + 32 * TN - 1) / (32 * TN);
    const int nmt = (p.M + 32 * TM - 1) / (32 * TM);
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wid >= nmt * nnt) return;
    const int mt = wid / nnt, nt = wid % nnt;  // waves of one block share the A panel
    const int m0 = mt * 32 * TM, n0 = nt * 32 * TN;

    const float* arow[TM];
    int ab[TM];
    bool aval[TM];
    const float* brow[TN];
    bool bval[TN];
    pw_rows<TM, TN>(p, m0, n0, l32, arow, ab, aval, brow, bval);
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    PwFrag<TM, TN> cur, nxt;
    pw_load<TM, TN>(p, nxt, arow, ab, aval, brow, bval, 16 * h);
    for (int k0 = 0; k0 < p.Kpad; k0 += 32) {
        cur = nxt;
        if (k0 + 32 < p.Kpad) pw_load<TM, TN>(p, nxt, arow, ab, aval, brow, bval, k0 + 32 + 16 * h);
        pw_mma<TM, TN>(cur, acc);
    }
    conv_epilogue<TM, TN>(p, acc, m0, n0, h, l32);
}

template <int TN, int NW>
__global__ void __launch_bounds__(NW * 64) pw_splitk_kernel(ConvParams p) {
    __shared__ floatx16 red[NW - 1][TN][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const int nnt = (p.Cout + 32 * TN - 1) / (32 * TN);
    const int mt = blockIdx.x / nnt, nt = blockIdx.x % nnt;
    const int m0 = mt * 32, n0 = nt * 32 * TN;

    const float* arow[1];
    int ab[1];
    bool aval[1];
    const float* brow[TN];
    bool bval[TN];
    pw_rows<1, TN>(p, m0, n0, l32, arow, ab, aval, brow, bval);
    floatx16 acc[1][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][j][r] = 0.f;
    const int nk = p.Kpad / 32;
    PwFrag<1, TN> cur, nxt;
    if (w < nk) pw_load<1, TN>(p, nxt, arow, ab, aval, brow, bval, w * 32 + 16 * h);
    for (int ks = w; ks < nk; ks += NW) {
        cur = nxt;
        if (ks + NW < nk) pw_load<1, TN>(p, nxt, arow, ab, aval, brow, bval, (ks + NW) * 32 + 16 * h);
        pw_mma<1, TN>(cur, acc);
    }
    if (w > 0)
#pragma unroll
        for (int j = 0; j < TN; ++j) red[w - 1][j][lane] = acc[0][j];
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        floatx16 t = acc[0][j];
        for (int q = 0; q < NW - 1; ++q) {  // fixed wave order
            const floatx16 r = red[q][j][lane];
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] += r[e];
        }
        acc[0][j] = t;
    }
    conv_epilogue<1, TN>(p, acc, m0, n0, h, l32);
}

// Streaming pointwise conv for the narrow HBM-bound 1x1 layers of the SSDLite early blocks (Cin <=
// 72, Cout <= 96, 16-image chains at 160^2 / 80^2 / 40^2): each wave walks 32-row blocks of the
// output with a grid stride, the next block's A rows in flight while the current one is multiplied
// and stored, so a wave never idles on one load-compute-store chain the way the one-tile-per-wave
// kernels do.  Exact fp32 MFMA (32x32x2): lane (r, h) holds A[row r][k = 8j + 4h + e] and the
// weight B[k][col r] for the same k (any consistent K order is a valid summation order), so K runs
// in 8-deep chunks (KJ = ceil(Cin / 8)) instead of the 32-deep padding, and the whole weight matrix
// (NB column blocks of 32 x KJ chunks) stays in registers for the wave's lifetime.
// ncg > 1: the Cout columns are split over ncg wave groups of NB blocks each (wave w takes column
// group w % ncg), so a wave's weights and accumulators stay small; PF: prefetch the next block.
template <int NB, int KJ, bool XF, bool PF>
__global__ void __launch_bounds__(256) pw_stream_kernel(ConvParams p, int ncg) {
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, r = lane & 31;
    const int nblk = (p.M + 31) / 32;
    const int wg = blockIdx.x * 4 + (threadIdx.x >> 6), nwg = gridDim.x * 4;
    const int cg = wg % ncg, gw = wg / ncg, nw = nwg / ncg;
    if (gw >= nblk || gw >= nw) return;
    const int n0 = cg * 32 * NB;
    f32x4 wb[NB][KJ];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        const int n = n0 + 32 * nb + r;
        const float* wr = p.w + (int64_t)(n < p.Cout ? n : 0) * p.Kpad + 4 * h;
#pragma unroll
        for (int j = 0; j < KJ; ++j)
            wb[nb][j] = n < p.Cout ? *reinterpret_cast<const f32x4*>(wr + 8 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto load_a = [&](int blk, f32x4 (&v)[KJ]) {
        const int m = blk * 32 + r;
        const bool ok = m < p.M;
        const float* row = p.x + (int64_t)(ok ? m : 0) * p.x_pstride + 4 * h;
        const int b = XF && ok ? (int)fdiv((uint32_t)m, p.div_howo) : 0;
#pragma unroll
        for (int j = 0; j < KJ; ++j) {
            const int k = 8 * j + 4 * h;
            f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
            if (ok && k < p.Cin) {
                x = *reinterpret_cast<const f32x4*>(row + 8 * j);
                if constexpr (XF) x = in_transform(p, x, b, k);
            }
            v[j] = x;
        }
    };
    f32x4 a[KJ];
    if (PF) load_a(gw, a);
    for (int blk = gw; blk < nblk; blk += nw) {
        const bool more = PF && blk + nw < nblk;
        f32x4 an[KJ];
        if (more) load_a(blk + nw, an);
        if (!PF) load_a(blk, a);
        floatx16 acc[1][NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[0][nb][q] = 0.f;
#pragma unroll
        for (int j = 0; j < KJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
                    acc[0][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j][e], wb[nb][j][e], acc[0][nb], 0, 0, 0);
        // lean epilogue (dense y and residual rows, checked by the launcher): one base address per
        // lane, row offsets (r & 3) + 8 (r >> 2) times the uniform pixel stride
        const int mb = blk * 32 + 4 * h;
        float bj[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) bj[nb] = p.bias[n0 + 32 * nb + r < p.Cout ? n0 + 32 * nb + r : 0];
        if (p.res) {
            const float* rb = p.res + (int64_t)mb * p.res_pstride + n0 + r;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int dm = (q & 3) + 8 * (q >> 2);
                const bool ok = mb + dm < p.M;
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
                    const bool cok = ok && n0 + 32 * nb + r < p.Cout;
                    acc[0][nb][q] = (acc[0][nb][q] + bj[nb]) + (cok ? rb[(int64_t)dm * p.res_pstride + 32 * nb] : 0.f);
                }
            }
        } else {
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[0][nb][q] += bj[nb];
        }
        switch (p.act) {
            case ACT_RELU: act_tile<1, NB, ACT_RELU>(acc); break;
            case ACT_RELU6: act_tile<1, NB, ACT_RELU6>(acc); break;
            case ACT_HSWISH: act_tile<1, NB, ACT_HSWISH>(acc); break;
            case ACT_HSIGMOID: act_tile<1, NB, ACT_HSIGMOID>(acc); break;
            case ACT_SIGMOID: act_tile<1, NB, ACT_SIGMOID>(acc); break;
            default: break;
        }
        float* yb = p.y + p.y_off + (int64_t)mb * p.y_pstride + n0 + r;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int dm = (q & 3) + 8 * (q >> 2);
            if (mb + dm < p.M)
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
                    if (n0 + 32 * nb + r < p.Cout) yb[(int64_t)dm * p.y_pstride + 32 * nb] = acc[0][nb][q];
        }
        if (more)
#pragma unroll
            for (int j = 0; j < KJ; ++j) a[j] = an[j];
    }
}

// ---------------------------------------------------------------------------------------------
// fp32 GEMM through the bf16 matrix cores: the six-term split ("bf16x6").
//
// gfx950 issues v_mfma_f32_32x32x16_bf16 at 16x the rate of v_mfma_f32_32x32x2_f32.  Every fp32
// operand is split exactly into three bf16 terms x = x0 + x1 + x2 (x0 = RN_bf16(x),
// x1 = RN_bf16(x - x0), x2 = x - x0 - x1, which fits bf16 exactly: 24 = 3 x 8 significant bits), and
// the product is accumulated from the six partial products whose magnitude is at or above
// 2^-24 |a b|:  a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0.  The three dropped terms are bounded by
// (2^-9 * 2^-18) * 3 < 2^-24 |a b|, below one fp32 rounding of the product, and every kept bf16 x bf16
// product is exact in the fp32 accumulator.  Six bf16 MFMAs (6 x 32 cycles) replace eight f32
// MFMAs (8 x 64 cycles) per 32x32x16 block: 2.67x the fp32-MFMA rate at fp32-grade accuracy.
//
// Weights arrive pre-split as three bf16 planes w3[3][Cout][Kpad] (plan.py split_bf16x3; the same
// RN split, of -w in the odd 32-wide K blocks: the sign-alternated stages, conv_x6b_body); activations are split once per block while staging (global fp32 -> registers ->
// three bf16 planes in LDS), so the split costs O(BM*K) VALU per block, not O(BM*BN*K).
// LDS: K stage of 16, rows of 16 bf16 padded to 24 (48 B: the 16-lane b128 read groups hit 16
// disjoint 4-bank groups), double-buffered through registers, one barrier per stage.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

constexpr int BK6 = 16;
constexpr int LDR6 = 24;  // padded LDS row, in bf16

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned bf16_pk(f32x2 v) {  // one v_cvt_pk_bf16_f32 (RN) for two values
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ f32x2 bf16_unpk(unsigned u) {
    return f32x2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
// x = hi + mid + lo (RN at each step), computed on element pairs: 6 packed converts, 8 unpacks and
// 8 scalar subtractions per f32x4.  The subtractions stay scalar: beside MFMAs a v_pk_add_f32
// costs about three v_sub_f32 (MI355X_MICROARCH.md, 'price of one filler'), and the library is built
// with -fno-slp-vectorize so the compiler does not re-pack them.
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ u16x8 u16x8_of(u16x4 a, u16x4 b) {
    return u16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ f32x2 sub2(f32x2 a, f32x2 b) { return f32x2{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ void split3_bf16(const f32x4& v, u16x4& h, u16x4& m, u16x4& l) {
    const f32x2 a{v.x, v.y}, b{v.z, v.w};
    const unsigned ha = bf16_pk(a), hb = bf16_pk(b);
    const f32x2 ra = sub2(a, bf16_unpk(ha)), rb = sub2(b, bf16_unpk(hb));
    const unsigned ma = bf16_pk(ra), mb = bf16_pk(rb);
    const f32x2 sa = sub2(ra, bf16_unpk(ma)), sb = sub2(rb, bf16_unpk(mb));
    h = __builtin_bit_cast(u16x4, uint2{ha, hb});
    m = __builtin_bit_cast(u16x4, uint2{ma, mb});
    l = __builtin_bit_cast(u16x4, uint2{bf16_pk(sa), bf16_pk(sb)});
}

template <int WM, int WN, int TM, int TN, bool XF, bool UT>
__global__ void __launch_bounds__(WM* WN * 64) conv_x6_kernel(ConvParams p) {
    constexpr int NT = WM * WN * 64;
    constexpr int BM = WM * TM * 32;
    constexpr int BN = WN * TN * 32;
    constexpr int AJ = BM * 4 / NT;      // f32x4 A loads per thread per stage
    constexpr int BL = 3 * BN * 2;             // 16-B B-plane loads per stage
    constexpr int BJ = (BL + NT - 1) / NT;     // ... per thread
    static_assert(AJ >= 1 && BM * 4 == AJ * NT, "tile too small for block");
    constexpr int PA = BM * LDR6, PB = BN * LDR6;  // one plane of one buffer (bf16 elements)

    __shared__ __attribute__((aligned(16))) unsigned short lds[2 * 3 * (PA + PB)];
    unsigned short* As = lds;                 // [buf][plane][BM][LDR6]
    unsigned short* Bs = lds + 2 * 3 * PA;    // [buf][plane][BN][LDR6]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wave_m = wid / WN;
    const int wave_n = wid % WN;

    const int nmt = (p.M + BM - 1) / BM;
    const int nnt = (p.Cout + BN - 1) / BN;
    const int nwg = nmt * nnt;
    int bid = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int mt = bid / nnt;
    const int nt = bid % nnt;
    const int m0 = mt * BM;
    const int n0 = nt * BN;

    const int c4 = tid & 3;  // f32x4 column within the 16-wide stage
    int64_t a_base[AJ];
    int a_ih0[AJ], a_iw0[AJ], a_b[AJ];
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
        const int row = (tid >> 2) + (NT / 4) * j;
        const int m = m0 + row;
        if (m < p.M && p.lin_x) {
            a_b[j] = XF ? (int)fdiv((uint32_t)m, p.div_howo) : 0;
            a_base[j] = (int64_t)m * p.x_pstride;
            a_ih0[j] = 0;
            a_iw0[j] = 0;
        } else if (m < p.M) {
            const int b = (int)fdiv((uint32_t)m, p.div_howo);
            const int rem = m - b * p.Ho * p.Wo;
            const int oh = (int)fdiv((uint32_t)rem, p.div_wo);
            const int ow = rem - oh * p.Wo;
            a_b[j] = b;
            a_base[j] = (int64_t)b * p.x_bstride;
            a_ih0[j] = oh * p.stride - p.pad;
            a_iw0[j] = ow * p.stride - p.pad;
        } else {
            a_b[j] = 0;
            a_base[j] = 0;
            a_ih0[j] = -(1 << 28);
            a_iw0[j] = 0;
        }
    }
    const int KHW = p.KH * p.KW;
    const int64_t wplane = (int64_t)p.Cout * p.Kpad;
    // Per-thread source pointers, fixed across K stages: the A row at filter tap (0, 0) (only
    // dereferenced when in bounds) and the B-plane row.
    const float* a_row[AJ];
#pragma unroll
    for (int j = 0; j < AJ; ++j) a_row[j] = p.x + a_base[j] + ((int64_t)a_ih0[j] * p.W + a_iw0[j]) * p.x_pstride;
    const unsigned short* b_row[BJ];
    bool b_ok[BJ];
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
        const int lin = tid + NT * j;
        const int half = lin & 1, row = (lin >> 1) % BN, pl = (lin >> 1) / BN;
        const int n = n0 + row;
        b_ok[j] = (BL % NT == 0 || lin < BL) && n < p.Cout;
        b_row[j] = reinterpret_cast<const unsigned short*>(p.w3) + pl * wplane + (int64_t)(b_ok[j] ? n : 0) * p.Kpad +
                   8 * half;
    }
    // Cin % 16 == 0: a 16-wide K stage never crosses a filter tap, so the tap of a stage is
    // wavefront-uniform (scalar) and a thread's A address is its row pointer plus a uniform offset.

    struct Regs {
        f32x4 a[AJ];
        uint4 b[BJ];
        float sg;  // the stage's sign (the split weights' odd 32-wide K blocks are negated, conv_x6b_body)
    };
    Regs r0, r1;

    auto load_stage = [&](Regs& R, int k0) {
        R.sg = ((k0 >> 5) & 1) ? -1.f : 1.f;
        if constexpr (UT) {
            const int tap = (int)fdiv((uint32_t)k0, p.div_cin);
            const int ci = k0 - tap * p.Cin + c4 * 4;
            const int kh = (int)fdiv((uint32_t)tap, p.div_kw);
            const int kw = tap - kh * p.KW;
            const bool kval = tap < KHW;
            const int64_t off = ((int64_t)kh * p.W + kw) * p.x_pstride + ci;
#pragma unroll
            for (int j = 0; j < AJ; ++j) {
                f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
                if (kval && (unsigned)(a_ih0[j] + kh) < (unsigned)p.H && (unsigned)(a_iw0[j] + kw) < (unsigned)p.W) {
                    v = *reinterpret_cast<const f32x4*>(a_row[j] + off);
                    if constexpr (XF) v = in_transform(p, v, a_b[j], ci);
                }
                R.a[j] = v;
            }
        } else {
            const int k = k0 + c4 * 4;
            const int tap = (int)fdiv((uint32_t)k, p.div_cin);
            const int ci = k - tap * p.Cin;
            const int kh = (int)fdiv((uint32_t)tap, p.div_kw);
            const int kw = tap - kh * p.KW;
            const bool kval = tap < KHW;
#pragma unroll
            for (int j = 0; j < AJ; ++j) {
                const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
                f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
                if (kval && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) {
                    v = *reinterpret_cast<const f32x4*>(p.x + a_base[j] + (int64_t)(ih * p.W + iw) * p.x_pstride + ci);
                    if constexpr (XF) v = in_transform(p, v, a_b[j], ci);
                }
                R.a[j] = v;
            }
        }
#pragma unroll
        for (int j = 0; j < BJ; ++j)
            R.b[j] = (BL % NT == 0 || tid + NT * j < BL) ? *reinterpret_cast<const uint4*>(b_row[j] + k0)
                                                       : uint4{0u, 0u, 0u, 0u};  // rows past Cout: row 0
    };
    float sgb0 = 1.f, sgb1 = 1.f;
    auto store_stage = [&](const Regs& R, int buf) {
        unsigned short* A = As + buf * 3 * PA;
        unsigned short* Bb = Bs + buf * 3 * PB;
        if (buf)
            sgb1 = R.sg;
        else
            sgb0 = R.sg;
#pragma unroll
        for (int j = 0; j < AJ; ++j) {
            const int row = (tid >> 2) + (NT / 4) * j;
            u16x4 h, m, l;
            split3_bf16(R.a[j], h, m, l);
            *reinterpret_cast<u16x4*>(A + 0 * PA + row * LDR6 + c4 * 4) = h;
            *reinterpret_cast<u16x4*>(A + 1 * PA + row * LDR6 + c4 * 4) = m;
            *reinterpret_cast<u16x4*>(A + 2 * PA + row * LDR6 + c4 * 4) = l;
        }
#pragma unroll
        for (int j = 0; j < BJ; ++j) {
            const int lin = tid + NT * j;
            const int half = lin & 1, row = (lin >> 1) % BN, pl = (lin >> 1) / BN;
            if (BL % NT == 0 || lin < BL) *reinterpret_cast<uint4*>(Bb + pl * PB + row * LDR6 + 8 * half) = R.b[j];
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = p.Kpad / BK6;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    auto compute = [&](int buf) {
        const unsigned short* A = As + buf * 3 * PA;
        const unsigned short* Bb = Bs + buf * 3 * PB;
        const float sg = buf ? sgb1 : sgb0;
        bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                af[i][pl] = *reinterpret_cast<const bf16x8*>(A + pl * PA + (wave_m * TM * 32 + i * 32 + l32) * LDR6 + 8 * h);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                bfr[j][pl] = *reinterpret_cast<const bf16x8*>(Bb + pl * PB + (wave_n * TN * 32 + j * 32 + l32) * LDR6 + 8 * h);
        // the stage's six split products, smallest first, into a stage sum that starts at zero, then
        // one fp32 add into the running output (the error structure of conv_x6b_body's mfma16)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                floatx16 s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][2], bfr[j][0], floatx16{}, 0, 0, 0);
                s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bfr[j][1], s, 0, 0, 0);
                s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bfr[j][2], s, 0, 0, 0);
                s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bfr[j][0], s, 0, 0, 0);
                s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bfr[j][1], s, 0, 0, 0);
                s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bfr[j][0], s, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_fmaf(sg, s[r], acc[i][j][r]);
            }
    };
    load_stage(r0, 0);
    store_stage(r0, 0);
    __syncthreads();
    for (int kc = 0; kc < nk; ++kc) {
        if (kc + 1 < nk) load_stage(r0, (kc + 1) * BK6);
        compute(kc & 1);
        if (kc + 1 < nk) store_stage(r0, (kc & 1) ^ 1);
        __syncthreads();
    }

    conv_epilogue<TM, TN>(p, acc, m0 + wave_m * TM * 32, n0 + wave_n * TN * 32, h, l32);
}

// bf16x6 with a 32-deep K stage: 256 x 128 block tile on 8 waves (4 x 2, 64 x 64 per wave), 48 MFMAs
// per wave between barriers.  LDS rows are 32 bf16 (64 B) with the 16-B chunks XOR-swizzled by
// row bit 3 (chunk' = chunk ^ ((row >> 2) & 2)).  The fragment reads are the 16x16x32 form (lane l:
// row l & 15, chunk l >> 4), and the four ds_read_b128 lane groups ({0-3,12-15,20-27}, {4-11,16-19,
// 28-31}, and the same +32) then hit 16 distinct 16-B slots of the 256-B bank row (conflict-free; the
// row bits 2..3 swizzle of the 32x32x16 form left them 2-way).  The double-buffered image of the
// three A and three B planes fits 144 KiB (one block of 8 waves per CU, two waves per SIMD).
constexpr int BK6B = 32;
constexpr int X3Z = 32;  // leading zero elements of a pre-split scratch (16-B aligned planes follow)

__device__ __forceinline__ int swz_key(int row) { return (row >> 2) & 2; }
__device__ __forceinline__ int swz64(int row, int chunk) { return row * 32 + 8 * (chunk ^ swz_key(row)); }

// XF: the input transform is active (SE scale / GN shift / ReLU); UT: Cin % 32 == 0, so every stage
// lies inside one filter tap and the tap decomposition is wave-uniform (scalar) work.
// PS: the input arrives pre-split (p.x3: three dense bf16 planes written by split_act_kernel, input
// transform already applied), so a stage is 2 rows x 3 planes of 16-B loads per thread, stored to
// LDS unchanged (requires UT, !XF).
// BM = 256: 4 x 2 waves of 64 x 64; BM = 128: 2 x 4 waves of 64 x 32 (twice the workgroups for the
// small-M layers, half the MFMAs per barrier); BM = 64: 2 x 4 waves of 32 x 32, 72 KiB of LDS and at
// most 128 VGPRs, so two workgroups (four waves per SIMD) share a CU.  PF = 2: two register stages
// (loads two stages ahead, B register-staged too) instead of the skewed one-register-stage pipeline.
// P1: 1x1, stride 1, dense input (p.lin_x): a stage's k0 is the channel, and rows past M load row 0
// (their outputs are never stored), so the A loads need no tap or bounds work; with Cin % 32 != 0
// (!UT) the chunks past Cin are zeroed (they meet the zero weight padding).
// BN = 64 (with BM = 128, the skewed 16x16x32 pipeline and LDS-DMA B only): 4 x 2 waves of 32 x 32
// for the Cout = 64 layers, which a 128-wide N tile computes half empty; waves 0..3 copy the B rows.
// BN = 256 (BM = 128, same conditions): 2 x 4 waves of 64 x 64 in the same 144 KiB, so a Cout = 256
// layer reads each A panel once (the 256 x 128 tile's two N tiles read it twice) and splits half the
// A elements per MFMA; each wave copies 32 B rows by LDS-DMA.
template <bool XF, bool UT, bool PS, int BM = 256, int PF = 1, bool P1 = false, int BN = 128>
__device__ __forceinline__ void conv_x6b_body(const ConvParams& p, const int blk) {
    static_assert(!PS || (UT && !XF), "pre-split input: uniform taps, transform applied by the split");
    static_assert(BM == 256 || ((BM == 128 || BM == 64) && !PS), "x6b tiles: 256 x 128, or 128 | 64 x 128 without pre-split input");
    static_assert(!P1 || !PS, "pointwise stages: fp32 input");
    constexpr bool GL = PF != 2;  // B planes by LDS-DMA (needs the one-register-stage loops)
    static_assert(BN == 128 || ((BN == 64 || BN == 256) && BM == 128 && GL && !PS), "x6b BN = 64 | 256: 128 x BN, LDS-DMA B");
    constexpr int WM = BN == 64 ? 4 : BN == 256 ? 2 : (BM == 256 ? 4 : 2), WN = 8 / WM;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32), NT = 512;
    constexpr int AJ = PS ? BM * 4 / NT : BM * BK6B / 4 / NT;  // A rows per thread (2 | 4 f32x4 loads)
    constexpr int AROWS = NT / (PS ? 4 : 8);                   // row step between a thread's A rows
    constexpr int PA = BM * BK6B, PB = BN * BK6B;  // bf16 elements per plane
    static_assert(3 * BN * BK6B / 8 == 3 * NT || GL, "register-staged B: one B-plane chunk per thread per plane");

    __shared__ __attribute__((aligned(16))) unsigned short lds[2 * 3 * (PA + PB)];
    unsigned short* As = lds;
    unsigned short* Bs = lds + 2 * 3 * PA;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wave_m = wid / WN;
    const int wave_n = wid % WN;

    const int nmt = (p.M + BM - 1) / BM;
    const int nnt = (p.Cout + BN - 1) / BN;
    const int nwg = nmt * nnt;
    const int ksp = p.ksplit > 1 ? 2 : 1;  // split-K: block 2t + s takes K half s of tile t
    int bid = blk / ksp;
    {
        const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int m0 = (bid / nnt) * BM;
    const int n0 = (bid % nnt) * BN;

    const int c8 = tid & 7;  // f32x4 column of the 32-deep stage
    // A rows of this thread: with LDS-DMA of the pre-split planes (PS && GL) wave w owns rows
    // 32w .. 32w+31 (two 1-KiB blocks, lane l -> 16-B slot l); otherwise rows step by AROWS
    const int a_row0 = PS ? (GL ? 32 * wid + (lane >> 2) : tid >> 2) : tid >> 3;
    constexpr int AST = PS && GL ? 16 : AROWS;
    // pixel / batch strides of the A source: the fp32 input, or the dense bf16 planes
    const int x_ps = PS ? p.Cin : p.x_pstride;
    const int64_t x_bs = PS ? (int64_t)p.H * p.W * p.Cin : p.x_bstride;
    int64_t a_base[AJ];
    int a_ih0[AJ], a_iw0[AJ], a_b[AJ];
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
        const int m = m0 + a_row0 + AST * j;
        if (m < p.M && p.lin_x) {
            a_b[j] = XF ? (int)fdiv((uint32_t)m, p.div_howo) : 0;
            a_base[j] = (int64_t)m * x_ps;
            a_ih0[j] = 0;
            a_iw0[j] = 0;
        } else if (m < p.M) {
            const int b = (int)fdiv((uint32_t)m, p.div_howo);
            const int rem = m - b * p.Ho * p.Wo;
            const int oh = (int)fdiv((uint32_t)rem, p.div_wo);
            const int ow = rem - oh * p.Wo;
            a_b[j] = b;
            a_ih0[j] = oh * p.stride - p.pad;
            a_iw0[j] = ow * p.stride - p.pad;
            // UT: fold the window origin into the base (the tap offset is added per stage)
            a_base[j] = (int64_t)b * x_bs + (UT ? (int64_t)(a_ih0[j] * p.W + a_iw0[j]) * x_ps : 0);
        } else {
            a_b[j] = 0;
            a_base[j] = 0;
            a_ih0[j] = -(1 << 28);
            a_iw0[j] = 0;
        }
    }
    const int KHW = p.KH * p.KW;
    const int64_t wplane = (int64_t)p.Cout * p.Kpad;
    const int b_row = tid >> 2, b_chunk = tid & 3;
    const bool b_ok = n0 + b_row < p.Cout;
    const unsigned short* b_src = reinterpret_cast<const unsigned short*>(p.w3) +
                                  (int64_t)(b_ok ? n0 + b_row : 0) * p.Kpad + 8 * b_chunk;

    struct Regs {
        f32x4 a[PS ? 1 : AJ];
        uint4 a3[PS ? AJ : 1][3];
        uint4 b[3];
        float sg;  // the stage's sign (sign-alternated stages, below)
    };
    const int64_t x3plane = (int64_t)p.B * p.H * p.W * p.Cin;
    // x3 scratch: X3Z zero elements (the source of padding taps under LDS-DMA), then the three planes
    const unsigned short* x3 = reinterpret_cast<const unsigned short*>(p.x3);
    // la / lb: load the stage's A rows (to registers, or to LDS by DMA under PS && GL) / its B rows
    // A stage's K position: k0, and (uniform-tap stages, channel-chunk-major order) its filter tap
    // and first channel, advanced incrementally by the cursor below
    struct StageK {
        int k0, kh, kw, ci;
    };
    auto stage_tap = [&](const StageK& sk, int& kh, int& kw, int& ci0) {
        kh = sk.kh;
        kw = sk.kw;
        ci0 = sk.ci;
    };
    auto load_stage = [&](Regs& R, const StageK& sk, int bbuf) {
        const int k0 = sk.k0;
        R.sg = ((k0 >> 5) & 1) ? -1.f : 1.f;  // the sign the split weights carry for this K block
        if constexpr (GL) {
            // B by LDS-DMA: wave w copies rows rb + 16w .. rb + 16w + 15 of each plane for every 128-row
            // block rb (1 KiB per instruction, lane l -> the 16-B slot l of the block); the swizzle is
            // applied on the source address
#pragma unroll
            for (int rb = 0; rb < BN; rb += 128) {
                if (rb + 16 * wid >= BN) break;
                const int row = rb + 16 * wid + (lane >> 2), pc = lane & 3, lc = pc ^ swz_key(row);
                const int n = n0 + row < p.Cout ? n0 + row : p.Cout - 1;
                const unsigned short* src = reinterpret_cast<const unsigned short*>(p.w3) + (int64_t)n * p.Kpad + k0 + 8 * lc;
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void*)(src + pl * wplane),
                        (__attribute__((address_space(3))) void*)(Bs + bbuf * 3 * PB + pl * PB + (rb + 16 * wid) * BK6B), 16,
                        0, 0);
            }
        }
        if constexpr (PS) {
            int kh, kw, ci0;
            stage_tap(sk, kh, kw, ci0);
            if constexpr (GL) {
                const unsigned short* xt = x3 + X3Z + (int64_t)(kh * p.W + kw) * p.Cin + ci0;
#pragma unroll
                for (int j = 0; j < AJ; ++j) {
                    const int row = a_row0 + AST * j;
                    const int lc = (lane & 3) ^ swz_key(row);  // swizzle on the source address
                    const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
                    const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
                        __builtin_amdgcn_global_load_lds(
                            (const __attribute__((address_space(1))) void*)(ok ? xt + pl * x3plane + a_base[j] + 8 * lc
                                                                               : x3),
                            (__attribute__((address_space(3))) void*)(As + bbuf * 3 * PA + pl * PA +
                                                                      (32 * wid + 16 * j) * BK6B),
                            16, 0, 0);
                }
            } else {
                const unsigned short* xt = x3 + X3Z + (int64_t)(kh * p.W + kw) * p.Cin + ci0 + 8 * (tid & 3);
#pragma unroll
                for (int j = 0; j < AJ; ++j) {
                    const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
                    const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
                        R.a3[j][pl] =
                            ok ? *reinterpret_cast<const uint4*>(xt + pl * x3plane + a_base[j]) : uint4{0u, 0u, 0u, 0u};
                }
            }
        } else if constexpr (P1) {
            const int ci = k0 + c8 * 4;
            const float* xt = p.x + ci;
#pragma unroll
            for (int j = 0; j < AJ; ++j) {
                // (a chunk past Cin loads from p.x: past the last pixel it would leave the buffer)
                const bool cok = UT || ci < p.Cin;
                f32x4 v = *reinterpret_cast<const f32x4*>(cok ? xt + a_base[j] : p.x);
                if constexpr (XF) v = in_transform(p, v, a_b[j], cok ? ci : 0);
                if constexpr (!UT) v = cok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
                R.a[j] = v;
            }
        } else if constexpr (UT) {
            int kh, kw, ci0;
            stage_tap(sk, kh, kw, ci0);
            const int ci = ci0 + c8 * 4;
            const float* xt = p.x + (int64_t)(kh * p.W + kw) * p.x_pstride + ci;
#pragma unroll
            for (int j = 0; j < AJ; ++j) {
                // (a branch-free form, padding taps loading from p.x and zeroed, measured 3-5% slower)
                const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
                const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
                f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
                if (ok) {
                    v = *reinterpret_cast<const f32x4*>(xt + a_base[j]);
                    if constexpr (XF) v = in_transform(p, v, a_b[j], ci);
                }
                R.a[j] = v;
            }
        } else {
            const int k = k0 + c8 * 4;
            const int tap = (int)fdiv((uint32_t)k, p.div_cin);
            const int ci = k - tap * p.Cin;
            const int kh = (int)fdiv((uint32_t)tap, p.div_kw);
            const int kw = tap - kh * p.KW;
            const bool kval = tap < KHW;
#pragma unroll
            for (int j = 0; j < AJ; ++j) {
                const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
                f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
                if (kval && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) {
                    v = *reinterpret_cast<const f32x4*>(p.x + a_base[j] + (int64_t)(ih * p.W + iw) * p.x_pstride + ci);
                    if constexpr (XF) v = in_transform(p, v, a_b[j], ci);
                }
                R.a[j] = v;
            }
        }
        if (!GL) {
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                R.b[pl] = b_ok ? *reinterpret_cast<const uint4*>(b_src + pl * wplane + k0) : uint4{0u, 0u, 0u, 0u};
        }
    };
    // Sign-alternated stages: the split weight planes hold -w in every odd 32-wide K block
    // (split_bf16x3_kernel), so those stages' sums come out negated and are subtracted.  The matrix
    // core aligns each lane group's 8 products to the largest and truncates the rest toward -inf
    // (a 22-bit window, fitted to tools/accuracy_probe.py), a bias that grows with K; on negated
    // stages the same truncation rounds the other way, so over the stages it cancels.
    // sgb<buf>: the sign of the stage held in LDS buffer buf.
    float sgb0 = 1.f, sgb1 = 1.f;
    auto store_stage = [&](const Regs& R, int buf) {
        unsigned short* A = As + buf * 3 * PA;
        unsigned short* Bb = Bs + buf * 3 * PB;
        if (buf)
            sgb1 = R.sg;
        else
            sgb0 = R.sg;
        if constexpr (PS && GL) {
            // A arrived by LDS-DMA
        } else if constexpr (PS) {
#pragma unroll
            for (int j = 0; j < AJ; ++j) {
                const int o = swz64(a_row0 + AROWS * j, tid & 3);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<uint4*>(A + pl * PA + o) = R.a3[j][pl];
            }
        } else {
#pragma unroll
            for (int j = 0; j < AJ; ++j) {
                const int row = a_row0 + AROWS * j;
                u16x4 h, m, l;
                split3_bf16(R.a[j], h, m, l);
                const int o = swz64(row, c8 >> 1) + 4 * (c8 & 1);
                *reinterpret_cast<u16x4*>(A + 0 * PA + o) = h;
                *reinterpret_cast<u16x4*>(A + 1 * PA + o) = m;
                *reinterpret_cast<u16x4*>(A + 2 * PA + o) = l;
            }
        }
        const int o = swz64(b_row, b_chunk);
        if constexpr (!GL)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<uint4*>(Bb + pl * PB + o) = R.b[pl];
    };

    const int nk_all = p.Kpad / BK6B;
    const int kbeg = ksp > 1 ? (blk & 1) * ((nk_all + 1) / 2) : 0;  // stage range of this block
    const int nk = ksp > 1 ? ((blk & 1) ? nk_all - kbeg : (nk_all + 1) / 2) : nk_all;
    // Stage order. Tap-major (stage s at k = 32 s, the weight layout) sweeps a block's whole input
    // panel once per filter tap; with a uniform tap the stages run channel-chunk-major instead (the
    // KH*KW taps of one 32-channel chunk back to back, k = tap * Cin + 32 * chunk; K = KH*KW*Cin is
    // then Kpad), so the chunk's input window is re-read from L2 across the taps rather than from
    // HBM.  Stages are loaded strictly in order, so the cursor advances by one per load, tap and
    // channel incrementally (no divisions in the loop).
    constexpr bool cm = UT && !P1;
    struct Cursor {
        int tap, chunk, k, kh, kw;
    };
    Cursor ca{cm ? kbeg % KHW : 0, cm ? kbeg / KHW : 0, kbeg * BK6B, 0, 0};
    if constexpr (cm) {
        ca.kh = ca.tap / p.KW;
        ca.kw = ca.tap - ca.kh * p.KW;
    }
    auto next_k = [&](Cursor& c) {
        StageK sk;
        if constexpr (cm) {
            sk = StageK{c.tap * p.Cin + c.chunk * BK6B, c.kh, c.kw, c.chunk * BK6B};
            ++c.tap;
            if (++c.kw == p.KW) {
                c.kw = 0;
                ++c.kh;
            }
            if (c.tap == KHW) {
                c.tap = 0;
                c.kh = 0;
                ++c.chunk;
            }
        } else {
            sk = StageK{c.k, -1, 0, 0};
            c.k += BK6B;
        }
        return sk;
    };
    const int h = lane >> 5;
    const int l32 = lane & 31;
    // 16x16x32 form: the wave's 32TM x 32TN tile as (2TM) x (2TN) 16x16 C tiles, each MFMA taking the
    // whole 32-deep stage (lane l: row l & 15, k chunk l >> 4 of the swizzled 64-B row).  Under load
    // the chip holds a higher clock for this shape than for 32x32x16 at the same cycles per FLOP
    // (MI355X_MICROARCH.md, DVFS item 7; FRCNN 311 -> 329 img/s same-box).  A fragment half is TM row
    // blocks (or TN column blocks) of 16, so a stage's MFMAs fall into four quadrants (row half,
    // column half).
    struct F16 {
        bf16x8 a[TM][3], b[TN][3];
    };
    f32x4 acc4[2 * TM][2 * TN];
#pragma unroll
    for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
        for (int j = 0; j < 2 * TN; ++j) acc4[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int r16 = lane & 15, c16 = lane >> 4;
    auto read16 = [&](F16& F, int buf, int s) {
        const unsigned short* A = As + buf * 3 * PA;
        const unsigned short* Bb = Bs + buf * 3 * PB;
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            const int o = swz64(wave_m * TM * 32 + 16 * (s * TM + t) + r16, c16);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) F.a[t][pl] = *reinterpret_cast<const bf16x8*>(A + pl * PA + o);
        }
#pragma unroll
        for (int u = 0; u < TN; ++u) {
            const int o = swz64(wave_n * TN * 32 + 16 * (s * TN + u) + r16, c16);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) F.b[u][pl] = *reinterpret_cast<const bf16x8*>(Bb + pl * PB + o);
        }
    };
    // Stage sums (mfma16 below: quadrant (ha, hb) from the A half in FA and the B half in FB).  The
    // stage's six split products (smallest first: a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0) chain into
    // a fresh stage sum that starts at zero, and the running output takes that sum with ONE fp32 add:
    // each MFMA rounds its lane-group partial sums into C one group at a time, so chaining the six
    // terms into the running output rounded it 24 times per stage at its full magnitude; the stage
    // sum takes those roundings at the stage's (K/32 times smaller) magnitude.  RMS error against
    // float64 on the 3x3 256->256 conv 1.39e-7 -> 3.2e-8, below torch's CPU conv.
    // Cost: the adds are VALU work the old chain did not have (box head 3x3 2.08 -> 2.36 ms).
    // A tile's stage-sum add is issued after the NEXT tile's six MFMAs (pend), so the MFMA result it
    // reads has landed and no wait states separate them; flush() adds the last pending one.
    struct Pend {
        f32x4 v;
        float sg;
        int i, j;  // acc4 tile, -1: none (constants after unrolling)
    } pend{f32x4{0.f, 0.f, 0.f, 0.f}, 1.f, -1, -1};
    auto flush = [&]() {
        if (pend.i >= 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r)  // c +- s, one rounding
                acc4[pend.i][pend.j][r] = __builtin_fmaf(pend.sg, pend.v[r], acc4[pend.i][pend.j][r]);
        }
        pend.i = -1;
    };
    auto mfma16 = [&](const F16& FA, const F16& FB, int ha, int hb, float sg) {
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int u = 0; u < TN; ++u) {
                f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA.a[t][2], FB.b[u][0], f32x4{0.f, 0.f, 0.f, 0.f},
                                                                  0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA.a[t][1], FB.b[u][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA.a[t][0], FB.b[u][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA.a[t][1], FB.b[u][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA.a[t][0], FB.b[u][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA.a[t][0], FB.b[u][0], c, 0, 0, 0);
                // nothing but memory and scalar work crosses: the previous tile's add stays behind this
                // chain (left free, the scheduler pulls each add up against its own chain and the two
                // serialise on a wait for the MFMA result; box head 3x3 2.44 -> 2.36 ms)
                __builtin_amdgcn_sched_barrier(0x3F4);
                flush();
                pend = Pend{c, sg, ha * TM + t, hb * TN + u};
            }
    };
    // static priority for waves 4..7, the arbitration losers of a two-waves-per-SIMD block
    // (MI355X_MICROARCH.md, two waves per SIMD, item 4)
    if constexpr (PF != 2) {
        // Skewed pipeline: quadrant (1, 1) of stage k-1 is carried across the barrier in F1, so after
        // the barrier the matrix pipe runs it while stage k's first fragments are read; stage k+1's
        // operands are written to the other buffer under stage k's MFMAs.
        Regs r0;
        F16 F0, F1;
        load_stage(r0, next_k(ca), 0);
        store_stage(r0, 0);
        __syncthreads();
        if (nk > 1) load_stage(r0, next_k(ca), 1);
        read16(F0, 0, 0);
        read16(F1, 0, 1);
        float sgc = sgb0;  // the sign of the stage in F0 / F1 (F1's quadrant (1, 1) is carried)
        mfma16(F0, F0, 0, 0, sgc);
        mfma16(F0, F1, 0, 1, sgc);
        mfma16(F1, F0, 1, 0, sgc);
        if (nk > 1) store_stage(r0, 1);
        flush();
        __syncthreads();
        for (int kc = 1; kc < nk; ++kc) {
            const int buf = kc & 1;
            if (kc + 1 < nk) load_stage(r0, next_k(ca), buf ^ 1);
            read16(F0, buf, 0);
            __builtin_amdgcn_sched_barrier(0);  // issue the reads before the carried quadrant that hides them
            mfma16(F1, F1, 1, 1, sgc);
            __builtin_amdgcn_sched_barrier(0);  // F1 is rewritten only after the carried quadrant issued
            sgc = buf ? sgb1 : sgb0;
            read16(F1, buf, 1);
            mfma16(F0, F0, 0, 0, sgc);
            mfma16(F0, F1, 0, 1, sgc);
            mfma16(F1, F0, 1, 0, sgc);
            store_stage(r0, buf ^ 1);  // on the last stage a dead write of the idle buffer
            flush();
            // Spread the split VALU, the LDS writes of stage k+1 and the fragment reads over the gaps
            // of the MFMAs (1 MFMA : 1 LDS read : 3 VALU : 1 LDS write; 0 groups cost FRCNN 3%, 1..5
            // VALU within 1%) instead of letting them bunch up after the last MFMA.
#pragma unroll
            for (int i = 0; i < TM * TN * 18; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // VALU
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
            }
            __syncthreads();
        }
        mfma16(F1, F1, 1, 1, sgc);
        flush();
    } else {
        // Two register stages: stage k+2's global loads are issued before stage k's MFMAs, stage k+1's
        // (issued one stage earlier) are stored to LDS after them, so each load has two stages of MFMA
        // time to land.
        Regs r0, r1;
        load_stage(r0, next_k(ca), 0);
        store_stage(r0, 0);
        if (nk > 1) load_stage(r1, next_k(ca), 1);
        __syncthreads();
        auto step = [&](int kc, Regs& hold, Regs& next) {
            if (kc + 2 < nk) load_stage(next, next_k(ca), kc & 1);  // (no LDS-DMA with two register stages)
            F16 F0, F1;
            read16(F0, kc & 1, 0);
            read16(F1, kc & 1, 1);
            const float sgc = (kc & 1) ? sgb1 : sgb0;
            mfma16(F0, F0, 0, 0, sgc);
            mfma16(F0, F1, 0, 1, sgc);
            mfma16(F1, F0, 1, 0, sgc);
            mfma16(F1, F1, 1, 1, sgc);
            if (kc + 1 < nk) store_stage(hold, (kc & 1) ^ 1);
            flush();
            __syncthreads();
        };
        for (int kc = 0; kc < nk; kc += 2) {
            step(kc, r1, r0);
            if (kc + 1 < nk) step(kc + 1, r0, r1);
        }
    }
    // back to the 32x32 block view of the epilogue: block (i, j) register 4(2ii + jj) + r
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[i][j][4 * q + r] = acc4[2 * i + (q >> 1)][2 * j + (q & 1)][r];
    conv_epilogue<TM, TN, true>(p, acc, m0 + wave_m * TM * 32, n0 + wave_n * TN * 32, h, l32);
}

// The kernel of one conv problem, and the grouped form (csrc/exec.hip EDGEDET_OP_GROUP): one launch
// over up to EDGEDET_MAX_GROUP independent problems of the same tile and template variant (e.g. the
// twelve SSDLite head 1x1 convs), workgroup ranges [g.start[k], g.start[k+1]) running problem k with
// its own XCD-aware block order.
// Timing probe of a launch (ConvParams::stamp, bench.py's in-pipeline roofline; a null pointer in every
// product plan, so the product path pays one uniform branch), on the 100 MHz constant clock with vector
// atomics: stamp[0] = the start of workgroup 0 (workgroups are dispatched in id order, so it is the
// first to start), stamp[1] = max of every workgroup's end.  The clock only grows and one slot serves
// one stream's launches in order, so the slot needs no reset between launches: stamp[1] - stamp[0]
// after a launch is that launch's span.
__device__ __forceinline__ void stamp_begin(unsigned long long* st) {
    if (st && threadIdx.x == 0 && blockIdx.x == 0)
        atomicExch(st, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void stamp_end(unsigned long long* st) {
    if (st) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(st + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

template <bool XF, bool UT, bool PS, int BM = 256, int PF = 1, bool P1 = false, int BN = 128>
__global__ void __launch_bounds__(512, BM == 64 || BN == 64 ? 2 : 1) conv_x6b_kernel(ConvParams p) {
    stamp_begin(p.stamp);
    conv_x6b_body<XF, UT, PS, BM, PF, P1, BN>(p, (int)blockIdx.x);
    stamp_end(p.stamp);
}

template <bool XF, bool UT, int BM, bool P1, int BN>
__global__ void __launch_bounds__(512, BM == 64 || BN == 64 ? 2 : 1) conv_x6b_group_kernel(ConvGroup g) {
    const int bx = (int)blockIdx.x;
    stamp_begin(g.p[0].stamp);
    int k = 0;
    while (k + 1 < g.n && bx >= g.start[k + 1]) ++k;  // uniform: scalar loads of the range table
    conv_x6b_body<XF, UT, false, BM, 1, P1, BN>(g.p[k], bx - g.start[k]);
    stamp_end(g.p[0].stamp);
}

// Pre-split of a conv input for the PS tile: out[pl][pix][c] (three dense bf16 planes, the RN split
// of split3_bf16) of transform(x[pix][c]); 8 channels per thread, a grid-stride pass.  HBM-bound:
// 4 B read + 6 B written per element.
template <bool XF>
__global__ void __launch_bounds__(256) split_act_kernel(ConvParams p) {
    const int C8 = p.Cin >> 3;
    const int64_t HW = (int64_t)p.H * p.W, npix = (int64_t)p.B * HW, n = npix * C8;
    unsigned short* out = reinterpret_cast<unsigned short*>(p.x3) + X3Z;
    if (blockIdx.x == 0 && threadIdx.x < X3Z / 8)  // the zero page padding taps read under LDS-DMA
        reinterpret_cast<uint4*>(p.x3)[threadIdx.x] = uint4{0u, 0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t pix = i / C8;
        const int c = (int)(i - pix * C8) * 8;
        const int64_t b = pix / HW;
        const float* src = p.x + b * p.x_bstride + (pix - b * HW) * p.x_pstride + c;
        f32x4 v0 = *reinterpret_cast<const f32x4*>(src), v1 = *reinterpret_cast<const f32x4*>(src + 4);
        if constexpr (XF) {
            v0 = in_transform(p, v0, (int)b, c);
            v1 = in_transform(p, v1, (int)b, c + 4);
        }
        u16x4 h0, m0, l0, h1, m1, l1;
        split3_bf16(v0, h0, m0, l0);
        split3_bf16(v1, h1, m1, l1);
        unsigned short* d = out + pix * p.Cin + c;
        const int64_t plane = npix * p.Cin;
        *reinterpret_cast<uint4*>(d) = __builtin_bit_cast(uint4, u16x8_of(h0, h1));
        *reinterpret_cast<uint4*>(d + plane) = __builtin_bit_cast(uint4, u16x8_of(m0, m1));
        *reinterpret_cast<uint4*>(d + 2 * plane) = __builtin_bit_cast(uint4, u16x8_of(l0, l1));
    }
}

static bool x6b_presplit(const ConvParams& p) {
    return p.x3 && p.Cin % BK6B == 0 && p.x_pstride % 4 == 0 && ((uintptr_t)p.x3 & 15) == 0;
}


template <int BM = 256, int PF = 1, int BN = 128>
static int launch_x6b(const ConvParams& p0, hipStream_t s) {
    ConvParams p = p0;
    EDGEDET_REQUIRE(p.w3 && ((uintptr_t)p.w3 & 15) == 0, "conv bf16x6: needs 16-byte aligned split weight planes");
    EDGEDET_REQUIRE(p.Kpad % BK6B == 0, "conv bf16x6: Kpad must be a multiple of 32");
    if (p.ksplit > 1)
        EDGEDET_REQUIRE(p.ksplit == 2 && !p.res && p.act == 0 && p.Kpad >= 2 * BK6B,
                        "conv split-K: 2 halves, no residual, no activation (y must be zeroed)");
    const int64_t nwg = cdiv(p.M, BM) * cdiv(p.Cout, BN) * (p.ksplit > 1 ? 2 : 1);
    EDGEDET_REQUIRE(nwg < (1ll << 31), "conv grid too large");
    const bool xf = p.in_scale || p.in_shift || p.in_relu, ut = p.Cin % BK6B == 0;
    if (BM == 256 && BN == 128 && x6b_presplit(p)) {
        const int64_t items = (int64_t)p.B * p.H * p.W * (p.Cin / 8);
        const unsigned g = (unsigned)std::min<int64_t>(cdiv(items, 256), 256 * 64);
        hipLaunchKernelGGL(xf ? split_act_kernel<true> : split_act_kernel<false>, dim3(g), dim3(256), 0, s, p);
        EDGEDET_LAUNCH_CHECK();
        hipLaunchKernelGGL((conv_x6b_kernel<false, true, true>), dim3((unsigned)nwg), dim3(512), 0, s, p);
        EDGEDET_LAUNCH_CHECK();
        return 0;
    }
    const bool p1 = p.lin_x && p.KH == 1 && p.KW == 1 && p.Cin % 4 == 0;
    auto k = p1 ? (xf ? (ut ? conv_x6b_kernel<true, true, false, BM, PF, true, BN> : conv_x6b_kernel<true, false, false, BM, PF, true, BN>)
                      : (ut ? conv_x6b_kernel<false, true, false, BM, PF, true, BN> : conv_x6b_kernel<false, false, false, BM, PF, true, BN>))
         : xf ? (ut ? conv_x6b_kernel<true, true, false, BM, PF, false, BN> : conv_x6b_kernel<true, false, false, BM, PF, false, BN>)
              : (ut ? conv_x6b_kernel<false, true, false, BM, PF, false, BN> : conv_x6b_kernel<false, false, false, BM, PF, false, BN>);
    hipLaunchKernelGGL(k, dim3((unsigned)nwg), dim3(512), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

template <int BM, int BN>
static int launch_x6b_group(ConvGroup& g, hipStream_t s) {
    const ConvParams& p = g.p[0];
    const bool xf = p.in_scale || p.in_shift || p.in_relu, ut = p.Cin % BK6B == 0;
    const bool p1 = p.lin_x && p.KH == 1 && p.KW == 1 && p.Cin % 4 == 0;
    int64_t total = 0;
    for (int k = 0; k < g.n; ++k) {
        const ConvParams& q = g.p[k];
        EDGEDET_REQUIRE(q.w3 && ((uintptr_t)q.w3 & 15) == 0 && q.Kpad % BK6B == 0 && q.ksplit <= 1,
                        "conv group: bf16x6 members with 16-byte aligned split planes, Kpad % 32 == 0, no split-K");
        const bool qxf = q.in_scale || q.in_shift || q.in_relu, qut = q.Cin % BK6B == 0;
        const bool qp1 = q.lin_x && q.KH == 1 && q.KW == 1 && q.Cin % 4 == 0;
        EDGEDET_REQUIRE(qxf == xf && qut == ut && qp1 == p1, "conv group: members of one kernel variant");
        g.start[k] = (int)total;
        total += cdiv(q.M, BM) * cdiv(q.Cout, BN);
        EDGEDET_REQUIRE(total < (1ll << 31), "conv group grid too large");
    }
    g.start[g.n] = (int)total;
    auto k = p1 ? (xf ? (ut ? conv_x6b_group_kernel<true, true, BM, true, BN> : conv_x6b_group_kernel<true, false, BM, true, BN>)
                      : (ut ? conv_x6b_group_kernel<false, true, BM, true, BN> : conv_x6b_group_kernel<false, false, BM, true, BN>))
         : xf ? (ut ? conv_x6b_group_kernel<true, true, BM, false, BN> : conv_x6b_group_kernel<true, false, BM, false, BN>)
              : (ut ? conv_x6b_group_kernel<false, true, BM, false, BN> : conv_x6b_group_kernel<false, false, BM, false, BN>);
    hipLaunchKernelGGL(k, dim3((unsigned)total), dim3(512), 0, s, g);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// Device-side weight split (the same RN three-term split as plan.py split_bf16x3): w[n] fp32 ->
// out[3][n] bf16 planes.
__global__ void split_bf16x3_kernel(const float* __restrict__ w, int64_t n, int64_t kpad,
                                    unsigned short* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = (((i % kpad) >> 5) & 1) ? -w[i] : w[i];  // odd 32-wide K blocks negated
    const __bf16 x0 = (__bf16)x;
    const float r1 = x - (float)x0;
    const __bf16 x1 = (__bf16)r1;
    const __bf16 x2 = (__bf16)(r1 - (float)x1);
    out[i] = __builtin_bit_cast(unsigned short, x0);
    out[n + i] = __builtin_bit_cast(unsigned short, x1);
    out[2 * n + i] = __builtin_bit_cast(unsigned short, x2);
}

template <int WM, int WN, int TM, int TN>
static int launch_x6(const ConvParams& p, hipStream_t s) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    EDGEDET_REQUIRE(p.w3 && ((uintptr_t)p.w3 & 15) == 0, "conv bf16x6: needs 16-byte aligned split weight planes");
    EDGEDET_REQUIRE(p.Kpad % BK6 == 0, "conv bf16x6: Kpad must be a multiple of 16");
    const int64_t nwg = cdiv(p.M, BM) * cdiv(p.Cout, BN);
    EDGEDET_REQUIRE(nwg < (1ll << 31), "conv grid too large");
    const bool xf = p.in_scale || p.in_shift || p.in_relu, ut = (p.Cin & 15) == 0;
    auto k = xf ? (ut ? conv_x6_kernel<WM, WN, TM, TN, true, true> : conv_x6_kernel<WM, WN, TM, TN, true, false>)
                : (ut ? conv_x6_kernel<WM, WN, TM, TN, false, true> : conv_x6_kernel<WM, WN, TM, TN, false, false>);
    hipLaunchKernelGGL(k, dim3((unsigned)nwg), dim3(WM * WN * 64), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

template <int TM, int TN>
static int launch_pw(const ConvParams& p, hipStream_t s) {
    const int64_t waves = cdiv(p.M, 32 * TM) * cdiv(p.Cout, 32 * TN);
    EDGEDET_REQUIRE(waves < (1ll << 31), "pw conv grid too large");
    hipLaunchKernelGGL((pw_mfma_kernel<TM, TN>), dim3((unsigned)cdiv(waves, 4)), dim3(256), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

template <int TN, int NW = 4>
static int launch_pw_splitk(const ConvParams& p, hipStream_t s) {
    const int64_t nwg = cdiv(p.M, 32) * cdiv(p.Cout, 32 * TN);
    EDGEDET_REQUIRE(nwg < (1ll << 31), "pw conv grid too large");
    hipLaunchKernelGGL((pw_splitk_kernel<TN, NW>), dim3((unsigned)nwg), dim3(NW * 64), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// Tiles 33-35 (pw_stream_kernel): 1x1 dense input and output rows, Cin <= 72, Cout <= 96.
// 33: every column block in one wave (weights of NB x KJ <= 18 chunks in registers); 34: one
// column block per wave (column groups over the waves), next block prefetched; 35: 34 without the
// prefetch (more waves per SIMD instead).
static int pw_stream_max_wg() {  // grid cap: 512 - 4096 workgroups measured alike (profiles/r2j_pws_grid.txt)
    return 256 * 8;
}

template <int NB, int KJ, bool PF>
static int launch_pw_stream_nk(const ConvParams& p, hipStream_t s) {
    const int ncg = (p.Cout + 32 * NB - 1) / (32 * NB);
    const int64_t waves = cdiv(p.M, 32) * ncg;
    const unsigned g = (unsigned)std::min<int64_t>(cdiv(waves, 4), pw_stream_max_wg());
    const bool xf = p.in_scale || p.in_shift || p.in_relu;
    auto k = xf ? pw_stream_kernel<NB, KJ, true, PF> : pw_stream_kernel<NB, KJ, false, PF>;
    hipLaunchKernelGGL(k, dim3(g), dim3(256), 0, s, p, ncg);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

template <int NB, bool PF>
static int launch_pw_stream_n(const ConvParams& p, int kj, hipStream_t s) {
    switch (kj) {
        case 1: case 2: return launch_pw_stream_nk<NB, 2, PF>(p, s);
        case 3: return launch_pw_stream_nk<NB, 3, PF>(p, s);
        case 4: return launch_pw_stream_nk<NB, 4, PF>(p, s);
        case 5: return launch_pw_stream_nk<NB, 5, PF>(p, s);
        case 6: return launch_pw_stream_nk<NB, 6, PF>(p, s);
        case 7: case 8: if constexpr (NB <= 2) return launch_pw_stream_nk<NB, 8, PF>(p, s); break;
        case 9: if constexpr (NB <= 2) return launch_pw_stream_nk<NB, 9, PF>(p, s); break;
        default: break;
    }
    EDGEDET_REQUIRE(false, "pw_stream: Cin / Cout outside the register-resident weight shapes");
    return -1;
}

static int launch_pw_stream(const ConvParams& p, int tile, hipStream_t s) {
    EDGEDET_REQUIRE(p.lin_x && p.KH == 1 && p.KW == 1, "pw_stream needs a 1x1/stride-1 dense input");
    EDGEDET_REQUIRE(p.ksplit <= 1, "pw_stream: no split-K");
    EDGEDET_REQUIRE(p.lin_y && (!p.res || p.lin_res), "pw_stream: dense output and residual rows");
    const int kj = (p.Cin + 7) / 8, nb = (p.Cout + 31) / 32;
    EDGEDET_REQUIRE(nb >= 1 && nb <= 3 && kj <= 9, "pw_stream: Cout <= 96, Cin <= 72");
    if (tile == 34) return launch_pw_stream_n<1, true>(p, kj, s);
    if (tile == 35) return launch_pw_stream_n<1, false>(p, kj, s);
    EDGEDET_REQUIRE(nb * kj <= 18, "pw_stream tile 33: NB x KJ <= 18");
    if (nb == 1) return launch_pw_stream_n<1, true>(p, kj, s);
    if (nb == 2) return launch_pw_stream_n<2, true>(p, kj, s);
    return launch_pw_stream_n<3, true>(p, kj, s);
}

template <int WM, int WN, int TM, int TN>
static int launch_cfg(const ConvParams& p, hipStream_t s) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    const int64_t nwg = cdiv(p.M, BM) * cdiv(p.Cout, BN);
    EDGEDET_REQUIRE(nwg < (1ll << 31), "conv grid too large");
    hipLaunchKernelGGL((conv_mfma_kernel<WM, WN, TM, TN>), dim3((unsigned)nwg), dim3(WM * WN * 64), 0, s, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

// Tile choice: the direct pointwise kernel for narrow-K 1x1 layers (HBM-bound, no reuse to stage);
// otherwise the largest LDS-staged tile that still gives about one workgroup per CU.
static int choose_tile(const ConvParams& p) {
    if (p.lin_x && p.Kpad >= 256 && p.Cout <= 96) return p.Cout <= 32 ? 13 : (p.Cout <= 64 ? 14 : 13);
    if (p.lin_x && (p.Kpad <= 128 || p.Cout <= 32)) {
        if (p.Cout <= 32) return 15;
        const int64_t w22 = cdiv(p.M, 64) * cdiv(p.Cout, 64);
        return w22 >= 4 * 256 ? 10 : 12;
    }
    struct C { int tile, bm, bn; };
    const C cands_wide[] = {{3, 128, 128}, {2, 128, 64}, {5, 64, 64}, {6, 32, 32}};
    const C cands_mid[] = {{2, 128, 64}, {5, 64, 64}, {6, 32, 32}};
    const C cands_narrow[] = {{1, 128, 32}, {6, 32, 32}};
    const C* c = p.Cout > 64 ? cands_wide : (p.Cout > 32 ? cands_mid : cands_narrow);
    const int nc = p.Cout > 64 ? 4 : (p.Cout > 32 ? 3 : 2);
    for (int i = 0; i < nc; ++i)
        if (cdiv(p.M, c[i].bm) * cdiv(p.Cout, c[i].bn) >= 240) return c[i].tile;
    return c[nc - 1].tile;
}

// Validation and the derived fields (fast divisors, dense-layout flags) of a conv problem.
int conv_prepare(ConvParams& p) {
    EDGEDET_REQUIRE(p.x && p.w && p.bias && p.y, "conv: null x/w/bias/y");
    EDGEDET_REQUIRE(p.Cin % 4 == 0, "conv: Cin must be a multiple of 4 (pad channels)");
    EDGEDET_REQUIRE(p.x_pstride % 4 == 0, "conv: input pixel stride must be a multiple of 4");
    EDGEDET_REQUIRE(p.Kpad % BK == 0 && p.Kpad >= p.K, "conv: Kpad must be a multiple of 32 and >= K");
    EDGEDET_REQUIRE(p.M > 0 && p.Cout > 0, "conv: empty problem");
    EDGEDET_REQUIRE(((uintptr_t)p.x & 15) == 0 && ((uintptr_t)p.w & 15) == 0, "conv: x/w must be 16-byte aligned");
    EDGEDET_REQUIRE((int64_t)p.B * p.Ho * p.Wo < (1ll << 31), "conv: M overflows int32");
    p.div_howo = make_fastdiv((uint32_t)(p.Ho * p.Wo));
    p.div_wo = make_fastdiv((uint32_t)p.Wo);
    p.div_cin = make_fastdiv((uint32_t)p.Cin);
    p.div_kw = make_fastdiv((uint32_t)p.KW);
    if (p.res_H <= 0) p.res_H = p.Ho;
    if (p.res_W <= 0) p.res_W = p.Wo;
    p.res_sh = (float)p.res_H / (float)p.Ho;
    p.res_sw = (float)p.res_W / (float)p.Wo;
    p.lin_x = (p.KH == 1 && p.KW == 1 && p.stride == 1 && p.pad == 0 && p.Ho == p.H && p.Wo == p.W &&
               p.x_bstride == (int64_t)p.H * p.W * p.x_pstride) ? 1 : 0;
    p.lin_y = (p.y_bstride == (int64_t)p.Ho * p.Wo * p.y_pstride) ? 1 : 0;
    p.lin_res = (p.res_H == p.Ho && p.res_W == p.Wo && p.res_bstride == (int64_t)p.Ho * p.Wo * p.res_pstride) ? 1 : 0;
    return 0;
}

// The kernel variant that runs: the requested tile, or the automatic choice (compute-bound LDS
// tiles switch to their bf16x6 form when the split weight planes are present).
int conv_resolve_tile(const ConvParams& p, int tile) {
    if (tile <= 0) {
        tile = choose_tile(p);
        if (p.w3 && tile >= 2 && tile <= 4) {
            tile += 20;
            // large problems: the 32-deep-stage 256 x 128 tile (>= 2 workgroups per CU)
            if (tile >= 23 && cdiv(p.M, 256) * cdiv(p.Cout, 128) >= 512) tile = 25;
        }
    }
    return tile;
}

// Host launcher shared by the plan executor and the unit C entry point.
int conv_launch(ConvParams p, int tile, hipStream_t s) {
    const int rc = conv_prepare(p);
    if (rc) return rc;
    tile = conv_resolve_tile(p, tile);
    switch (tile) {
        case 21: return launch_x6<2, 2, 1, 1>(p, s);  // 64 x 64, bf16x6
        case 22: return launch_x6<2, 2, 2, 1>(p, s);  // 128 x 64, bf16x6
        case 23: return launch_x6<2, 2, 2, 2>(p, s);  // 128 x 128, bf16x6
        case 24: return launch_x6<4, 2, 2, 2>(p, s);  // 256 x 128, bf16x6
        case 25: return launch_x6b(p, s);             // 256 x 128, bf16x6, 32-deep swizzled stages
        case 27: return launch_x6<4, 2, 1, 1>(p, s);  // 128 x 64, bf16x6, 8 waves (32 x 32 each)
        case 28: return launch_x6<4, 2, 1, 2>(p, s);  // 128 x 128, bf16x6, 8 waves (32 x 64 each)
        case 29: return launch_x6b<128, 1>(p, s);     // 128 x 128, bf16x6, 32-deep swizzled stages, skewed pipeline
        case 30: return launch_x6b<128, 2>(p, s);     // the same, two register stages
        case 31: return launch_x6b<64, 1>(p, s);      // 64 x 128, bf16x6, two workgroups per CU
        case 32: return launch_x6b<64, 2>(p, s);      // the same, two register stages
        case 38: return launch_x6b<128, 1, 64>(p, s); // 128 x 64, bf16x6, 32-deep swizzled stages (Cout <= 64 layers)
        case 39: return launch_x6b<128, 1, 256>(p, s); // 128 x 256: the A panel read once per Cout = 256 layer
        case 26: {                                    // the same, K split in two halves (atomics into zeroed y)
            ConvParams q = p;
            q.ksplit = 2;
            return launch_x6b(q, s);
        }
        case 33:                                      // streaming 1x1, fp32 MFMA, weights in registers
        case 34:
        case 35: return launch_pw_stream(p, tile, s);
        case 1: return launch_cfg<4, 1, 1, 1>(p, s);  // 128 x 32
        case 2: return launch_cfg<2, 2, 2, 1>(p, s);  // 128 x 64
        case 3: return launch_cfg<2, 2, 2, 2>(p, s);  // 128 x 128
        case 4: return launch_cfg<4, 2, 2, 2>(p, s);  // 256 x 128
        case 5: return launch_cfg<2, 2, 1, 1>(p, s);  // 64 x 64
        case 6: return launch_cfg<1, 1, 1, 1>(p, s);  // 32 x 32 (one wave)
        case 10:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw<2, 2>(p, s);               // direct, 64 x 64 per wave
        case 11:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw<4, 1>(p, s);               // direct, 128 x 32 per wave
        case 12:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw<1, 2>(p, s);               // direct, 32 x 64 per wave
        case 15:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw<2, 1>(p, s);               // direct, 64 x 32 per wave
        case 13:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw_splitk<1>(p, s);           // split-K over 4 waves, 32 x 32
        case 16:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw_splitk<1, 8>(p, s);        // split-K over 8 waves, 32 x 32
        case 17:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw_splitk<2, 8>(p, s);        // split-K over 8 waves, 32 x 64
        case 14:
            EDGEDET_REQUIRE(p.lin_x, "pw tiles need a 1x1/stride-1 dense input");
            return launch_pw_splitk<2>(p, s);           // split-K over 4 waves, 32 x 64
        default: EDGEDET_REQUIRE(false, "conv: unknown tile config");
    }
}

// Grouped launch of up to EDGEDET_MAX_GROUP conv problems (exec.hip EDGEDET_OP_GROUP).  Every member
// must resolve to the same x6b tile (29 / 31 / 38 / 25, no pre-split input) and kernel variant; returns
// 1 without launching when they do not, and the caller then issues them one by one.
int conv_group_launch(const ConvParams* ps, int n, int tile, hipStream_t s) {
    EDGEDET_REQUIRE(n >= 1 && n <= EDGEDET_MAX_GROUP, "conv group: 1..EDGEDET_MAX_GROUP members");
    ConvGroup gl;  // about 3 KB, passed by value as the kernel's argument block
    gl.n = n;
    int t0 = -1;
    for (int k = 0; k < n; ++k) {
        gl.p[k] = ps[k];
        const int rc = conv_prepare(gl.p[k]);
        if (rc) return rc;
        const int t = conv_resolve_tile(gl.p[k], tile);
        if (k == 0) t0 = t;
        if (t != t0 || gl.p[k].x3) return 1;
    }
    switch (t0) {
        case 25: return launch_x6b_group<256, 128>(gl, s);
        case 29: return launch_x6b_group<128, 128>(gl, s);
        case 31: return launch_x6b_group<64, 128>(gl, s);
        case 38: return launch_x6b_group<128, 64>(gl, s);
        case 39: return launch_x6b_group<128, 256>(gl, s);
        default: return 1;
    }
}

}  // namespace edgedet

using namespace edgedet;

extern "C" int64_t edgedet_conv_weight_k(int32_t KH, int32_t KW, int64_t Cin) {
    return cdiv((int64_t)KH * KW * Cin, BK) * BK;
}

extern "C" int edgedet_split_bf16x3(const float* w, int64_t n, int64_t kpad, uint16_t* out, void* stream) {
    EDGEDET_REQUIRE(w && out && n > 0, "split_bf16x3: null pointer or empty");
    EDGEDET_REQUIRE(kpad > 0 && kpad % BK6B == 0 && n % kpad == 0, "split_bf16x3: rows of kpad, a multiple of 32");
    hipLaunchKernelGGL(split_bf16x3_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, w, n,
                       kpad, reinterpret_cast<unsigned short*>(out));
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

extern "C" int edgedet_conv2d_x3(const float* x, uint16_t* x3, int64_t B, int64_t H, int64_t W, int64_t Cin,
                                 const float* w, const uint16_t* w3, const float* bias, int64_t Cout, int32_t KH,
                                 int32_t KW, int32_t stride, int32_t pad, int32_t act, const float* res, float* y,
                                 int32_t tile, void* stream) {
    ConvParams p{};
    p.w3 = w3;
    p.x3 = x3;
    p.x = x;
    p.w = w;
    p.bias = bias;
    p.y = y;
    p.res = res;
    p.B = (int)B;
    p.H = (int)H;
    p.W = (int)W;
    p.Cin = (int)Cin;
    p.Cout = (int)Cout;
    p.KH = KH;
    p.KW = KW;
    p.stride = stride;
    p.pad = pad;
    p.act = act;
    p.Ho = (int)((H + 2 * pad - KH) / stride + 1);
    p.Wo = (int)((W + 2 * pad - KW) / stride + 1);
    p.K = (int)(KH * KW * Cin);
    p.Kpad = (int)edgedet_conv_weight_k(KH, KW, Cin);
    p.M = (int)(B * p.Ho * p.Wo);
    p.x_pstride = (int)Cin;
    p.x_bstride = H * W * Cin;
    p.y_pstride = (int)Cout;
    p.y_bstride = (int64_t)p.Ho * p.Wo * Cout;
    p.res_pstride = (int)Cout;
    p.res_bstride = p.y_bstride;
    return conv_launch(p, tile, (hipStream_t)stream);
}

extern "C" int edgedet_conv2d_ex(const float* x, int64_t B, int64_t H, int64_t W, int64_t Cin, const float* w,
                                 const uint16_t* w3, const float* bias, int64_t Cout, int32_t KH, int32_t KW,
                                 int32_t stride, int32_t pad, int32_t act, const float* res, float* y, int32_t tile,
                                 void* stream) {
    return edgedet_conv2d_x3(x, nullptr, B, H, W, Cin, w, w3, bias, Cout, KH, KW, stride, pad, act, res, y, tile,
                             stream);
}

extern "C" int edgedet_conv2d(const float* x, int64_t B, int64_t H, int64_t W, int64_t Cin, const float* w,
                              const float* bias, int64_t Cout, int32_t KH, int32_t KW, int32_t stride,
                              int32_t pad, int32_t act, const float* res, float* y, void* stream) {
    return edgedet_conv2d_ex(x, B, H, W, Cin, w, nullptr, bias, Cout, KH, KW, stride, pad, act, res, y, 0, stream);
}
