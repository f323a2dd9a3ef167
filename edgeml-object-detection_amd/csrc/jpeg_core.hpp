// Baseline-JPEG pixel reconstruction, shared by the gfx950 kernels (csrc/jpeg.hip) and the host
// checker entry (edgedet_jpeg_reconstruct_host): integer arithmetic only, so device and host results
// are identical, and identical to the decoder the reference reads images with.
//
// The reference decodes with torchvision.io.read_image(path, ImageReadMode.RGB) (detect.py:57, libjpeg);
// this build's host decoder is PIL's libjpeg-turbo, and both run libjpeg's default decompression
// path, restated here:
//   * dequantisation and the "islow" integer IDCT (jidctint.c jpeg_idct_islow: CONST_BITS 13,
//     PASS1_BITS 2, the twelve FIX_* constants, DESCALE = round-half-up arithmetic shift), output
//     through the post-IDCT range-limit table (x & 1023 -> clamp(x + 128), wrapping beyond +-512);
//   * "fancy" (triangular) chroma upsampling (jdsample.c h2v2_fancy_upsample / h2v1_fancy_upsample,
//     with the edge columns and rows replicated and the +8/+7 and +1/+2 rounding biases);
//   * YCbCr -> RGB (jdcolor.c ycc_rgb_convert: SCALEBITS 16 fixed-point tables, clamp to 0..255).
// Grayscale images become RGB by replication (PIL's convert("RGB") of an "L" image).
#pragma once
#include <cstdint>

#ifndef EDGEDET_HD
#define EDGEDET_HD __host__ __device__ __forceinline__
#endif

namespace edgedet {
namespace jpeg {

// natural (row-major) index of the k-th coefficient in zig-zag order (jutils.c jpeg_natural_order)
constexpr int kNatural[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                              41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                              30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int32_t FIX_0_298631336 = 2446, FIX_0_390180644 = 3196, FIX_0_541196100 = 4433, FIX_0_765366865 = 6270,
                  FIX_0_899976223 = 7373, FIX_1_175875602 = 9633, FIX_1_501321110 = 12299, FIX_1_847759065 = 15137,
                  FIX_1_961570560 = 16069, FIX_2_053119869 = 16819, FIX_2_562915447 = 20995, FIX_3_072711026 = 25172;

EDGEDET_HD int32_t descale(int32_t x, int n) { return (x + (1 << (n - 1))) >> n; }

// jdmaster.c prepare_range_limit_table as used by the IDCT (IDCT_range_limit = table + CENTERJSAMPLE):
// index x & 1023 of the descaled output x
EDGEDET_HD uint8_t idct_limit(int32_t x) {
    const int i = x & 1023;
    if (i < 128) return (uint8_t)(i + 128);
    if (i < 512) return 255;
    if (i < 896) return 0;
    return (uint8_t)(i - 896);
}

// One 1-D pass of jpeg_idct_islow on eight inputs in[0..7] (already dequantised in pass 1).  Returns
// the eight outputs before their final descale: out[j] for j in 0..7 as the sums tmp10 + tmp3 ... in
// the reference's output order.
EDGEDET_HD void idct_1d(const int32_t in[8], int32_t out[8]) {
    int32_t z2 = in[2], z3 = in[6];
    int32_t z1 = (z2 + z3) * FIX_0_541196100;
    const int32_t tmp2e = z1 + z3 * (-FIX_1_847759065);
    const int32_t tmp3e = z1 + z2 * FIX_0_765366865;
    const int32_t tmp0e = (in[0] + in[4]) * (1 << CONST_BITS);
    const int32_t tmp1e = (in[0] - in[4]) * (1 << CONST_BITS);
    const int32_t tmp10 = tmp0e + tmp3e, tmp13 = tmp0e - tmp3e, tmp11 = tmp1e + tmp2e, tmp12 = tmp1e - tmp2e;
    int32_t tmp0 = in[7], tmp1 = in[5], tmp2 = in[3], tmp3 = in[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int32_t z4 = tmp1 + tmp3;
    const int32_t z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 = tmp0 * FIX_0_298631336;
    tmp1 = tmp1 * FIX_2_053119869;
    tmp2 = tmp2 * FIX_3_072711026;
    tmp3 = tmp3 * FIX_1_501321110;
    z1 = z1 * (-FIX_0_899976223);
    z2 = z2 * (-FIX_2_562915447);
    z3 = z3 * (-FIX_1_961570560) + z5;
    z4 = z4 * (-FIX_0_390180644) + z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    out[0] = tmp10 + tmp3;
    out[7] = tmp10 - tmp3;
    out[1] = tmp11 + tmp2;
    out[6] = tmp11 - tmp2;
    out[2] = tmp12 + tmp1;
    out[5] = tmp12 - tmp1;
    out[3] = tmp13 + tmp0;
    out[4] = tmp13 - tmp0;
}

// Pass 1 (a column of dequantised coefficients c[0..7], top to bottom) -> work values.  The all-AC-zero
// shortcut of the reference (dc << PASS1_BITS) equals the full computation, so it is not special-cased.
EDGEDET_HD void idct_col(const int32_t c[8], int32_t w[8]) {
    int32_t o[8];
    idct_1d(c, o);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = descale(o[j], CONST_BITS - PASS1_BITS);
}

// Pass 2 (a row of work values) -> eight samples.
EDGEDET_HD void idct_row(const int32_t w[8], uint8_t s[8]) {
    int32_t o[8];
    idct_1d(w, o);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = idct_limit(descale(o[j], CONST_BITS + PASS1_BITS + 3));
}

// jdcolor.c build_ycc_rgb_table entries (SCALEBITS 16, ONE_HALF 1 << 15, FIX(x) = x * 65536 + 0.5)
constexpr int32_t FIX_1_40200 = 91881, FIX_1_77200 = 116130, FIX_0_71414 = 46802, FIX_0_34414 = 22554;
EDGEDET_HD uint8_t clamp255(int32_t v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
EDGEDET_HD void ycc_rgb(int32_t y, int32_t cb, int32_t cr, uint8_t& r, uint8_t& g, uint8_t& b) {
    const int32_t xcr = cr - 128, xcb = cb - 128;
    const int32_t crr = (FIX_1_40200 * xcr + (1 << 15)) >> 16;
    const int32_t cbb = (FIX_1_77200 * xcb + (1 << 15)) >> 16;
    const int32_t crg = -FIX_0_71414 * xcr;
    const int32_t cbg = -FIX_0_34414 * xcb + (1 << 15);
    r = clamp255(y + crr);
    g = clamp255(y + ((cbg + crg) >> 16));
    b = clamp255(y + cbb);
}

// Horizontal fancy upsampling of one chroma row (jdsample.c h2v1 / the horizontal half of h2v2):
// the output sample at x from "column sums" cs(c) of the downsampled row (width cw), with
// (weight 3, edge / neighbour) and the reference's bias pair (b_even, b_odd) and shift.
//   h2v2: cs(c) = 3 * row0[c] + row1[c]; even x: (3 cs(c) + cs(c-1) + 8) >> 4, first column
//         (4 cs(0) + 8) >> 4; odd x: (3 cs(c) + cs(c+1) + 7) >> 4, last column (4 cs(cw-1) + 7) >> 4.
//   h2v1: cs(c) = row[c];  even x: (3 cs(c) + cs(c-1) + 1) >> 2, first column cs(0);
//         odd x: (3 cs(c) + cs(c+1) + 2) >> 2, last column cs(cw-1).

}  // namespace jpeg
}  // namespace edgedet
