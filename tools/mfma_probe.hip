// Rounding behaviour of the gfx950 matrix instructions (diagnostic, not product code).
//
// One wave per launch.  Every A row holds the same K values, every B entry is 1.0, so each output
// element is C + sum_k A[k]: the experiments place a 1.0 and a few small exact values at chosen
// (lane group, element) positions of the A fragment and read back C' - 1 in units of 2^-24 (half an
// ulp of 1.0 from above):
//   c_rne_pos   C = 1, one product +1.5 * 2^-24    : RNE -> +2, truncation -> 0
//   c_rne_neg   C = 1, one product -1.2 * 2^-24    : RNE -> -1, toward zero / -inf -> -2
//   in_group    C = 0, 1.0 and seven 2^-25 in the SAME lane's fragment:  exact 1 + 1.75 ulp -> RNE +4,
//               each product aligned to the group's largest and truncated -> 0
//   cross_group C = 0, 1.0 in lane group 0, +1.5 * 2^-24 in another lane group of the same k step:
//               exact then RNE -> +2, truncated -> 0
//   many_small  C = 0, 1.0 and 31 (or K-1) copies of 2^-25 spread over all positions
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mfma_probe.hip -o tools/libmfma_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { EXP_C_POS = 0, EXP_C_NEG, EXP_IN_GROUP, EXP_CROSS, EXP_MANY, NEXP };

// value of A at (lane group g, element e) for experiment x; KG = elements per lane, G = lane groups
__device__ float a_value(int x, int g, int e, int KG) {
    const float t = 0x1p-25f;
    switch (x) {
        case EXP_C_POS: return (g == 0 && e == 0) ? 0x1.8p-24f : 0.f;
        case EXP_C_NEG: return (g == 0 && e == 0) ? -0x1.333334p-24f : 0.f;
        case EXP_IN_GROUP: return (g == 0 && e == 0) ? 1.f : (g == 0 && e < 8 && e < KG ? t : 0.f);
        case EXP_CROSS: return (g == 0 && e == 0) ? 1.f : (g == 1 && e == 0 ? 0x1.8p-24f : 0.f);
        default: return (g == 0 && e == 0) ? 1.f : t;
    }
}
__device__ float c_value(int x) { return (x == EXP_C_POS || x == EXP_C_NEG) ? 1.f : 0.f; }

// kind: 0 16x16x32 bf16, 1 32x32x16 bf16, 2 16x16x16 bf16_1k, 3 32x32x8 bf16_1k, 4 16x16x32 f16,
//       5 16x16x4 f32, 6 32x32x2 f32
__global__ void probe_kernel(int kind, float* out) {
    const int lane = threadIdx.x;
    for (int x = 0; x < NEXP; ++x) {
        float r = 0.f;
        if (kind == 0 || kind == 4) {  // lane l: row l % 16, k = 8 (l / 16) + e
            const int g = lane / 16;
            if (kind == 0) {
                bf16x8 a, b;
                for (int e = 0; e < 8; ++e) { a[e] = (__bf16)a_value(x, g, e, 8); b[e] = (__bf16)1.f; }
                f32x4 c = {c_value(x), c_value(x), c_value(x), c_value(x)};
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
                r = c[0];
            } else {
                f16x8 a, b;
                for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(x == EXP_C_POS || x == EXP_C_NEG || x == EXP_CROSS ? 0.f : a_value(x, g, e, 8)); b[e] = (_Float16)1.f; }
                // f16 cannot hold 2^-25 next to 1.0 in one element range: only the group experiments with
                // representable values are meaningful (2^-25 is a normal f16? no: f16 min normal 2^-14)
                f32x4 c = {c_value(x), c_value(x), c_value(x), c_value(x)};
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
                r = c[0];
            }
        } else if (kind == 1) {  // lane l: row l % 32, k = 8 (l / 32) + e
            const int g = lane / 32;
            bf16x8 a, b;
            for (int e = 0; e < 8; ++e) { a[e] = (__bf16)a_value(x, g, e, 8); b[e] = (__bf16)1.f; }
            f32x16 c;
            for (int i = 0; i < 16; ++i) c[i] = c_value(x);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
            r = c[0];
        } else if (kind == 2) {  // lane l: row l % 16, k = 4 (l / 16) + e
            const int g = lane / 16;
            bf16x4 a, b;
            for (int e = 0; e < 4; ++e) { a[e] = (__bf16)a_value(x, g, e, 4); b[e] = (__bf16)1.f; }
            f32x4 c = {c_value(x), c_value(x), c_value(x), c_value(x)};
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(short __attribute__((ext_vector_type(4))), a),
                                                           __builtin_bit_cast(short __attribute__((ext_vector_type(4))), b), c, 0, 0, 0);
            r = c[0];
        } else if (kind == 3) {  // lane l: row l % 32, k = 4 (l / 32) + e
            const int g = lane / 32;
            bf16x4 a, b;
            for (int e = 0; e < 4; ++e) { a[e] = (__bf16)a_value(x, g, e, 4); b[e] = (__bf16)1.f; }
            f32x16 c;
            for (int i = 0; i < 16; ++i) c[i] = c_value(x);
            c = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(__builtin_bit_cast(short __attribute__((ext_vector_type(4))), a),
                                                          __builtin_bit_cast(short __attribute__((ext_vector_type(4))), b), c, 0, 0, 0);
            r = c[0];
        } else if (kind == 5) {  // lane l: row l % 16, k = l / 16
            const int g = lane / 16;
            f32x4 c = {c_value(x), c_value(x), c_value(x), c_value(x)};
            c = __builtin_amdgcn_mfma_f32_16x16x4f32(a_value(x, g, 0, 1), 1.f, c, 0, 0, 0);
            r = c[0];
        } else {  // lane l: row l % 32, k = l / 32
            const int g = lane / 32;
            f32x16 c;
            for (int i = 0; i < 16; ++i) c[i] = c_value(x);
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(a_value(x, g, 0, 1), 1.f, c, 0, 0, 0);
            r = c[0];
        }
        if (lane == 0) out[x] = r;
    }
}

extern "C" int mfma_probe(int kind, float* out_host) {
    float* d = nullptr;
    if (hipMalloc(&d, NEXP * sizeof(float)) != hipSuccess) return -1;
    hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, 0, kind, d);
    const hipError_t e = hipMemcpy(out_host, d, NEXP * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? 0 : -2;
}
