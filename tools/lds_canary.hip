// LDS canary (diagnostic for the round-4 table nondeterminism; not product code).
//
// Hypothesis under test: an LDS-DMA load (global_load_lds, used by the bf16x6 conv tiles to stage
// their weight planes, csrc/conv.hip conv_x6b_body) of one workgroup can write LDS outside that
// workgroup's allocation, i.e. into the LDS of a workgroup of ANOTHER kernel resident on the same CU.
// A kernel whose LDS holds long-lived state (the round-4 3 x 256 normalisation table, filled once and
// read for the whole tile) would then read corrupted values whenever it co-runs with such a kernel:
// results that depend on timing, as measured (profiles/r4k_lut_race.txt).
//
// canary_kernel: every workgroup fills `words` words of LDS with a pattern derived from its id, then
// re-reads the whole array `iters` times (with short sleeps, so it stays resident while other kernels
// run beside it), counting and repairing every word that changed; the count goes to bad[0] (a vector
// global atomic), the first corrupt value and word index to bad[1], bad[2].
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/lds_canary.hip -o tools/liblds_canary.so
#include <hip/hip_runtime.h>

#include <cstdint>

__global__ void __launch_bounds__(256) canary_kernel(unsigned* bad, int iters, int words) {
    extern __shared__ unsigned s[];
    const unsigned tag = (blockIdx.x + 1u) * 2654435761u;
    for (int i = threadIdx.x; i < words; i += blockDim.x) s[i] = tag ^ (unsigned)i;
    __syncthreads();
    unsigned nbad = 0, first = 0, where = 0;
    for (int it = 0; it < iters; ++it) {
        for (int i = threadIdx.x; i < words; i += blockDim.x) {
            const unsigned v = s[i];
            if (v != (tag ^ (unsigned)i)) {
                if (!nbad) {
                    first = v;
                    where = (unsigned)i;
                }
                ++nbad;
                s[i] = tag ^ (unsigned)i;
            }
        }
        __builtin_amdgcn_s_sleep(4);
    }
    if (nbad) {
        atomicAdd(bad, nbad);
        atomicExch(bad + 1, first);
        atomicExch(bad + 2, where);
    }
}

extern "C" int lds_canary_launch(unsigned* bad, int grid, int iters, int words, void* stream) {
    hipLaunchKernelGGL(canary_kernel, dim3(grid), dim3(256), (size_t)words * 4, (hipStream_t)stream, bad, iters,
                       words);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
