// ORIE (offloading reward) on the device: the consumer of the detection files.
//
// Replaces the CPU work of reward.py:16-52 (compute_orie) and lib/data.py:46-84 (set_data's
// box_correct), whose cost is N images x 2 (weak / strong) x ap_per_class over an E+1 image ensemble
// (lib/metrics.py:89-148): a sort of E x ~300 detections and a Python loop over the classes per call.
//
// box_correct_kernel  one workgroup per (image, detector): the TP flag of every detection at
//     IoU >= thr (lib/metrics.py:38-64).  The reference matches with argsort + two np.unique passes:
//     (1) every detection keeps its highest-IoU same-class label (ties: the larger label index, the
//     row-major order reversed by [::-1]); (2) every label keeps the smallest detection index among the
//     detections that chose it (np.unique over the det-sorted matches).  IoU in float64 with the
//     reference's op order (lib/metrics.py:67-86).
//
// orie_ap_kernel  one workgroup per (evaluation, class); an evaluation = (target image i, detector
//     v in {weak, strong}).  All detections of the dataset are pre-sorted per class by (conf desc,
//     image, row, weak-before-strong) once; a detection is a member of evaluation (i, v) iff its image
//     is in i's ensemble (weak detections), or it is image i's own detection of detector v.  The
//     member subsequence of a class segment is exactly the class's rows of the reference's
//     np.argsort(-conf) over the concatenated ensemble (the tie order between equal confidences is the
//     one place the reference is implementation-defined: quicksort; here it is the fixed order above).
//     Pass 1 counts members (n_p) and their TPs; pass 2 walks the segment backwards in chunks and,
//     per member k, forms tpc_k, precision tpc_k / k, recall tpc_k / (n_l + 1e-16), the precision
//     envelope (suffix max), and evaluates np.interp(linspace(0, 1, 101), mrec, mpre) on the grid
//     points whose bracketing index is k (lib/metrics.py:127-148, numpy's arr_interp with its
//     "x == xp[j]" and "last point" branches), then np.trapz with numpy's pairwise (8-accumulator)
//     summation order.  Every value is computed in float64 in the reference's operation order
//     (-ffp-contract=off), so AP values are bit-identical to the reference's.
#include "kernels.hpp"

namespace edgedet {

constexpr int ORIE_NT = 256;
constexpr int ORIE_GRID = 101;

struct OrieApParams {
    const int32_t* ent_img;   // [n_ent] image of each sorted entry
    const uint8_t* ent_flag;  // [n_ent] bit0 TP, bit1 strong-detector entry
    const int64_t* seg_off;   // [n_cls + 1] class segments of the sorted entries
    const int32_t* lab_cnt;   // [n_img][n_cls] ground-truth boxes per image and class
    const int32_t* target;    // [n_eval] target image of each evaluation
    const int32_t* ens;       // [n_eval][E] ensemble images (target excluded)
    const uint32_t* wmask;    // mask mode (test.py test_map): [n_eval][bitmap_words] images whose weak
    const uint32_t* smask;    //   / strong detections take part; null = ORIE mode (target + ensemble)
    double* ap;               // [n_eval][2][n_cls] (weak, strong)
    int32_t* n_l;             // [n_eval][n_cls] labels of the class in the ensemble + target
    int n_cls, E, n_img, bitmap_words;
    int64_t n_eval;
};

__device__ __forceinline__ double grid_x(int j) {  // np.linspace(0, 1, 101): j * (1.0 / 100), last = 1.0
    return j == ORIE_GRID - 1 ? 1.0 : (double)j * (1.0 / 100.0);
}

// Block-wide inclusive scan (sum) of one int per thread, in thread order; returns the total.
__device__ __forceinline__ int block_scan_incl(int v, int* sh, int& total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int pre = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < ORIE_NT / 64; ++k) {
        const int t = sh[k];
        if (k < w) pre += t;
        total += t;
    }
    __syncthreads();
    return x + pre;
}

__global__ void __launch_bounds__(ORIE_NT) orie_ap_kernel(OrieApParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* bitmap = smem;                                      // ensemble membership, n_img bits
    double* vals = reinterpret_cast<double*>(smem + ((2 * P.bitmap_words + 1) & ~1));  // [2][101]
    __shared__ int sh_int[8];
    __shared__ double sh_r[ORIE_NT + 1], sh_e[ORIE_NT + 1];
    __shared__ double sh_carry[2];

    const int tid = threadIdx.x;
    const int c = (int)(blockIdx.x % (unsigned)P.n_cls);
    const int64_t e = blockIdx.x / (unsigned)P.n_cls;
    const bool mask_mode = P.wmask != nullptr;
    const int img = mask_mode ? -1 : P.target[e];
    uint32_t* sbitmap = bitmap + P.bitmap_words;  // mask mode only (allocated by the launcher)

    int nl = 0;
    if (mask_mode) {
        const uint32_t* wm = P.wmask + e * P.bitmap_words;
        const uint32_t* sm = P.smask + e * P.bitmap_words;
        for (int w = tid; w < P.bitmap_words; w += ORIE_NT) {
            bitmap[w] = wm[w];
            sbitmap[w] = sm[w];
        }
        for (int im = tid; im < P.n_img; im += ORIE_NT)
            if (((wm[im >> 5] | sm[im >> 5]) >> (im & 31)) & 1u) nl += P.lab_cnt[(int64_t)im * P.n_cls + c];
        __syncthreads();
    } else {
        const int32_t* ens = P.ens + e * P.E;
        for (int w = tid; w < P.bitmap_words; w += ORIE_NT) bitmap[w] = 0u;
        __syncthreads();
        for (int s = tid; s < P.E; s += ORIE_NT) {
            const int im = ens[s];
            atomicOr(&bitmap[im >> 5], 1u << (im & 31));
            nl += P.lab_cnt[(int64_t)im * P.n_cls + c];
        }
    }
    // n_l = labels of class c over the evaluated images (reward.py:40-41 / test.py:56, np.unique counts)
    int tot;
    block_scan_incl(nl, sh_int, tot);
    const int n_l = tot + (mask_mode ? 0 : P.lab_cnt[(int64_t)img * P.n_cls + c]);
    if (tid == 0) P.n_l[e * P.n_cls + c] = n_l;
    __syncthreads();
    auto member = [&](int im, bool strong, int v) -> bool {
        if (mask_mode) return (((strong ? sbitmap : bitmap)[im >> 5] >> (im & 31)) & 1u) != 0;
        return strong ? (im == img && v == 1) : (((bitmap[im >> 5] >> (im & 31)) & 1u) || (im == img && v == 0));
    };

    const int64_t s0 = P.seg_off[c], s1 = P.seg_off[c + 1];
    for (int v = 0; v < (mask_mode ? 1 : 2); ++v) {
        double* out = P.ap + (e * 2 + v) * P.n_cls + c;
        // ---- pass 1: members and their TPs
        int np_ = 0, nt_ = 0;
        for (int64_t q = s0 + tid; q < s1; q += ORIE_NT) {
            const int f = P.ent_flag[q];
            const bool mem = member(P.ent_img[q], f & 2, v);
            np_ += mem;
            nt_ += mem && (f & 1);
        }
        int n_p, T;
        block_scan_incl(np_, sh_int, n_p);
        block_scan_incl(nt_, sh_int, T);
        if (n_l == 0 || n_p == 0) {  // ap stays 0 (lib/metrics.py:112-113)
            if (tid == 0) *out = 0.0;
            continue;
        }
        const double denom = (double)n_l + 1e-16;
        // ---- pass 2: backwards over chunks of ORIE_NT entries
        int after_m = 0, after_t = 0;   // members / TPs after the current chunk
        double r_next = 1.0, e_next = 0.0;  // mrec, envelope at the first member after the chunk
        double* val = vals + v * ORIE_GRID;
        const int64_t len = s1 - s0;
        const int64_t nchunks = (len + ORIE_NT - 1) / ORIE_NT;
        for (int64_t ch = nchunks - 1; ch >= 0; --ch) {
            const int64_t q = s0 + ch * ORIE_NT + tid;
            bool mem = false, tp = false;
            if (q < s1) {
                const int f = P.ent_flag[q];
                mem = member(P.ent_img[q], f & 2, v);
                tp = mem && (f & 1);
            }
            int cm, ct;
            const int im_incl = block_scan_incl(mem ? 1 : 0, sh_int, cm);
            const int it_incl = block_scan_incl(tp ? 1 : 0, sh_int, ct);
            if (cm == 0) continue;  // uniform
            // member rank within the chunk (0-based, forward order) and k, tpc of each member
            const int rk = im_incl - 1;
            const int mem_after_in = cm - im_incl;     // members strictly after, within the chunk
            const int tp_after_in = ct - it_incl;
            double pk = 0.0, rrk = 0.0;
            if (mem) {
                const long long k = (long long)n_p - after_m - mem_after_in;
                const long long tpc = (long long)T - after_t - tp_after_in;
                pk = (double)tpc / (double)k;  // precision = tpc / (tpc + fpc)
                rrk = (double)tpc / denom;     // recall = tpc / (n_l + eps)
                sh_r[rk] = rrk;
                sh_e[rk] = pk;
            }
            if (tid == 0) {
                sh_r[cm] = r_next;
                sh_e[cm] = e_next;
            }
            __syncthreads();
            // envelope: suffix max over the chunk's members (+ the carry), serial over <= 256 values
            if (tid == 0) {
                double m = e_next;
                for (int t = cm - 1; t >= 0; --t) {
                    m = sh_e[t] > m ? sh_e[t] : m;  // np.maximum
                    sh_e[t] = m;
                }
            }
            __syncthreads();
            if (mem) {
                // grid points x_j with r_k <= x_j < r_{k+1} are bracketed by member k
                const double rk1 = sh_r[rk + 1], ek = sh_e[rk], ek1 = sh_e[rk + 1];
                if (rk1 > rrk) {
                    int j = (int)floor(rrk * 100.0) - 1;
                    if (j < 0) j = 0;
                    while (j < ORIE_GRID && grid_x(j) < rrk) ++j;
                    const double slope = (ek1 - ek) / (rk1 - rrk);
                    for (; j < ORIE_GRID && grid_x(j) < rk1; ++j) {
                        const double x = grid_x(j);
                        val[j] = (x == rrk) ? ek : slope * (x - rrk) + ek;
                    }
                }
            }
            __syncthreads();
            if (tid == 0) {
                r_next = sh_r[0];
                e_next = sh_e[0];
                sh_carry[0] = r_next;
                sh_carry[1] = e_next;
            }
            after_m += cm;
            after_t += ct;
            __syncthreads();
            r_next = sh_carry[0];
            e_next = sh_carry[1];
        }
        // mrec[0] = 0, mpre_env[0] = 1 (max(1, ...)): grid points below r_1, and the last grid point
        // (x = 1.0 = mrec[-1]: numpy returns mpre[-1] = 0)
        if (tid == 0) {
            const double r1 = r_next, e1 = e_next;
            const double slope = (e1 - 1.0) / (r1 - 0.0);
            for (int j = 0; j < ORIE_GRID && grid_x(j) < r1; ++j) {
                const double x = grid_x(j);
                val[j] = (x == 0.0) ? 1.0 : slope * (x - 0.0) + 1.0;
            }
            val[ORIE_GRID - 1] = 0.0;
            // np.trapz(y, x) = (d * (y[1:] + y[:-1]) / 2.0).sum(): numpy's pairwise sum of the 100
            // terms (n <= 128: eight running sums over the first 96, a fixed tree, then the rest).
            constexpr int NTERM = ORIE_GRID - 1, NBLK = NTERM - NTERM % 8;
            double r[8];
            double res = 0.0;
            for (int k = 0; k < NTERM; ++k) {
                const double term = (grid_x(k + 1) - grid_x(k)) * (val[k + 1] + val[k]) / 2.0;
                if (k < 8) {
                    r[k] = term;
                } else if (k < NBLK) {
                    r[k & 7] += term;
                } else {
                    if (k == NBLK) res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                    res += term;
                }
            }
            *out = res;
        }
        __syncthreads();
    }
}

struct BoxCorrectParams {
    const double* det;      // [n_det][4] xyxy
    const int32_t* det_cls;
    const int64_t* det_off; // [n_img + 1]
    const double* lab;      // [n_lab][4] xyxy
    const int32_t* lab_cls;
    const int64_t* lab_off; // [n_img + 1]
    double thr;
    uint8_t* tp;            // [n_det]
};

// Labels are processed in chunks of BC_CHUNK (the per-label LDS slots): every chunk recomputes each
// detection's best label over ALL labels and keeps only the choices that fall in the chunk, so any
// label count works (lib/metrics.py has no limit); one chunk (<= 1024 labels) is the common case.
constexpr int BC_CHUNK = 1024;

__global__ void __launch_bounds__(256) box_correct_kernel(BoxCorrectParams P) {
    __shared__ int best_det[BC_CHUNK];  // per label of the chunk: smallest detection index that chose it
    const int im = blockIdx.x;
    const int64_t d0 = P.det_off[im], d1 = P.det_off[im + 1];
    const int64_t l0 = P.lab_off[im], l1 = P.lab_off[im + 1];
    const int nd = (int)(d1 - d0), nl = (int)(l1 - l0);
    for (int d = threadIdx.x; d < nd; d += blockDim.x) P.tp[d0 + d] = 0;
    if (nl == 0 || nd == 0) return;
    for (int c0 = 0; c0 < nl; c0 += BC_CHUNK) {
        const int cn = nl - c0 < BC_CHUNK ? nl - c0 : BC_CHUNK;
        __syncthreads();  // the previous chunk's TP writes have read best_det
        for (int l = threadIdx.x; l < cn; l += blockDim.x) best_det[l] = 0x7fffffff;
        __syncthreads();
        for (int d = threadIdx.x; d < nd; d += blockDim.x) {
            const double* b2 = P.det + (d0 + d) * 4;
            const int dc = P.det_cls[d0 + d];
            const double a2 = (b2[2] - b2[0]) * (b2[3] - b2[1]);
            double best = -1.0;
            int bl = -1;
            for (int l = 0; l < nl; ++l) {
                if (P.lab_cls[l0 + l] != dc) continue;
                const double* b1 = P.lab + (l0 + l) * 4;
                const double x1 = fmax(b1[0], b2[0]), y1 = fmax(b1[1], b2[1]);
                const double x2 = fmin(b1[2], b2[2]), y2 = fmin(b1[3], b2[3]);
                const double inter = fmax(0.0, x2 - x1) * fmax(0.0, y2 - y1);
                const double a1 = (b1[2] - b1[0]) * (b1[3] - b1[1]);
                const double iou = inter / (a1 + a2 - inter);
                if (iou >= P.thr && iou >= best) {  // ties -> the larger label index
                    best = iou;
                    bl = l;
                }
            }
            if (bl >= c0 && bl < c0 + cn) atomicMin(&best_det[bl - c0], d);
        }
        __syncthreads();
        for (int l = threadIdx.x; l < cn; l += blockDim.x)
            if (best_det[l] != 0x7fffffff) P.tp[d0 + best_det[l]] = 1;
    }
}

// lib/data.py:127-160 extract_output_feature for many images: the top-k rows (file order = score
// order) of each image's detection file -> [num_class + (ncol - 1) * k] float64: per-class counts of the
// k rows, then the rows' remaining columns flattened.  One thread per image.
__global__ void output_feature_kernel(const double* __restrict__ rows, const int64_t* __restrict__ off, int n_img,
                                      int ncol, int num_class, int k, double* __restrict__ out) {
    const int im = blockIdx.x * blockDim.x + threadIdx.x;
    if (im >= n_img) return;
    const int width = num_class + (ncol - 1) * k;
    double* f = out + (int64_t)im * width;
    for (int j = 0; j < width; ++j) f[j] = 0.0;
    const int64_t r0 = off[im];
    int nr = (int)(off[im + 1] - r0);
    nr = nr < k ? nr : k;
    for (int r = 0; r < nr; ++r) {
        const double* row = rows + (r0 + r) * ncol;
        const int c = (int)row[0];  // int(data[0]): truncation
        if (c >= 0 && c < num_class) f[c] += 1.0;
        for (int q = 1; q < ncol; ++q) f[num_class + r * (ncol - 1) + (q - 1)] = row[q];
    }
}

}  // namespace edgedet

using namespace edgedet;

extern "C" int edgedet_box_correct(const double* det_xyxy, const int32_t* det_cls, const int64_t* det_off,
                                   const double* lab_xyxy, const int32_t* lab_cls, const int64_t* lab_off,
                                   int64_t n_img, double iou_thr, uint8_t* tp, int64_t max_labels, void* stream) {
    (void)max_labels;  // any count: the kernel matches labels in 1024-label chunks
    EDGEDET_REQUIRE(det_off && lab_off && tp, "box_correct: null pointer");
    EDGEDET_REQUIRE(n_img >= 0 && n_img < (1ll << 31), "box_correct: bad image count");
    if (n_img == 0) return 0;
    BoxCorrectParams P{det_xyxy, det_cls, det_off, lab_xyxy, lab_cls, lab_off, iou_thr, tp};
    hipLaunchKernelGGL(box_correct_kernel, dim3((unsigned)n_img), dim3(256), 0, (hipStream_t)stream, P);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

static int ap_launch(const int32_t* ent_img, const uint8_t* ent_flag, const int64_t* seg_off, int32_t n_cls,
                     const int32_t* lab_cnt, int64_t n_img, const int32_t* target, const int32_t* ens, int32_t E,
                     const uint32_t* wmask, const uint32_t* smask, int64_t n_eval, double* ap, int32_t* n_l,
                     void* stream) {
    EDGEDET_REQUIRE(seg_off && lab_cnt && ap && n_l, "orie_ap: null pointer");
    EDGEDET_REQUIRE(n_cls > 0 && n_img > 0 && E >= 0, "orie_ap: bad sizes");
    EDGEDET_REQUIRE(n_img <= (1 << 20), "orie_ap: more than 2^20 images (membership bitmap)");
    EDGEDET_REQUIRE(n_eval * n_cls < (1ll << 31), "orie_ap: grid too large");
    if (n_eval == 0) return 0;
    OrieApParams P{};
    P.ent_img = ent_img;
    P.ent_flag = ent_flag;
    P.seg_off = seg_off;
    P.lab_cnt = lab_cnt;
    P.target = target;
    P.ens = ens;
    P.wmask = wmask;
    P.smask = smask;
    P.ap = ap;
    P.n_l = n_l;
    P.n_cls = n_cls;
    P.E = E;
    P.n_img = (int)n_img;
    P.bitmap_words = (int)((n_img + 31) / 32);
    P.n_eval = n_eval;
    const size_t shm = (size_t)((2 * P.bitmap_words + 1) & ~1) * 4 + 2 * ORIE_GRID * sizeof(double);
    EDGEDET_REQUIRE(shm <= 150 * 1024, "orie_ap: membership bitmap too large for LDS");
    hipLaunchKernelGGL(orie_ap_kernel, dim3((unsigned)(n_eval * n_cls)), dim3(ORIE_NT), shm, (hipStream_t)stream, P);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

extern "C" int edgedet_orie_ap(const int32_t* ent_img, const uint8_t* ent_flag, const int64_t* seg_off,
                               int32_t n_cls, const int32_t* lab_cnt, int64_t n_img, const int32_t* target,
                               const int32_t* ens, int32_t E, int64_t n_eval, double* ap, int32_t* n_l,
                               void* stream) {
    EDGEDET_REQUIRE(target && (E == 0 || ens), "orie_ap: null target / ensemble");
    return ap_launch(ent_img, ent_flag, seg_off, n_cls, lab_cnt, n_img, target, ens, E, nullptr, nullptr, n_eval, ap,
                     n_l, stream);
}

extern "C" int edgedet_map_eval(const int32_t* ent_img, const uint8_t* ent_flag, const int64_t* seg_off,
                                int32_t n_cls, const int32_t* lab_cnt, int64_t n_img, const uint32_t* weak_mask,
                                const uint32_t* strong_mask, int64_t n_eval, double* ap, int32_t* n_l, void* stream) {
    EDGEDET_REQUIRE(weak_mask && strong_mask, "map_eval: null membership masks");
    return ap_launch(ent_img, ent_flag, seg_off, n_cls, lab_cnt, n_img, nullptr, nullptr, 0, weak_mask, strong_mask,
                     n_eval, ap, n_l, stream);
}

extern "C" int edgedet_output_features(const double* rows, const int64_t* off, int64_t n_img, int32_t ncol,
                                       int32_t num_class, int32_t k, double* out, void* stream) {
    EDGEDET_REQUIRE(off && out && n_img >= 0 && ncol >= 1 && num_class > 0 && k >= 0, "output_features: bad args");
    if (n_img == 0) return 0;
    hipLaunchKernelGGL(output_feature_kernel, dim3((unsigned)cdiv(n_img, 64)), dim3(64), 0, (hipStream_t)stream, rows,
                       off, (int)n_img, ncol, num_class, k, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}
