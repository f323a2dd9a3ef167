// ORIE estimator training on the device (BASELINE config 5).
//
// Replaces regression.py:242-355 (fit_CNN) for the stage-24 features (lib/data.py:127-160, the
// "output features" of the weak detector's detection file): lib/nn_model.py:28-112 EdgeDetectionNet
// with no conv layers, i.e. an MLP d0 -> d1 -> ... -> 1 whose hidden layers are
// Linear -> BatchNorm1d -> ReLU -> Dropout(p) and whose last layer is a plain Linear, trained with
// MSELoss (or the reward-weighted loss), Adam(lr, weight_decay) and MultiStepLR(milestones, gamma),
// batch 64 in dataset order (the reference's DataLoader has no shuffle), testing on the validation
// fold after every epoch and keeping the best model (lowest test loss) and the last one.
//
// mlp_fit_kernel: one workgroup per cross-validation fold runs the whole training (every epoch,
//     batch, forward, backward, Adam step and test pass) with the parameters and gradients in LDS;
//     Adam's moments live in a global scratch.  Every reduction is a fixed-order loop, so a fit is
//     deterministic; dropout masks come from a counter-based hash of (seed, fold, step, layer, unit).
//     Arithmetic follows ATen's CPU order: BatchNorm1d train forward with the biased batch variance
//     and the unbiased one for the running estimate (momentum 0.1, eps 1e-5), BatchNorm backward
//     (dy - mean(dy) - xhat * mean(dy * xhat)) * gamma * invstd, Adam's lerp / addcmul / addcdiv
//     with the bias corrections in double.
// mlp_predict_kernel: eval-mode forward (running statistics, no dropout), one thread per row.
#include "kernels.hpp"

namespace edgedet {

constexpr int MLP_NT = 256;
constexpr int MLP_MAXL = 8;    // linear layers
constexpr int MLP_MAXH = 64;   // hidden width
constexpr int MLP_MAXB = 64;   // batch
constexpr int MLP_MAXD0 = 1024;

struct MlpLayout {
    int L, d[MLP_MAXL + 1];
    int w[MLP_MAXL], b[MLP_MAXL], g[MLP_MAXL], be[MLP_MAXL], rm[MLP_MAXL], rv[MLP_MAXL];
    int np, ns;  // trainable parameters, full state (+ running statistics)
};

// State vector: for each layer l, W_l [d_{l+1}][d_l], b_l [d_{l+1}], and for hidden layers gamma_l,
// beta_l [d_{l+1}]; then the running mean / var of every hidden layer (edgeml_amd/estimator.py
// MlpSpec builds the same layout).
static MlpLayout mlp_layout(int L, const int* dims) {
    MlpLayout m{};
    m.L = L;
    for (int l = 0; l <= L; ++l) m.d[l] = dims[l];
    int o = 0;
    for (int l = 0; l < L; ++l) {
        m.w[l] = o;
        o += m.d[l + 1] * m.d[l];
        m.b[l] = o;
        o += m.d[l + 1];
        if (l < L - 1) {
            m.g[l] = o;
            o += m.d[l + 1];
            m.be[l] = o;
            o += m.d[l + 1];
        }
    }
    m.np = o;
    for (int l = 0; l < L - 1; ++l) {
        m.rm[l] = o;
        o += m.d[l + 1];
        m.rv[l] = o;
        o += m.d[l + 1];
    }
    m.ns = o;
    return m;
}

struct MlpFitParams {
    const float* x;  // [N][D0]
    const float* y;  // [F][N] per-fold targets
    const int32_t* tr_idx;
    const int64_t* tr_off;  // [F + 1]
    const int32_t* va_idx;
    const int64_t* va_off;
    const float* init;  // [F][ns]
    float* best;        // [F][ns]
    float* last;        // [F][ns]
    float* adam;        // [F][2 np]
    float* train_loss;  // [F][epochs]
    float* test_loss;   // [F][epochs]
    MlpLayout lay;
    int D0, epochs, batch, weighted, n_milestones;
    int64_t N;
    int H;  // widest hidden layer: the row stride of the activation buffers
    int milestones[8];
    float lr, gamma, weight_decay, dropout;
    uint64_t seed;
};

__device__ __forceinline__ uint32_t mlp_hash(uint64_t a, uint64_t b) {  // splitmix64 finalizer
    uint64_t z = a * 0x9E3779B97F4A7C15ull + b + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) >> 32);
}

// keep test of one dropout unit: u in [0, 1) with 24 bits; kept when u >= p (probability 1 - p)
__device__ __forceinline__ bool mlp_keep(const MlpFitParams& p, int fold, int64_t step, int layer, int unit) {
    const uint32_t h = mlp_hash(p.seed ^ ((uint64_t)fold << 48), ((uint64_t)step << 20) ^ ((uint64_t)layer << 16) ^
                                                                     (uint64_t)unit);
    return (float)(h >> 8) * (1.0f / 16777216.0f) >= p.dropout;
}

struct MlpSmem {
    float* P;    // [np] parameters
    float* G;    // [np] gradients
    float* RS;   // running statistics (ns - np)
    float* xb;   // [B][D0]
    float* yb;   // [B]
    float* xh;   // [L-1][B][H] normalized pre-activations
    float* act;  // [L-1][B][H] post ReLU + dropout outputs
    float* da;   // [B][max(H, 1)] gradient w.r.t. the current layer's output
    float* dz;   // [B][H]
    float* pred; // [B]
    float* st;   // [2][H] batch mean / invstd
    float* red;  // [MLP_NT] scratch
};

// z[i][o] = b[o] + sum_k in[i][k] W[o][k]   (k ascending, a single fma chain per output)
__device__ __forceinline__ void mlp_linear(const float* in, int ld_in, int n, int din, int dout, const float* W,
                                           const float* bias, float* z, int ld_z) {
    for (int t = threadIdx.x; t < n * dout; t += MLP_NT) {
        const int i = t / dout, o = t - i * dout;
        const float* r = in + i * ld_in;
        const float* w = W + o * din;
        float acc = 0.f;
        for (int k = 0; k < din; ++k) acc = fmaf(r[k], w[k], acc);
        z[i * ld_z + o] = acc + bias[o];
    }
}

// One forward pass over the n rows in S.xb; train mode uses batch statistics (and updates the
// running ones) and dropout.  Leaves the prediction in S.pred.
__device__ void mlp_forward(const MlpFitParams& p, const MlpSmem& S, int n, bool train, int fold, int64_t step) {
    const MlpLayout& m = p.lay;
    const int H = p.H;
    const float* in = S.xb;
    int ld_in = p.D0;
    for (int l = 0; l < m.L; ++l) {
        const int din = m.d[l], dout = m.d[l + 1];
        if (l == m.L - 1) {
            mlp_linear(in, ld_in, n, din, dout, S.P + m.w[l], S.P + m.b[l], S.pred, 1);
            __syncthreads();
            break;
        }
        float* xh = S.xh + l * p.batch * H;
        float* a = S.act + l * p.batch * H;
        mlp_linear(in, ld_in, n, din, dout, S.P + m.w[l], S.P + m.b[l], xh, H);  // z, normalized in place below
        __syncthreads();
        if (threadIdx.x < dout) {
            const int o = threadIdx.x;
            float mean, invstd;
            if (train) {
                float s = 0.f;
                for (int i = 0; i < n; ++i) s += xh[i * H + o];
                mean = s / (float)n;
                float v = 0.f;
                for (int i = 0; i < n; ++i) {
                    const float d = xh[i * H + o] - mean;
                    v = fmaf(d, d, v);
                }
                const float var = v / (float)n;
                invstd = 1.f / sqrtf(var + 1e-5f);
                float* rm = S.RS + (m.rm[l] - m.np);
                float* rv = S.RS + (m.rv[l] - m.np);
                rm[o] = 0.9f * rm[o] + 0.1f * mean;
                rv[o] = 0.9f * rv[o] + 0.1f * (n > 1 ? v / (float)(n - 1) : var);
            } else {
                mean = S.RS[m.rm[l] - m.np + o];
                invstd = 1.f / sqrtf(S.RS[m.rv[l] - m.np + o] + 1e-5f);
            }
            S.st[o] = mean;
            S.st[H + o] = invstd;
            S.st[(2 + l) * H + o] = invstd;  // kept for the backward pass
        }
        __syncthreads();
        const float scale = train && p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
        for (int t = threadIdx.x; t < n * dout; t += MLP_NT) {
            const int i = t / dout, o = t - i * dout;
            const float h = (xh[i * H + o] - S.st[o]) * S.st[H + o];
            xh[i * H + o] = h;
            float r = fmaxf(S.P[m.g[l] + o] * h + S.P[m.be[l] + o], 0.f);
            if (train && p.dropout > 0.f) r = mlp_keep(p, fold, step, l, i * dout + o) ? r * scale : 0.f;
            a[i * H + o] = r;
        }
        __syncthreads();
        in = a;
        ld_in = H;
    }
}

// mean over the batch of (pred - y)^2 (times y when weighted), summed in row order
__device__ float mlp_batch_loss(const MlpFitParams& p, const MlpSmem& S, int n) {
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int i = 0; i < n; ++i) {
            const float d = S.pred[i] - S.yb[i];
            s += p.weighted ? d * d * S.yb[i] : d * d;
        }
        S.red[0] = s / (float)n;
    }
    __syncthreads();
    const float v = S.red[0];
    __syncthreads();
    return v;
}

__device__ void mlp_backward(const MlpFitParams& p, const MlpSmem& S, int n) {
    const MlpLayout& m = p.lay;
    const int H = p.H;
    const float scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
    // d loss / d pred
    for (int i = threadIdx.x; i < n; i += MLP_NT) {
        const float d = S.pred[i] - S.yb[i];
        S.dz[i * H] = (p.weighted ? 2.f * d * S.yb[i] : 2.f * d) / (float)n;
    }
    __syncthreads();
    for (int l = m.L - 1; l >= 0; --l) {
        const int din = m.d[l], dout = m.d[l + 1];
        const float* in = l == 0 ? S.xb : S.act + (l - 1) * p.batch * H;
        const int ld_in = l == 0 ? p.D0 : H;
        if (l < m.L - 1) {
            // dz from da: dropout + ReLU, then BatchNorm backward per unit
            const float* xh = S.xh + l * p.batch * H;
            const float* a = S.act + l * p.batch * H;
            for (int t = threadIdx.x; t < n * dout; t += MLP_NT) {
                const int i = t / dout, o = t - i * dout;
                S.dz[i * H + o] = a[i * H + o] > 0.f ? S.da[i * H + o] * scale : 0.f;  // dy
            }
            __syncthreads();
            if (threadIdx.x < dout) {
                const int o = threadIdx.x;
                float sdy = 0.f, sdyx = 0.f;
                for (int i = 0; i < n; ++i) {
                    sdy += S.dz[i * H + o];
                    sdyx = fmaf(S.dz[i * H + o], xh[i * H + o], sdyx);
                }
                S.G[m.g[l] + o] = sdyx;
                S.G[m.be[l] + o] = sdy;
                S.st[o] = sdy / (float)n;
                S.st[H + o] = sdyx / (float)n;
            }
            __syncthreads();
            for (int t = threadIdx.x; t < n * dout; t += MLP_NT) {  // (dy - mean dy - xhat mean(dy xhat)) invstd gamma
                const int i = t / dout, o = t - i * dout;
                const float dy = S.dz[i * H + o];
                S.dz[i * H + o] = (dy - S.st[o] - xh[i * H + o] * S.st[H + o]) * S.st[(2 + l) * H + o] *
                                  S.P[m.g[l] + o];
            }
            __syncthreads();
        }
        // linear layer l: dW, db, and da for the layer below
        for (int t = threadIdx.x; t < dout * din; t += MLP_NT) {
            const int o = t / din, k = t - o * din;
            float acc = 0.f;
            for (int i = 0; i < n; ++i) acc = fmaf(S.dz[i * H + o], in[i * ld_in + k], acc);
            S.G[m.w[l] + t] = acc;
        }
        for (int o = threadIdx.x; o < dout; o += MLP_NT) {
            float acc = 0.f;
            for (int i = 0; i < n; ++i) acc += S.dz[i * H + o];
            S.G[m.b[l] + o] = acc;
        }
        if (l > 0) {
            const float* W = S.P + m.w[l];
            for (int t = threadIdx.x; t < n * din; t += MLP_NT) {
                const int i = t / din, k = t - i * din;
                float acc = 0.f;
                for (int o = 0; o < dout; ++o) acc = fmaf(S.dz[i * H + o], W[o * din + k], acc);
                S.da[i * H + k] = acc;
            }
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(MLP_NT) mlp_fit_kernel(MlpFitParams p) {
    const MlpLayout& m = p.lay;
    const int fold = blockIdx.x;
    const int H = p.H, B = p.batch, L = m.L;
    extern __shared__ __attribute__((aligned(16))) float mlp_sm[];
    MlpSmem S;
    S.P = mlp_sm;
    S.G = S.P + m.np;
    S.RS = S.G + m.np;
    S.xb = S.RS + (m.ns - m.np);
    S.yb = S.xb + B * p.D0;
    S.xh = S.yb + B;
    S.act = S.xh + (L - 1) * B * H;
    S.da = S.act + (L - 1) * B * H;
    S.dz = S.da + B * H;
    S.pred = S.dz + B * H;
    S.st = S.pred + B;  // [2 + L - 1][H]: mean / invstd (or backward sums), per-layer invstd
    S.red = S.st + (2 + MLP_MAXL) * H;
    const float* init = p.init + (int64_t)fold * m.ns;
    for (int t = threadIdx.x; t < m.ns; t += MLP_NT) S.P[t < m.np ? t : t + m.np] = init[t];  // P | G | RS
    float* am = p.adam + (int64_t)fold * 2 * m.np;
    float* av = am + m.np;
    for (int t = threadIdx.x; t < 2 * m.np; t += MLP_NT) am[t] = 0.f;
    float* best = p.best + (int64_t)fold * m.ns;
    __syncthreads();

    const int64_t tr0 = p.tr_off[fold], ntr = p.tr_off[fold + 1] - tr0;
    const int64_t va0 = p.va_off[fold], nva = p.va_off[fold + 1] - va0;
    float best_loss = __builtin_inff();
    int64_t step = 0;
    auto stage = [&](const int32_t* idx, int64_t b0, int n) {
        for (int t = threadIdx.x; t < n * p.D0; t += MLP_NT) {
            const int i = t / p.D0, k = t - i * p.D0;
            S.xb[t] = p.x[(int64_t)idx[b0 + i] * p.D0 + k];
        }
        for (int i = threadIdx.x; i < n; i += MLP_NT) S.yb[i] = p.y[(int64_t)fold * p.N + idx[b0 + i]];
        __syncthreads();
    };
    for (int ep = 0; ep < p.epochs; ++ep) {
        int nm = 0;
        for (int j = 0; j < p.n_milestones; ++j) nm += p.milestones[j] <= ep ? 1 : 0;
        double lr = p.lr;  // MultiStepLR: lr * gamma per milestone reached, in double as the scheduler
        for (int j = 0; j < nm; ++j) lr *= (double)p.gamma;
        float tr_sum = 0.f;
        int nb = 0;
        for (int64_t b0 = 0; b0 < ntr; b0 += B, ++nb) {
            const int n = (int)(ntr - b0 < B ? ntr - b0 : B);
            stage(p.tr_idx + tr0, b0, n);
            mlp_forward(p, S, n, true, fold, step);
            tr_sum += mlp_batch_loss(p, S, n);
            mlp_backward(p, S, n);
            ++step;
            // Adam (torch.optim.Adam, single-tensor path): grad += wd * param; m.lerp_(g, 1 - b1);
            // v = b2 v + (1 - b2) g^2; p += (-lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
            const double bc1 = 1.0 - pow(0.9, (double)step), bc2 = 1.0 - pow(0.999, (double)step);
            const float step_size = (float)(lr / bc1), bc2s = (float)sqrt(bc2);
            for (int t = threadIdx.x; t < m.np; t += MLP_NT) {
                const float g = S.G[t] + p.weight_decay * S.P[t];
                const float mm = am[t] + 0.1f * (g - am[t]);
                const float vv = 0.999f * av[t] + 0.001f * g * g;
                am[t] = mm;
                av[t] = vv;
                const float denom = sqrtf(vv) / bc2s + 1e-8f;
                S.P[t] = S.P[t] + (-step_size * mm) / denom;
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) p.train_loss[(int64_t)fold * p.epochs + ep] = nb ? tr_sum / (float)nb : 0.f;
        // test pass on the validation fold (eval mode), mean of the batch losses
        float te_sum = 0.f;
        int nbv = 0;
        for (int64_t b0 = 0; b0 < nva; b0 += B, ++nbv) {
            const int n = (int)(nva - b0 < B ? nva - b0 : B);
            stage(p.va_idx + va0, b0, n);
            mlp_forward(p, S, n, false, fold, step);
            te_sum += mlp_batch_loss(p, S, n);
        }
        const float te = nbv ? te_sum / (float)nbv : 0.f;
        if (threadIdx.x == 0) p.test_loss[(int64_t)fold * p.epochs + ep] = te;
        if (te < best_loss) {  // uniform
            best_loss = te;
            for (int t = threadIdx.x; t < m.ns; t += MLP_NT) best[t] = S.P[t < m.np ? t : t + m.np];
        }
        __syncthreads();
    }
    float* last = p.last + (int64_t)fold * m.ns;
    for (int t = threadIdx.x; t < m.ns; t += MLP_NT) last[t] = S.P[t < m.np ? t : t + m.np];
}

// Eval-mode forward, one thread per row: out[r] = net(x[idx[r]]) with the running statistics.
__global__ void __launch_bounds__(MLP_NT) mlp_predict_kernel(const float* __restrict__ x, int D0,
                                                             const int32_t* __restrict__ idx, int64_t n,
                                                             MlpLayout m, const float* __restrict__ state,
                                                             float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * MLP_NT + threadIdx.x;
    if (r >= n) return;
    const float* xr = x + (int64_t)(idx ? idx[r] : r) * D0;
    float h0[MLP_MAXH], h1[MLP_MAXH];
    const float* in = xr;
    float* outv = h0;
    for (int l = 0; l < m.L; ++l) {
        const int din = m.d[l], dout = m.d[l + 1];
        const float* W = state + m.w[l];
        const float* bias = state + m.b[l];
        for (int o = 0; o < dout; ++o) {
            float acc = 0.f;
            for (int k = 0; k < din; ++k) acc = fmaf(in[k], W[o * din + k], acc);
            float z = acc + bias[o];
            if (l < m.L - 1) {
                const float h = (z - state[m.rm[l] + o]) * (1.f / sqrtf(state[m.rv[l] + o] + 1e-5f));
                z = fmaxf(state[m.g[l] + o] * h + state[m.be[l] + o], 0.f);
            }
            outv[o] = z;
        }
        in = outv;
        outv = outv == h0 ? h1 : h0;
    }
    out[r] = in[0];
}

static bool mlp_layout_ok(int L, const int* dims, int D0) {
    if (L < 1 || L > MLP_MAXL || dims[0] != D0 || D0 < 1 || D0 > MLP_MAXD0 || dims[L] != 1) return false;
    for (int l = 1; l < L; ++l)
        if (dims[l] < 1 || dims[l] > MLP_MAXH) return false;
    return true;
}

extern "C" int64_t edgedet_mlp_state_size(int32_t L, const int32_t* dims) {
    if (L < 1 || L > MLP_MAXL) return -1;
    return mlp_layout(L, dims).ns;
}

extern "C" int edgedet_mlp_fit(const float* x, int64_t N, int64_t D0, const float* y, const int32_t* tr_idx,
                               const int64_t* tr_off, const int32_t* va_idx, const int64_t* va_off, int32_t folds,
                               int32_t L, const int32_t* dims, const float* init, float* best, float* last,
                               float* adam, float* train_loss, float* test_loss, int32_t epochs, int32_t batch,
                               float lr, float gamma, const int32_t* milestones, int32_t n_milestones,
                               float weight_decay, int32_t weighted, float dropout, uint64_t seed, void* stream) {
    EDGEDET_REQUIRE(x && y && tr_idx && tr_off && va_idx && va_off && dims && init && best && last && adam &&
                        train_loss && test_loss,
                    "mlp_fit: null pointer");
    EDGEDET_REQUIRE(mlp_layout_ok(L, dims, (int)D0), "mlp_fit: layers d0 (<= 1024) -> hidden (<= 64) -> 1, <= 8 layers");
    EDGEDET_REQUIRE(folds >= 1 && epochs >= 1 && batch >= 2 && batch <= MLP_MAXB && N >= 1, "mlp_fit: sizes");
    EDGEDET_REQUIRE(n_milestones >= 0 && n_milestones <= 8 && dropout >= 0.f && dropout < 1.f, "mlp_fit: options");
    MlpFitParams p{};
    p.x = x;
    p.y = y;
    p.tr_idx = tr_idx;
    p.tr_off = tr_off;
    p.va_idx = va_idx;
    p.va_off = va_off;
    p.init = init;
    p.best = best;
    p.last = last;
    p.adam = adam;
    p.train_loss = train_loss;
    p.test_loss = test_loss;
    p.lay = mlp_layout(L, dims);
    p.D0 = (int)D0;
    p.N = N;
    p.epochs = epochs;
    p.batch = batch;
    p.weighted = weighted;
    p.n_milestones = n_milestones;
    for (int j = 0; j < n_milestones; ++j) p.milestones[j] = milestones[j];
    p.lr = lr;
    p.gamma = gamma;
    p.weight_decay = weight_decay;
    p.dropout = dropout;
    p.seed = seed;
    const MlpLayout& m = p.lay;
    p.H = 1;
    for (int l = 1; l < L; ++l) p.H = dims[l] > p.H ? dims[l] : p.H;
    const size_t H = p.H;
    const size_t floats = 2 * (size_t)m.np + (m.ns - m.np) + (size_t)batch * D0 + batch + 2 * (size_t)(L - 1) * batch * H +
                          2 * (size_t)batch * H + batch + (2 + MLP_MAXL) * H + MLP_NT;
    const size_t lds = floats * sizeof(float);
    EDGEDET_REQUIRE(lds <= 160 * 1024, "mlp_fit: parameters + batch exceed the 160 KiB LDS of a workgroup");
    static bool attr = false;
    if (!attr) {
        EDGEDET_CHECK_HIP(
            hipFuncSetAttribute((const void*)mlp_fit_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    hipLaunchKernelGGL(mlp_fit_kernel, dim3((unsigned)folds), dim3(MLP_NT), lds, (hipStream_t)stream, p);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

extern "C" int edgedet_mlp_predict(const float* x, int64_t D0, const int32_t* idx, int64_t n, int32_t L,
                                   const int32_t* dims, const float* state, float* out, void* stream) {
    EDGEDET_REQUIRE(x && dims && state && out, "mlp_predict: null pointer");
    EDGEDET_REQUIRE(mlp_layout_ok(L, dims, (int)D0), "mlp_predict: layers d0 (<= 1024) -> hidden (<= 64) -> 1");
    if (n <= 0) return 0;
    hipLaunchKernelGGL(mlp_predict_kernel, dim3((unsigned)cdiv(n, MLP_NT)), dim3(MLP_NT), 0, (hipStream_t)stream, x,
                       (int)D0, idx, n, mlp_layout(L, dims), state, out);
    EDGEDET_LAUNCH_CHECK();
    return 0;
}

}  // namespace edgedet
