// Native model lowering: the detector call of torch_models/detect.py:78 as a C-ABI entry.
//
// The reference's seam is the torchvision model call model(images) -> boxes/scores/labels
// (detect.py:72,78).  This file turns a detector configuration (SSDLite320-MobileNetV3 of
// detect.py:24/26, Faster R-CNN R50-FPN-v2 of detect.py:30/32) into the same static execution plan
// the Python host builds (edgeml_amd/models.py + plan.py): packed weights (BatchNorm folded in
// float64, conv weights K-contiguous with K padded to 32, bf16x3 planes, depthwise tap-major, SE fc2
// transposed, FC6 permuted to (h, w, c), predictor rows [bbox | cls]), one workspace carved into
// buffers in the same order with the same 256-byte alignment, and the same op records (tiles from
// the same tuned table).  So a C / C++ / Go host can run a detector with nothing but this library:
//   edgedet_<model>_pack            torchvision-named host tensors -> packed weight blob (host)
//   edgedet_<model>_workspace_size  bytes of the caller-owned workspace for (B, H, W, input dtype)
//   edgedet_<model>_prepare         write the plan's constants (anchors, rescale ratios) into it
//   edgedet_<model>_forward         run the forward (preprocess -> NMS -> rescale) on a stream
// and the results are bit-identical to the Python model object's (tests/test_native_model.py,
// tests/test_gpu_native_model.py).  Everything here is host code; the kernels are in the other units.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <tuple>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "kernels.hpp"

namespace edgedet {
namespace lower {

// ------------------------------------------------------------------------------------ tile table
static const std::unordered_map<std::string, int>& tile_table() {
    static const std::unordered_map<std::string, int> t = {
#include "conv_tiles_gfx950.inc"
    };
    return t;
}

static bool env_is(const char* k, const char* v, const char* dflt) {
    const char* e = getenv(k);
    return std::string(e ? e : dflt) == v;
}
static int env_int(const char* k, int dflt) {
    const char* e = getenv(k);
    return e && *e ? atoi(e) : dflt;
}

enum Act { A_NONE = 0, A_RE = 1, A_R6 = 2, A_HS = 3 };

// ------------------------------------------------------------------------------------ weights
// Named host parameters (torchvision state_dict keys).  With values == nullptr the packer only lays
// the blob out (sizes, offsets): what lowering needs.
struct Params {
    std::map<std::string, std::pair<const float*, int64_t>> m;
    bool values = false;
    const float* get(const std::string& k, int64_t n) const {
        auto it = m.find(k);
        if (it == m.end()) throw std::runtime_error("missing parameter " + k);
        if (it->second.second != n)
            throw std::runtime_error("size mismatch for " + k + ": got " + std::to_string(it->second.second) +
                                     " elements, expected " + std::to_string(n));
        return it->second.first;
    }
    void check(const std::string&, int64_t) const {}  // layout-only packing: nothing to check
};

struct WRef {
    int64_t off = -1, n = 0;  // float offset / count in the blob
    int64_t split = -1;       // float offset of the bf16x3 planes (conv weights)
};

// plan.py WeightPack: arrays at 64-float boundaries.
struct Pack {
    bool values = false;
    std::vector<float> blob;
    int64_t size = 0;
    WRef add(const float* a, int64_t n) {
        WRef r;
        r.off = size;
        r.n = n;
        size += (n + 63) / 64 * 64;
        if (values) {
            blob.resize((size_t)size, 0.f);
            if (a) std::memcpy(blob.data() + r.off, a, (size_t)n * 4);
        }
        return r;
    }
    WRef add_u16(const uint16_t* a, int64_t n) {
        const int64_t nf = (n + 1) / 2;
        WRef r = add(nullptr, nf);
        if (values && a) std::memcpy(blob.data() + r.off, a, (size_t)n * 2);
        return r;
    }
};

static uint16_t bf16_rn(float x, float* back) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    const uint32_t r = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    const uint32_t b = r << 16;
    std::memcpy(back, &b, 4);
    return (uint16_t)r;
}

// plan.split_bf16x3: x0 = RN(x), x1 = RN(x - x0), x2 = RN(x - x0 - x1); planes [3][n] of rows of
// kpad, x = -w in the odd 32-wide K blocks (the bf16x6 kernels' sign-alternated stages).
static std::vector<uint16_t> split_bf16x3(const std::vector<float>& w, int64_t kpad) {
    const size_t n = w.size();
    std::vector<uint16_t> out(3 * n);
    for (size_t i = 0; i < n; ++i) {
        float f0, f1, f2;
        const float x = (((int64_t)i % kpad) >> 5) & 1 ? -w[i] : w[i];
        out[i] = bf16_rn(x, &f0);
        const float r1 = x - f0;
        out[n + i] = bf16_rn(r1, &f1);
        const float r2 = r1 - f1;
        out[2 * n + i] = bf16_rn(r2, &f2);
    }
    return out;
}

struct ConvW {
    WRef w, b;
    int64_t K = 0, Kpad = 0, cin = 0;
    bool dw = false;
};

class Packer {
  public:
    Packer(const Params& P, Pack& pk) : P_(P), pk_(pk) {}

    // fold_bn + pack_conv_weight (+ bf16x3 planes), or pack_dw_weight for a depthwise conv.
    ConvW conv_bn(const std::string& wkey, const std::string& bnp, double eps, int64_t cout, int64_t cin, int k,
                  bool depthwise, int64_t cin_pad = 0) {
        auto key = "cbn:" + wkey;
        auto it = cache_.find(key);
        if (it != cache_.end()) return it->second;
        const int64_t cin_w = depthwise ? 1 : cin;
        const int64_t nw = cout * cin_w * k * k;
        std::vector<double> wf((size_t)nw, 0.0);
        std::vector<double> bf((size_t)cout, 0.0);
        if (pk_.values) {
            const float* w = P_.get(wkey, nw);
            const float* g = P_.get(bnp + ".weight", cout);
            const float* be = P_.get(bnp + ".bias", cout);
            const float* mu = P_.get(bnp + ".running_mean", cout);
            const float* var = P_.get(bnp + ".running_var", cout);
            for (int64_t o = 0; o < cout; ++o) {
                const double scale = (double)g[o] / std::sqrt((double)var[o] + eps);
                for (int64_t j = 0; j < cin_w * k * k; ++j) wf[(size_t)(o * cin_w * k * k + j)] = (double)w[o * cin_w * k * k + j] * scale;
                bf[(size_t)o] = (double)be[o] - (double)mu[o] * scale;
            }
        } else {
            P_.check(wkey, nw);
        }
        std::vector<float> w32(wf.begin(), wf.end()), b32(bf.begin(), bf.end());
        ConvW r;
        if (depthwise) {  // [C][1][k][k] -> [k*k][C]
            std::vector<float> t((size_t)nw);
            for (int64_t c = 0; c < cout; ++c)
                for (int64_t q = 0; q < k * k; ++q) t[(size_t)(q * cout + c)] = w32[(size_t)(c * k * k + q)];
            r.w = pk_.add(t.data(), nw);
            r.b = pk_.add(b32.data(), cout);
            r.K = k;
            r.cin = cout;
            r.dw = true;
        } else {
            r = conv_w(w32, cout, cin, k, cin_pad);
            r.b = pk_.add(b32.data(), cout);
        }
        cache_[key] = r;
        return r;
    }

    // A conv with bias and no BatchNorm (weights as given); w may be a Linear [cout][cin].
    ConvW conv_bias(const std::string& wkey, const std::string& bkey, int64_t cout, int64_t cin, int k) {
        auto key = "cb:" + wkey;
        auto it = cache_.find(key);
        if (it != cache_.end()) return it->second;
        const int64_t nw = cout * cin * k * k;
        std::vector<float> w((size_t)nw, 0.f), b((size_t)cout, 0.f);
        if (pk_.values) {
            std::memcpy(w.data(), P_.get(wkey, nw), (size_t)nw * 4);
            std::memcpy(b.data(), P_.get(bkey, cout), (size_t)cout * 4);
        } else {
            P_.check(wkey, nw);
        }
        ConvW r = conv_w(w, cout, cin, k, 0);
        r.b = pk_.add(b.data(), cout);
        cache_[key] = r;
        return r;
    }

    // A conv without bias and without BatchNorm (RetinaNet GroupNorm towers): a zero bias.
    ConvW conv_nobias(const std::string& wkey, int64_t cout, int64_t cin, int k) {
        auto key = "cn:" + wkey;
        auto it = cache_.find(key);
        if (it != cache_.end()) return it->second;
        const int64_t nw = cout * cin * k * k;
        std::vector<float> w((size_t)nw, 0.f), b((size_t)cout, 0.f);
        if (pk_.values)
            std::memcpy(w.data(), P_.get(wkey, nw), (size_t)nw * 4);
        else
            P_.check(wkey, nw);
        ConvW r = conv_w(w, cout, cin, k, 0);
        r.b = pk_.add(b.data(), cout);
        cache_[key] = r;
        return r;
    }

    // pack_conv_weight on an already-built [cout][cin][k][k] fp32 weight + its bias (FC6, predictor).
    ConvW conv_given(const std::string& key, const std::vector<float>& w, const std::vector<float>& b, int64_t cout,
                     int64_t cin, int k) {
        auto it = cache_.find(key);
        if (it != cache_.end()) return it->second;
        ConvW r = conv_w(w, cout, cin, k, 0);
        r.b = pk_.add(b.data(), cout);
        cache_[key] = r;
        return r;
    }

    WRef raw(const std::string& key, const std::vector<float>& a) {
        auto it = raw_.find(key);
        if (it != raw_.end()) return it->second;
        return raw_[key] = pk_.add(a.data(), (int64_t)a.size());
    }

    bool values() const { return pk_.values; }
    const Params& params() const { return P_; }

  private:
    // [cout][cin][k][k] -> [cout][Kpad] (kh, kw, ci), cin zero-padded to cin_pad; + bf16x3 planes.
    ConvW conv_w(const std::vector<float>& w, int64_t cout, int64_t cin, int k, int64_t cin_pad) {
        const int64_t ci = cin_pad > cin ? cin_pad : cin;
        const int64_t K = (int64_t)k * k * ci, Kpad = (K + 31) / 32 * 32;
        std::vector<float> wp;
        if (pk_.values) {
            wp.assign((size_t)(cout * Kpad), 0.f);
            for (int64_t o = 0; o < cout; ++o)
                for (int kh = 0; kh < k; ++kh)
                    for (int kw = 0; kw < k; ++kw)
                        for (int64_t c = 0; c < cin; ++c)
                            wp[(size_t)(o * Kpad + ((int64_t)kh * k + kw) * ci + c)] =
                                w[(size_t)(((o * cin + c) * k + kh) * k + kw)];
        }
        ConvW r;
        r.w = pk_.add(pk_.values ? wp.data() : nullptr, cout * Kpad);
        if (pk_.values) {
            auto s = split_bf16x3(wp, Kpad);
            r.w.split = pk_.add_u16(s.data(), (int64_t)s.size()).off;
        } else {
            r.w.split = pk_.add_u16(nullptr, 3 * cout * Kpad).off;
        }
        r.K = K;
        r.Kpad = Kpad;
        r.cin = ci;
        return r;
    }

    const Params& P_;
    Pack& pk_;
    std::map<std::string, ConvW> cache_;
    std::map<std::string, WRef> raw_;
};

// ------------------------------------------------------------------------------------ plan
// A pointer field of a record, resolved at finalize: a workspace buffer (+ byte offset: batch views),
// a weight-blob offset, or nothing.
struct Ref {
    enum Kind { NONE, BUF, W } kind = NONE;
    int idx = -1;          // buffer index
    int64_t byte_off = 0;  // BUF: bytes into the buffer; W: float offset into the blob
};

// element types of workspace buffers (edgedet_buffer.dtype); Plan::buf takes the element size, or I32
enum : int { I32 = -4 };
struct Buf {
    std::vector<int64_t> shape;
    int esize = 4;
    int dtype = EDGEDET_DT_F32;
    int64_t nbytes = 0;
    int64_t off = 0;
    std::string name;
};

struct OpRec {
    int64_t kind = 0;
    int lane = 0;
    std::string name;
    std::map<int, int64_t> i;
    std::map<int, Ref> p;
    std::map<int, double> d;
    std::map<int, float> f;
};

struct External {
    uint64_t weights = 0, workspace = 0, images = 0, count = 0, boxes = 0, scores = 0, labels = 0;
    bool operator==(const External& o) const {
        return weights == o.weights && workspace == o.workspace && images == o.images && count == o.count &&
               boxes == o.boxes && scores == o.scores && labels == o.labels;
    }
};

// Redzone (diagnostic, edgedet_set_redzone; 0 in production): bytes left unused before the first
// workspace buffer, between consecutive buffers and after the last, so a test can fill them with a
// canary and find any kernel that writes outside its buffers.
static int64_t g_redzone = 0;

struct Plan {
    std::shared_ptr<const std::vector<edgedet_op>> resolved;  // records of the last forward's pointers
    External resolved_for;
    std::vector<Buf> bufs;
    std::vector<OpRec> ops;
    std::vector<std::pair<int, std::vector<uint8_t>>> consts;  // (buffer, bytes)
    int cur_lane = 0, forked = 0;
    std::map<int, int> x3;  // lane -> scratch buffer
    int64_t arena = 0;
    uint64_t last_use = 0;
    int input = -1, out_box = -1, out_score = -1, out_label = -1, out_count = -1;
    int dets = 0;

    int buf(std::vector<int64_t> shape, int esize, const std::string& name) {
        Buf b;
        b.shape = shape;
        b.dtype = esize == I32 ? EDGEDET_DT_I32
                  : esize == 1 ? EDGEDET_DT_U8
                  : esize == 2 ? EDGEDET_DT_I16
                  : esize == 8 ? EDGEDET_DT_I64
                               : EDGEDET_DT_F32;
        if (esize == I32) esize = 4;
        b.esize = esize;
        int64_t n = 1;
        for (auto s : shape) n *= s;
        b.nbytes = n * esize;
        b.name = name;
        bufs.push_back(b);
        return (int)bufs.size() - 1;
    }
    template <typename T>
    int cnst(const std::vector<T>& a, std::vector<int64_t> shape, const std::string& name) {
        const int k = buf(shape, (int)sizeof(T), name);
        std::vector<uint8_t> raw(a.size() * sizeof(T));
        std::memcpy(raw.data(), a.data(), raw.size());
        consts.push_back({k, raw});
        return k;
    }
    Ref ref(int b, int64_t byte_off = 0) const {
        Ref r;
        r.kind = Ref::BUF;
        r.idx = b;
        r.byte_off = byte_off;
        return r;
    }
    // BufView: images [b0, b0 + n) of a batch-leading buffer
    Ref view(int b, int64_t b0) const { return ref(b, b0 * (bufs[(size_t)b].nbytes / bufs[(size_t)b].shape[0])); }
    static Ref wref(const WRef& w) {
        Ref r;
        r.kind = Ref::W;
        r.byte_off = w.off;
        return r;
    }
    static Ref wsplit(const WRef& w) {
        Ref r;
        r.kind = Ref::W;
        r.byte_off = w.split;
        return r;
    }
    int x3_scratch(int64_t n) {
        auto it = x3.find(cur_lane);
        if (it == x3.end()) {
            const int k = buf({n}, 2, "x3.lane" + std::to_string(cur_lane));
            x3[cur_lane] = k;
            return k;
        }
        Buf& b = bufs[(size_t)it->second];
        if (b.shape[0] < n) {
            b.shape[0] = n;
            b.nbytes = 2 * n;
        }
        return it->second;
    }
    OpRec& add(OpRec o) {
        if (o.lane == 0 && cur_lane) o.lane = cur_lane;
        ops.push_back(o);
        return ops.back();
    }
    void fork(int n) {
        OpRec o;
        o.kind = EDGEDET_OP_FORK;
        o.name = "fork";
        o.i[0] = n;
        ops.push_back(o);
        forked = n;
    }
    void lane(int k) { cur_lane = k; }
    void join() {
        cur_lane = 0;
        OpRec o;
        o.kind = EDGEDET_OP_JOIN;
        o.name = "join";
        o.i[0] = forked;
        ops.push_back(o);
        forked = 0;
    }
    void finalize() {
        const int64_t rz = g_redzone;
        int64_t off = rz;
        for (auto& b : bufs) {
            b.off = off;
            off += (b.nbytes + 255) / 256 * 256 + rz;
        }
        arena = off > 256 ? off : 256;
    }
};

static std::string conv_key(const OpRec& o) {
    auto I = [&](int k) {
        auto it = o.i.find(k);
        return it == o.i.end() ? (int64_t)0 : it->second;
    };
    const int lin = I(7) == 1 && I(8) == 1 && I(9) == 1 && I(10) == 0;
    auto has = [&](int k) {
        auto it = o.p.find(k);
        return it != o.p.end() && it->second.kind != Ref::NONE;
    };
    std::string s;
    const int64_t v[12] = {I(0), I(1), I(2), I(3), I(4), I(5), I(6), I(7), I(9), lin, has(6), has(7)};
    for (int j = 0; j < 12; ++j) s += (j ? "," : "") + std::to_string(v[j]);
    return s;
}

struct ConvArgs {
    Ref x, y, res, in_scale, in_shift;
    std::vector<int64_t> xs, ys;  // (B, H, W, C) / (B, Ho, Wo, Cout)
    ConvW w;
    int64_t cout = 0;
    int k = 1, stride = 1, pad = 0, act = 0;
    int64_t y_pstride = -1, y_bstride = -1, y_off = 0, x_pstride = -1, x_bstride = -1;
    int res_h = -1, res_w = -1, tile = 0;
    bool in_relu = false;
    std::string name;
};

// plan.conv_op
static void conv_op(Plan& P, const ConvArgs& a) {
    const int64_t B = a.xs[0], H = a.xs[1], W = a.xs[2], C = a.xs[3];
    const int64_t Ho = a.ys[1], Wo = a.ys[2];
    if (Ho != (H + 2 * a.pad - a.k) / a.stride + 1 || Wo != (W + 2 * a.pad - a.k) / a.stride + 1)
        throw std::runtime_error("conv_op: output size mismatch");
    if (a.w.K != (int64_t)a.k * a.k * C) throw std::runtime_error("conv_op: K != k*k*C");
    const int64_t xp = a.x_pstride < 0 ? C : a.x_pstride;
    const int64_t yp = a.y_pstride < 0 ? a.cout : a.y_pstride;
    const int64_t rH = a.res_h < 0 ? Ho : a.res_h, rW = a.res_w < 0 ? Wo : a.res_w;
    OpRec o;
    o.kind = EDGEDET_OP_CONV;
    o.name = a.name;
    const int64_t iv[25] = {B, H, W, C, Ho, Wo, a.cout, a.k, a.k, a.stride, a.pad, a.act, a.w.K, a.w.Kpad, xp, yp,
                            a.cout, a.x_bstride < 0 ? H * W * xp : a.x_bstride,
                            a.y_bstride < 0 ? Ho * Wo * yp : a.y_bstride, rH * rW * a.cout, a.y_off, rH, rW, a.tile,
                            a.in_relu ? 1 : 0};
    for (int j = 0; j < 25; ++j) o.i[j] = iv[j];
    const bool bf16x6 = !env_is("EDGEDET_CONV_MATH", "f32", "bf16x6");
    o.p[0] = a.x;
    o.p[1] = Plan::wref(a.w.w);
    o.p[2] = Plan::wref(a.w.b);
    o.p[3] = a.y;
    o.p[4] = a.res;
    o.p[5] = a.in_scale;
    o.p[6] = bf16x6 ? Plan::wsplit(a.w.w) : Ref();
    o.p[7] = a.in_shift;
    const bool w3 = o.p[6].kind != Ref::NONE;
    if (!a.tile && env_int("EDGEDET_CONV_TUNED", 1) == 1) {
        auto it = tile_table().find(conv_key(o));
        if (it != tile_table().end() && it->second && (w3 || it->second < 20)) o.i[23] = it->second;
    }
    // the Cout = 256 layers the table puts on 256 x 128 run the 128 x 256 tile: one N tile, so each A
    // panel is read once (FRCNN 362.6 / 362.5 -> 369.9 / 373.8 img/s in alternated runs; box head 3x3
    // 2.09 -> 1.88 ms in the conv microbench, profiles/r4c_conv39.txt); input-transformed layers keep
    // 25 and its pre-split input (below)
    const bool xf = a.in_scale.kind != Ref::NONE || a.in_shift.kind != Ref::NONE || a.in_relu;
    if (o.i[23] == 25 && a.cout == 256 && !xf) o.i[23] = 39;
    if (o.i[23] == 26) {
        const bool dense = yp == a.cout && a.y_off == 0 && (a.y_bstride < 0 || a.y_bstride == Ho * Wo * a.cout);
        if (a.act == 0 && a.res.kind == Ref::NONE && dense && w3) {
            OpRec m;
            m.kind = EDGEDET_OP_MEMSET;
            m.name = a.name + ".zero";
            m.i[0] = B * Ho * Wo * a.cout * 4;
            m.p[0] = a.y;
            P.add(m);
        } else {
            o.i[23] = 25;
        }
    }
    // pre-split input planes only where an input transform is fused (GN / SE / ReLU on load): the split
    // pass then also takes the per-element transform out of the GEMM loop; for a plain input the extra
    // HBM pass measured slower (FRCNN 336 -> 313 img/s)
    if (xf && w3 && C % 32 == 0 && (o.i[23] == 0 || o.i[23] == 25))
        o.p[8] = P.ref(P.x3_scratch(3 * B * H * W * C + 32));
    P.add(o);
}

// ------------------------------------------------------------------------------------ SSDLite
struct Block {
    int cin, k, exp, cout;
    bool se;
    int act, stride;
};

static std::vector<Block> mnv3_blocks(bool reduced) {
    const int c4 = reduced ? 80 : 160, e4 = reduced ? 480 : 960;
    return {{16, 3, 16, 16, false, A_RE, 1},   {16, 3, 64, 24, false, A_RE, 2},  {24, 3, 72, 24, false, A_RE, 1},
            {24, 5, 72, 40, true, A_RE, 2},    {40, 5, 120, 40, true, A_RE, 1},  {40, 5, 120, 40, true, A_RE, 1},
            {40, 3, 240, 80, false, A_HS, 2},  {80, 3, 200, 80, false, A_HS, 1}, {80, 3, 184, 80, false, A_HS, 1},
            {80, 3, 184, 80, false, A_HS, 1},  {80, 3, 480, 112, true, A_HS, 1}, {112, 3, 672, 112, true, A_HS, 1},
            {112, 5, 672, c4, true, A_HS, 2},  {c4, 5, e4, c4, true, A_HS, 1},   {c4, 5, e4, c4, true, A_HS, 1}};
}

static int make_divisible(double v, int d = 8) {
    int nv = std::max(d, (int)(v + d / 2.0) / d * d);
    if (nv < 0.9 * v) nv += d;
    return nv;
}

struct Prefixes {
    std::string pe, pd, ps, pp;
};
static Prefixes block_prefixes(const Block& b, const std::string& base) {
    Prefixes r;
    int j = 0;
    if (b.exp != b.cin) r.pe = base + "." + std::to_string(j++);
    r.pd = base + "." + std::to_string(j++);
    if (b.se) r.ps = base + "." + std::to_string(j++);
    r.pp = base + "." + std::to_string(j);
    return r;
}

struct Cur {
    Ref x;
    std::vector<int64_t> s;  // (B, H, W, C)
};

struct Config {
    int kind = 0;  // 0 ssdlite, 1 frcnn
    int num_classes = 91;
    bool reduced_tail = true;
};

// anchors.ssd_default_boxes for a 320 x 320 input: [A, 4] xyxy pixels, order (map, i, j, a)
static std::vector<float> ssd_default_boxes(const std::vector<std::pair<int, int>>& grids, int S) {
    const int n = 6;
    std::vector<double> scales;
    for (int k = 0; k < n; ++k) scales.push_back(0.2 + (0.95 - 0.2) * k / (n - 1.0));
    scales.push_back(1.0);
    std::vector<float> out;
    for (int k = 0; k < (int)grids.size(); ++k) {
        const int fh = grids[(size_t)k].first, fw = grids[(size_t)k].second;
        const double sk = scales[(size_t)k], spk = std::sqrt(scales[(size_t)k] * scales[(size_t)k + 1]);
        std::vector<std::pair<double, double>> whd = {{sk, sk}, {spk, spk}};
        for (int ar : {2, 3}) {
            const double sq = std::sqrt((double)ar);
            whd.push_back({sk * sq, sk / sq});
            whd.push_back({sk / sq, sk * sq});
        }
        std::vector<std::pair<float, float>> wh;
        for (auto& p : whd) {
            float a = (float)p.first, b = (float)p.second;
            a = a < 0.f ? 0.f : (a > 1.f ? 1.f : a);
            b = b < 0.f ? 0.f : (b > 1.f ? 1.f : b);
            wh.push_back({a, b});
        }
        for (int i = 0; i < fh; ++i)
            for (int j = 0; j < fw; ++j) {
                const float cx = ((float)j + 0.5f) / (float)fw, cy = ((float)i + 0.5f) / (float)fh;
                for (auto& p : wh) {
                    const float hw = 0.5f * p.first, hh = 0.5f * p.second;
                    out.push_back((cx - hw) * (float)S);
                    out.push_back((cy - hh) * (float)S);
                    out.push_back((cx + hw) * (float)S);
                    out.push_back((cy + hh) * (float)S);
                }
            }
    }
    return out;
}

struct Lowered {
    std::unique_ptr<Plan> plan;
    int64_t weights_floats = 0;
};

class SSDLite {
  public:
    static constexpr double EPS = 1e-3;
    static constexpr int S = 320, DETS = 300, TOPK = 300;
    static constexpr double SCORE = 0.001, NMS = 0.55;
    // one x6b tile for the grouped head 1x1 convs: 128 x 64 (the cls heads' 546 columns fill 9 N tiles
    // of 64 to 95 %, 5 of 128 to 85 %): the group alone 60.5 -> 51.3 us, SSD +0.8 % in alternated
    // runs against 64 x 128 (tile 31; 128 x 128: 68.6 us, +0.5 %), profiles/r6h_head_tile_ab.txt
    static constexpr int HEAD_TILE = 38;

    SSDLite(const Config& c, Packer& pk) : cfg_(c), pk_(pk), blocks_(mnv3_blocks(c.reduced_tail)) {}

    // models.SSDLite320._pack_all: build_plan(1, 320, 320, pack_only=True) walks the network in order
    void pack_all() { lower(1, S, S, false, true); }

    std::unique_ptr<Plan> lower(int B, int H, int W, bool u8, bool pack_only = false) {
        auto P = std::make_unique<Plan>();
        int nch = pack_only ? 1 : n_chains(B);
        const int inp = P->buf({B, 3, H, W}, u8 ? 1 : 4, "images");
        Shared sh;
        if (nch > 1) P->fork(nch - 1);
        const int q = B / nch, r = B % nch;
        for (int c = 0; c < nch; ++c) {
            const int b0 = c * q + std::min(c, r), bc = q + (c < r ? 1 : 0);
            if (nch > 1) P->lane(c);
            chain(*P, c, b0, bc, B, H, W, u8, inp, sh, nch, pack_only);
            if (pack_only) return P;
        }
        if (nch > 1) P->join();
        P->input = inp;
        P->out_box = sh.ob;
        P->out_score = sh.os;
        P->out_label = sh.ol;
        P->out_count = sh.oc;
        P->dets = DETS;
        return P;
    }

  private:
    struct Shared {
        int cls = -1, reg = -1, anchors = -1, scores_t = -1, boxes = -1, ratio = -1, ob = -1, os = -1, ol = -1,
            oc = -1;
    };

    int n_chains(int B) const {
        const int n = env_int("EDGEDET_SSD_CHAINS", 0) ? env_int("EDGEDET_SSD_CHAINS", 0) : 2;
        return std::max(1, std::min({n, EDGEDET_MAX_LANES, B >= 16 ? B / 8 : 1}));
    }

    ConvW cbn(const std::string& prefix, int64_t cout, int64_t cin, int k, bool dw, int64_t cin_pad = 0) {
        return pk_.conv_bn(prefix + ".0.weight", prefix + ".1", EPS, cout, cin, k, dw, cin_pad);
    }

    void chain(Plan& P, int c, int img0, int B, int Btot, int H, int W, bool u8, int inp, Shared& sh, int nch,
               bool pack_only) {
        const int NC = cfg_.num_classes;
        const std::string sfx = nch > 1 ? "#" + std::to_string(c) : "";
        auto view = [&](int b) { return nch > 1 ? P.view(b, img0) : P.ref(b); };
        // the transform (normalise 0.5 / 0.5, resize to S x S): folded into the fused stem's input loads
        // (EDGEDET_SSD_STEM_FUSE=1, the default), else its own record into an NHWC4 buffer
        const bool stem_fuse = env_int("EDGEDET_SSD_STEM_FUSE", 1) == 1 && !pack_only;
        Cur cur;
        if (!stem_fuse) {
            const int x = P.buf({B, S, S, 4}, 4, "pre" + sfx);
            OpRec o;
            o.kind = EDGEDET_OP_PREPROCESS;
            o.name = "transform";
            const int64_t iv[7] = {B, H, W, S, S, S, S};
            for (int j = 0; j < 7; ++j) o.i[j] = iv[j];
            o.p[u8 ? 2 : 0] = view(inp);
            o.p[1] = P.ref(x);
            for (int j = 0; j < 6; ++j) o.f[j] = 0.5f;
            P.add(o);
            cur = Cur{P.ref(x), {B, S, S, 4}};
        }

        auto conv = [&](const Cur& in, const std::string& prefix, int64_t cout, int k, int stride, int act,
                        Ref res = Ref(), Ref in_scale = Ref(), int64_t cin_pad = 0) {
            ConvW w = cbn(prefix, cout, cin_pad ? 3 : in.s[3], k, false, cin_pad);
            const int pad = (k - 1) / 2;
            const int64_t Ho = (in.s[1] + 2 * pad - k) / stride + 1, Wo = (in.s[2] + 2 * pad - k) / stride + 1;
            std::vector<int64_t> ys = {B, Ho, Wo, cout};
            const int y = P.buf(ys, 4, prefix + sfx);
            ConvArgs a;
            a.x = in.x;
            a.xs = in.s;
            a.w = w;
            a.cout = cout;
            a.k = k;
            a.stride = stride;
            a.pad = pad;
            a.act = act;
            a.y = P.ref(y);
            a.ys = ys;
            a.res = res;
            a.in_scale = in_scale;
            a.name = prefix;
            conv_op(P, a);
            return Cur{P.ref(y), ys};
        };
        struct DwOut {
            Cur y;
            int part = -1, parts = 0;
        };
        auto dw = [&](const Cur& in, const std::string& prefix, int k, int stride, int act, bool se_part) {
            const int64_t C = in.s[3];
            ConvW w = cbn(prefix, C, C, k, true);
            const int pad = (k - 1) / 2;
            const int64_t Ho = (in.s[1] + 2 * pad - k) / stride + 1, Wo = (in.s[2] + 2 * pad - k) / stride + 1;
            std::vector<int64_t> ys = {B, Ho, Wo, C};
            const int y = P.buf(ys, 4, prefix + sfx);
            const int64_t groups = Ho * ((Wo + 3) / 4);
            const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(SE_PARTS, groups / 16));
            const int part = se_part ? P.buf({B, parts, C}, 4, prefix + ".se_partial_sums" + sfx) : -1;
            OpRec o;
            o.kind = EDGEDET_OP_DWCONV;
            o.name = prefix;
            const int64_t iv[11] = {B, in.s[1], in.s[2], C, Ho, Wo, k, stride, pad, act, parts};
            for (int j = 0; j < 11; ++j) o.i[j] = iv[j];
            o.p[0] = in.x;
            o.p[1] = Plan::wref(w.w);
            o.p[2] = Plan::wref(w.b);
            o.p[3] = P.ref(y);
            o.p[4] = part >= 0 ? P.ref(part) : Ref();
            P.add(o);
            return DwOut{Cur{P.ref(y), ys}, part, parts};
        };
        auto se = [&](const DwOut& in, const std::string& p) {
            const int64_t C = in.y.s[3];
            const int sq = make_divisible(C / 4, 8);
            WRef w1, b1, w2t, b2;
            se_weights(p, C, sq, w1, b1, w2t, b2);
            const int scale = P.buf({B, C}, 4, p + ".scale" + sfx);
            const int hidden = P.buf({B, sq}, 4, p + ".hidden" + sfx);
            OpRec o;
            o.kind = EDGEDET_OP_SE_FC;
            o.name = p;
            const int64_t iv[5] = {B, C, sq, in.y.s[1] * in.y.s[2], in.parts};
            for (int j = 0; j < 5; ++j) o.i[j] = iv[j];
            o.p[0] = P.ref(in.part);
            o.p[1] = Plan::wref(w1);
            o.p[2] = Plan::wref(b1);
            o.p[3] = Plan::wref(w2t);
            o.p[4] = Plan::wref(b2);
            o.p[5] = P.ref(scale);
            o.p[6] = P.ref(hidden);
            P.add(o);
            return P.ref(scale);
        };
        auto mb_block = [&](const Cur& in, const Block& b, const Prefixes& pf) {
            ConvW w1 = cbn(pf.pe, b.exp, b.cin, 1, false);
            ConvW wd = cbn(pf.pd, b.exp, b.exp, b.k, true);
            ConvW w2 = cbn(pf.pp, b.cout, b.exp, 1, false);
            const int pad = (b.k - 1) / 2;
            const int64_t Ho = (in.s[1] + 2 * pad - b.k) / b.stride + 1, Wo = (in.s[2] + 2 * pad - b.k) / b.stride + 1;
            std::vector<int64_t> ys = {B, Ho, Wo, b.cout};
            const int y = P.buf(ys, 4, pf.pp + sfx);
            OpRec o;
            o.kind = EDGEDET_OP_MBCONV;
            o.name = pf.pe.substr(0, pf.pe.rfind('.'));
            const int64_t iv[15] = {B, in.s[1], in.s[2], b.cin, b.exp, b.cout, Ho, Wo, b.k, b.stride, pad, b.act,
                                    w1.Kpad, w2.Kpad, (b.stride == 1 && b.cin == b.cout) ? 1 : 0};
            for (int j = 0; j < 15; ++j) o.i[j] = iv[j];
            o.p[0] = in.x;
            o.p[1] = Plan::wref(w1.w);
            o.p[2] = Plan::wref(w1.b);
            o.p[3] = Plan::wref(wd.w);
            o.p[4] = Plan::wref(wd.b);
            o.p[5] = Plan::wref(w2.w);
            o.p[6] = Plan::wref(w2.b);
            o.p[7] = P.ref(y);
            P.add(o);
            return Cur{P.ref(y), ys};
        };
        auto inverted_residual = [&](const Cur& in, const Block& b, const std::string& base) {
            Prefixes pf = block_prefixes(b, base);
            // blocks 0.2 / 0.3 as one MBCONV launch each (EDGEDET_MB_BLOCK=0: the three separate ops);
            // SSD 27.5k -> 28.4k img/s with the 8-wave kernel (r3g); one wave per 16 channels since r3n
            if (env_int("EDGEDET_MB_BLOCK", 1) == 1 && !pack_only && !pf.pe.empty() && !b.se && b.cin <= 32 &&
                b.cin % 4 == 0 && b.cout <= 32 && b.exp <= 128)
                return mb_block(in, b, pf);
            Cur y = in;
            if (!pf.pe.empty()) y = conv(y, pf.pe, b.exp, 1, 1, b.act);
            DwOut d = dw(y, pf.pd, b.k, b.stride, b.act, b.se);
            Ref scale = b.se ? se(d, pf.ps) : Ref();
            Ref res = (b.stride == 1 && b.cin == b.cout) ? in.x : Ref();
            return conv(d.y, pf.pp, b.cout, 1, 1, A_NONE, res, scale);
        };

        int first = 0;
        if (stem_fuse) {
            ConvW w0 = cbn("backbone.features.0.0", 16, 3, 3, false, 4);
            Prefixes pf = block_prefixes(blocks_[0], "backbone.features.0.1.block");
            ConvW wd = cbn(pf.pd, 16, 16, 3, true);
            ConvW w1 = cbn(pf.pp, 16, 16, 1, false);
            const int64_t Ho = (S - 1) / 2 + 1, Wo = Ho;
            std::vector<int64_t> ys = {B, Ho, Wo, 16};
            const int y = P.buf(ys, 4, "backbone.features.0.1" + sfx);
            OpRec o;
            o.kind = EDGEDET_OP_SSD_STEM;
            o.name = "transform+backbone.features.0.0+0.1";
            const int64_t iv[9] = {B, S, S, Ho, Wo, w0.Kpad, w1.Kpad, H, W};
            for (int j = 0; j < 9; ++j) o.i[j] = iv[j];
            o.p[u8 ? 9 : 8] = view(inp);  // the source image; the transform runs in the stem's loads
            for (int j = 0; j < 6; ++j) o.f[j] = 0.5f;
            o.p[1] = Plan::wref(w0.w);
            o.p[2] = Plan::wref(w0.b);
            o.p[3] = Plan::wref(wd.w);
            o.p[4] = Plan::wref(wd.b);
            o.p[5] = Plan::wref(w1.w);
            o.p[6] = Plan::wref(w1.b);
            o.p[7] = P.ref(y);
            P.add(o);
            cur = Cur{P.ref(y), ys};
            first = 1;
        } else {
            cur = conv(cur, "backbone.features.0.0", 16, 3, 2, A_HS, Ref(), Ref(), 4);
        }
        for (int i = first; i < 12; ++i)
            cur = inverted_residual(cur, blocks_[(size_t)i], "backbone.features.0." + std::to_string(i + 1) + ".block");
        const Block& b12 = blocks_[12];
        cur = conv(cur, "backbone.features.0.13", b12.exp, 1, 1, b12.act);
        std::vector<Cur> feats = {cur};
        DwOut d = dw(cur, "backbone.features.1.0.1", b12.k, b12.stride, b12.act, true);
        Ref scale = se(d, "backbone.features.1.0.2");
        cur = conv(d.y, "backbone.features.1.0.3", b12.cout, 1, 1, A_NONE, Ref(), scale);
        for (int i : {13, 14})
            cur = inverted_residual(cur, blocks_[(size_t)i], "backbone.features.1." + std::to_string(i - 12) + ".block");
        const int c4 = blocks_[14].cout;
        cur = conv(cur, "backbone.features.1.3", 6 * c4, 1, 1, A_HS);
        feats.push_back(cur);
        const int outs[4] = {512, 256, 256, 128};
        for (int e = 0; e < 4; ++e) {
            const std::string p = "backbone.extra." + std::to_string(e);
            cur = conv(cur, p + ".0", outs[e] / 2, 1, 1, A_R6);
            cur = dw(cur, p + ".1", 3, 2, A_R6, false).y;
            cur = conv(cur, p + ".2", outs[e], 1, 1, A_R6);
            feats.push_back(cur);
        }
        std::vector<std::pair<int, int>> grids;
        int64_t A = 0;
        for (auto& f : feats) {
            grids.push_back({(int)f.s[1], (int)f.s[2]});
            A += f.s[1] * f.s[2] * 6;
        }
        if (sh.cls < 0) {
            sh.cls = P.buf({Btot, A, NC}, 4, "cls_logits");
            sh.reg = P.buf({Btot, A, 4}, 4, "bbox_regression");
        }
        // SSDLiteHead: per map a depthwise 3x3 (+BN, ReLU6) then a 1x1 conv with bias, for the cls and
        // the reg branch.  The weights are packed in the module order (map, branch); the records run as
        // two grouped launches (EDGEDET_OP_GROUP): the twelve depthwise convs, then the twelve 1x1
        // convs, which store straight into the concatenated head tensors (pixel stride 6 * cols, map
        // anchor offset) -- 24 sequential launches per chain become 2: SSD 28.97k / 28.71k -> 30.75k / 30.84k
        // img/s (alternated 750-step runs, profiles/r4b_ab_heads.txt).
        struct HeadOp {
            std::string p;
            int64_t cols, off;
            int out;
            const Cur* f;
        };
        std::vector<HeadOp> hops;
        int64_t off = 0;
        for (size_t i = 0; i < feats.size(); ++i) {
            const Cur& f = feats[i];
            for (int h = 0; h < 2; ++h) {
                const std::string name = h == 0 ? "classification_head" : "regression_head";
                const int64_t cols = h == 0 ? NC : 4;
                const std::string p = "head." + name + ".module_list." + std::to_string(i);
                cbn(p + ".0", f.s[3], f.s[3], 3, true);  // pack order: module order
                pk_.conv_bias(p + ".1.weight", p + ".1.bias", 6 * cols, f.s[3], 1);
                hops.push_back({p, cols, off, h == 0 ? sh.cls : sh.reg, &f});
            }
            off += f.s[1] * f.s[2] * 6;
        }
        const int ng = (int)hops.size();
        auto group = [&](const std::string& name) {
            OpRec g;
            g.kind = EDGEDET_OP_GROUP;
            g.name = name + sfx;
            g.i[0] = ng;
            P.add(g);
        };
        std::vector<Cur> hdw;
        group("head.depthwise");
        for (auto& h : hops) hdw.push_back(dw(*h.f, h.p + ".0", 3, 1, A_R6, false).y);
        group("head.pointwise");
        for (int k = 0; k < ng; ++k) {
            const HeadOp& h = hops[(size_t)k];
            const Cur& f = *h.f;
            ConvW w = pk_.conv_bias(h.p + ".1.weight", h.p + ".1.bias", 6 * h.cols, f.s[3], 1);
            ConvArgs a;
            a.x = hdw[(size_t)k].x;
            a.xs = hdw[(size_t)k].s;
            a.w = w;
            a.cout = 6 * h.cols;
            a.k = 1;
            a.y = P.ref(h.out);
            a.ys = {B, f.s[1], f.s[2], 6 * h.cols};
            a.y_pstride = 6 * h.cols;
            a.y_bstride = A * h.cols;
            a.y_off = (int64_t)img0 * A * h.cols + h.off * h.cols;
            a.tile = env_is("EDGEDET_CONV_MATH", "f32", "bf16x6") ? 0 : HEAD_TILE;  // f32: alone
            a.name = h.p + ".1" + sfx;
            conv_op(P, a);
        }
        if (pack_only) return;

        if (sh.anchors < 0) {
            sh.anchors = P.cnst(ssd_default_boxes(grids, S), {A, 4}, "anchors");
            sh.scores_t = P.buf({Btot, NC, A}, 4, "scores_t");
            sh.boxes = P.buf({Btot, A, 4}, 4, "boxes");
            std::vector<float> ratio;
            for (int b = 0; b < Btot; ++b) {
                ratio.push_back((float)W / (float)S);
                ratio.push_back((float)H / (float)S);
            }
            sh.ratio = P.cnst(ratio, {Btot, 2}, "ratio");
            sh.ob = P.buf({Btot, DETS, 4}, 4, "out.boxes");
            sh.os = P.buf({Btot, DETS}, 4, "out.scores");
            sh.ol = P.buf({Btot, DETS}, 8, "out.labels");
            sh.oc = P.buf({Btot}, I32, "out.count");
        }
        {
            OpRec o;
            o.kind = EDGEDET_OP_SSD_SCORES;
            o.name = "postprocess.scores" + sfx;
            o.i[0] = B;
            o.i[1] = A;
            o.i[2] = NC;
            o.p[0] = view(sh.cls);
            o.p[1] = view(sh.reg);
            o.p[2] = P.ref(sh.anchors);
            o.p[3] = view(sh.scores_t);
            o.p[4] = view(sh.boxes);
            o.f[0] = (float)S;
            o.f[1] = (float)S;
            P.add(o);
        }
        const int64_t NS = NC - 1, KM = TOPK;
        // shapes past the image-greedy kernel's limits: per-(image, class) NMS on every class's top-k,
        // then the per-image merge
        if (NS * KM <= 512 * 54 && DETS <= 1024) {
            const int pk = P.buf({B, NS, KM}, I32, "pool.key" + sfx);
            const int pr = P.buf({B, NS, KM}, I32, "pool.ref" + sfx);
            OpRec o;
            o.kind = EDGEDET_OP_SSD_POSTPROCESS;
            o.name = "postprocess.nms" + sfx;
            const int64_t iv[5] = {B, A, NC, KM, DETS};
            for (int j = 0; j < 5; ++j) o.i[j] = iv[j];
            o.i[5] = 0;  // class selection: the four-wave block form (1: the one-wave form, unit tests)
            o.p[0] = view(sh.scores_t);
            o.p[1] = view(sh.boxes);
            o.p[2] = P.ref(pk);
            o.p[3] = P.ref(pr);
            o.p[4] = view(sh.ratio);
            o.p[5] = view(sh.ob);
            o.p[6] = view(sh.os);
            o.p[7] = view(sh.ol);
            o.p[8] = view(sh.oc);
            o.f[0] = (float)SCORE;
            o.d[0] = NMS;
            P.add(o);
        } else {
            const int rb = P.buf({B, NS, KM, 4}, 4, "rec.box" + sfx), rs = P.buf({B, NS, KM}, 4, "rec.score" + sfx);
            const int rt = P.buf({B, NS, KM}, I32, "rec.tb" + sfx), rl = P.buf({B, NS, KM}, I32, "rec.label" + sfx);
            const int rc = P.buf({B, NS}, I32, "rec.count" + sfx);
            OpRec o;
            o.kind = EDGEDET_OP_SSD_CLASS_NMS;
            o.name = "postprocess.class_nms" + sfx;
            const int64_t iv[5] = {B, A, NC, TOPK, KM};
            for (int j = 0; j < 5; ++j) o.i[j] = iv[j];
            o.p[0] = view(sh.scores_t);
            o.p[1] = view(sh.boxes);
            o.p[2] = P.ref(rb);
            o.p[3] = P.ref(rs);
            o.p[4] = P.ref(rt);
            o.p[5] = P.ref(rl);
            o.p[6] = P.ref(rc);
            o.f[0] = (float)SCORE;
            o.d[0] = NMS;
            P.add(o);
            OpRec m;
            m.kind = EDGEDET_OP_MERGE_TOPK;
            m.name = "postprocess.merge" + sfx;
            const int64_t mv[4] = {B, NS, KM, DETS};
            for (int j = 0; j < 4; ++j) m.i[j] = mv[j];
            m.p[0] = P.ref(rb);
            m.p[1] = P.ref(rs);
            m.p[2] = P.ref(rt);
            m.p[3] = P.ref(rl);
            m.p[4] = P.ref(rc);
            m.p[5] = view(sh.ratio);
            m.p[6] = view(sh.ob);
            m.p[7] = view(sh.os);
            m.p[8] = view(sh.ol);
            m.p[9] = view(sh.oc);
            P.add(m);
        }
    }

    void se_weights(const std::string& p, int64_t C, int64_t S_, WRef& w1, WRef& b1, WRef& w2t, WRef& b2) {
        auto key = "se:" + p;
        auto it = se_.find(key);
        if (it != se_.end()) {
            w1 = it->second[0];
            b1 = it->second[1];
            w2t = it->second[2];
            b2 = it->second[3];
            return;
        }
        std::vector<float> a1((size_t)(S_ * C)), c1((size_t)S_), a2t((size_t)(S_ * C)), c2((size_t)C);
        const Params& P = pk_.params();
        if (pk_.values()) {
            const float* f1 = P.get(p + ".fc1.weight", S_ * C);  // [S][C][1][1]
            const float* f2 = P.get(p + ".fc2.weight", C * S_);  // [C][S][1][1]
            std::memcpy(a1.data(), f1, a1.size() * 4);
            std::memcpy(c1.data(), P.get(p + ".fc1.bias", S_), c1.size() * 4);
            for (int64_t cc = 0; cc < C; ++cc)
                for (int64_t s = 0; s < S_; ++s) a2t[(size_t)(s * C + cc)] = f2[cc * S_ + s];
            std::memcpy(c2.data(), P.get(p + ".fc2.bias", C), c2.size() * 4);
        }
        w1 = pk_.raw(key + ".w1", a1);
        b1 = pk_.raw(key + ".b1", c1);
        w2t = pk_.raw(key + ".w2t", a2t);
        b2 = pk_.raw(key + ".b2", c2);
        se_[key] = {w1, b1, w2t, b2};
    }

    Config cfg_;
    Packer& pk_;
    std::vector<Block> blocks_;
    std::map<std::string, std::vector<WRef>> se_;
};

// ------------------------------------------------------------------------------------ Faster R-CNN
// Shared by Faster R-CNN and RetinaNet (models.FasterRCNNFPNv2._lower_body): GeneralizedRCNNTransform
// (min 800 / max 1333, ImageNet mean / std, pad to /32) and the ResNet-50 body C2..C5.
class ResNetFPN {
  public:
    static constexpr double EPS = 1e-5;
    static constexpr int MIN_SIZE = 800, MAX_SIZE = 1333, DIV = 32;

    ResNetFPN(const Config& c, Packer& pk) : cfg_(c), pk_(pk) {}
    virtual ~ResNetFPN() = default;

    // [TV] GeneralizedRCNNTransform resize (detect.py:78): the scale is a float32 tensor
    // op, min(800. / min_f32, 1333. / max_f32), where `float / Tensor` is reciprocal(t) * x; the sizes
    // are floor(side * double(scale)) (recompute_scale_factor=True). volatile keeps each fp32 rounding.
    static void resized_size(int H, int W, int& Ho, int& Wo) {
        volatile float rmin = 1.0f / (float)std::min(H, W), rmax = 1.0f / (float)std::max(H, W);
        volatile float a = rmin * (float)MIN_SIZE, b = rmax * (float)MAX_SIZE;
        const double scale = (double)std::min((float)a, (float)b);
        Ho = (int)std::floor(H * scale);
        Wo = (int)std::floor(W * scale);
    }

  protected:
    // options of one conv (models.FasterRCNNFPNv2._lower_body.conv): BatchNorm prefix, or a bias key,
    // or neither (no bias: RetinaNet GroupNorm towers); fused input transform; strided output
    struct COpt {
        std::string bnp, bias_key, name;
        Ref res, in_scale, in_shift;
        int res_h = -1, res_w = -1;
        int64_t cin_pad = 0;
        bool in_relu = false;
        int out = -1;  // store into this buffer (pixel stride out_p, batch stride out_b, element offset out_off)
        int64_t out_p = -1, out_b = -1, out_off = 0;
        int tile = 0;  // 0 = the tuned table's
    };

    Cur conv(Plan& P, const Cur& in, const std::string& wkey, int64_t cout, int k, int stride, int act,
             const COpt& o) {
        ConvW w;
        if (!o.bias_key.empty())
            w = pk_.conv_bias(wkey, o.bias_key, cout, in.s[3], k);
        else if (o.bnp.empty())
            w = pk_.conv_nobias(wkey, cout, in.s[3], k);
        else
            w = pk_.conv_bn(wkey, o.bnp, EPS, cout, o.cin_pad ? 3 : in.s[3], k, false, o.cin_pad);
        const int pad = (k - 1) / 2;
        const int64_t Ho_ = (in.s[1] + 2 * pad - k) / stride + 1, Wo_ = (in.s[2] + 2 * pad - k) / stride + 1;
        std::vector<int64_t> ys = {in.s[0], Ho_, Wo_, cout};
        const int y = o.out >= 0 ? o.out : P.buf(ys, 4, o.name.empty() ? wkey : o.name);
        ConvArgs a;
        a.x = in.x;
        a.xs = in.s;
        a.w = w;
        a.cout = cout;
        a.k = k;
        a.stride = stride;
        a.pad = pad;
        a.act = act;
        a.y = P.ref(y);
        a.ys = ys;
        a.res = o.res;
        a.res_h = o.res_h;
        a.res_w = o.res_w;
        a.in_relu = o.in_relu;
        a.in_scale = o.in_scale;
        a.in_shift = o.in_shift;
        a.name = o.name.empty() ? wkey : o.name;
        a.tile = o.tile;
        if (o.out >= 0) {
            a.y_pstride = o.out_p;
            a.y_bstride = o.out_b;
            a.y_off = o.out_off;
        }
        conv_op(P, a);
        return Cur{P.ref(y), ys};
    }
    Cur conv_bn(Plan& P, const Cur& in, const std::string& wkey, const std::string& bnp, int64_t cout, int k,
                int stride, int act, Ref res = Ref(), int res_h = -1, int res_w = -1, bool in_relu = false) {
        COpt o;
        o.bnp = bnp;
        o.res = res;
        o.res_h = res_h;
        o.res_w = res_w;
        o.in_relu = in_relu;
        return conv(P, in, wkey, cout, k, stride, act, o);
    }
    Cur conv_b(Plan& P, const Cur& in, const std::string& p, int64_t cout, int k, int stride, int act,
               const std::string& name = "", Ref res = Ref(), int res_h = -1, int res_w = -1, bool in_relu = false) {
        COpt o;
        o.bias_key = p + ".bias";
        o.name = name;
        o.res = res;
        o.res_h = res_h;
        o.res_w = res_w;
        o.in_relu = in_relu;
        return conv(P, in, p + ".weight", cout, k, stride, act, o);
    }
    Cur maxpool(Plan& P, const Cur& in, int k, int stride, int pad, const std::string& name) {
        const int64_t Ho_ = (in.s[1] + 2 * pad - k) / stride + 1, Wo_ = (in.s[2] + 2 * pad - k) / stride + 1;
        std::vector<int64_t> ys = {in.s[0], Ho_, Wo_, in.s[3]};
        const int y = P.buf(ys, 4, name);
        OpRec o;
        o.kind = EDGEDET_OP_MAXPOOL;
        o.name = name;
        const int64_t iv[9] = {in.s[0], in.s[1], in.s[2], in.s[3], Ho_, Wo_, k, stride, pad};
        for (int j = 0; j < 9; ++j) o.i[j] = iv[j];
        o.p[0] = in.x;
        o.p[1] = P.ref(y);
        P.add(o);
        return Cur{P.ref(y), ys};
    }

    struct Body {
        int inp = -1, Ho = 0, Wo = 0, Hp = 0, Wp = 0;
        std::vector<Cur> cs;  // C2..C5
    };
    Body body(Plan& P, int B, int H, int W, bool u8) {
        Body r;
        resized_size(H, W, r.Ho, r.Wo);
        r.Hp = (r.Ho + DIV - 1) / DIV * DIV;
        r.Wp = (r.Wo + DIV - 1) / DIV * DIV;
        r.inp = P.buf({B, 3, H, W}, u8 ? 1 : 4, "images");
        const int x = P.buf({B, r.Hp, r.Wp, 4}, 4, "pre");
        {
            OpRec o;
            o.kind = EDGEDET_OP_PREPROCESS;
            o.name = "transform";
            const int64_t iv[7] = {B, H, W, r.Ho, r.Wo, r.Hp, r.Wp};
            for (int j = 0; j < 7; ++j) o.i[j] = iv[j];
            o.p[u8 ? 2 : 0] = P.ref(r.inp);
            o.p[1] = P.ref(x);
            const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
            for (int j = 0; j < 3; ++j) {
                o.f[j] = mean[j];
                o.f[3 + j] = stdv[j];
            }
            P.add(o);
        }
        Cur cur{P.ref(x), {B, r.Hp, r.Wp, 4}};
        const std::string pb = "backbone.body.";
        {
            COpt o;
            o.bnp = pb + "bn1";
            o.cin_pad = 4;
            cur = conv(P, cur, pb + "conv1.weight", 64, 7, 2, A_RE, o);
        }
        cur = maxpool(P, cur, 3, 2, 1, "backbone.body.maxpool");
        // deep-K 3x3 convs on small maps fill the GPU only with split-K (tile 26), which cannot apply the
        // ReLU: conv3 then applies it to its input
        const char* lname[4] = {"layer1", "layer2", "layer3", "layer4"};
        const int nblk[4] = {3, 4, 6, 3}, width[4] = {64, 128, 256, 512}, lstride[4] = {1, 2, 2, 2};
        for (int L = 0; L < 4; ++L) {
            for (int bi = 0; bi < nblk[L]; ++bi) {
                const std::string q = pb + lname[L] + "." + std::to_string(bi) + ".";
                const int s = bi == 0 ? lstride[L] : 1;
                const int wd = width[L];
                Cur y = conv_bn(P, cur, q + "conv1.weight", q + "bn1", wd, 1, 1, A_RE);
                const int64_t m = y.s[0] * ((y.s[1] - 1) / s + 1) * ((y.s[2] - 1) / s + 1);
                const bool defer = 9 * wd >= 2048 && ((m + 255) / 256) * ((wd + 127) / 128) < 200;
                y = conv_bn(P, y, q + "conv2.weight", q + "bn2", wd, 3, s, defer ? A_NONE : A_RE);
                Cur idn = bi == 0 ? conv_bn(P, cur, q + "downsample.0.weight", q + "downsample.1", wd * 4, 1, s, A_NONE)
                                  : cur;
                cur = conv_bn(P, y, q + "conv3.weight", q + "bn3", wd * 4, 1, 1, A_RE, idn.x, -1, -1, defer);
            }
            r.cs.push_back(cur);
        }
        return r;
    }

    Config cfg_;
    Packer& pk_;
};

// anchors.rpn_anchors / retina_anchors: per level [gh*gw*A, 4], order (y, x, a), a ratio-major over the
// level's scales; strides = image_size // grid
static std::vector<float> grid_anchors(int gh, int gw, int Hp, int Wp, const std::vector<int>& scales) {
    const float ratios[3] = {0.5f, 1.0f, 2.0f};
    std::vector<std::array<float, 4>> base;
    for (int a = 0; a < 3; ++a) {
        const float hr = std::sqrt(ratios[a]);
        const float wr = 1.0f / hr;
        for (int sc : scales) {
            const float ws = wr * (float)sc, hs = hr * (float)sc;
            const float v[4] = {-ws / 2.0f, -hs / 2.0f, ws / 2.0f, hs / 2.0f};
            std::array<float, 4> b;
            for (int j = 0; j < 4; ++j) b[(size_t)j] = std::nearbyint(v[j]);  // round half to even, as torch.round
            base.push_back(b);
        }
    }
    const int sh = Hp / gh, sw = Wp / gw;
    std::vector<float> out;
    out.reserve((size_t)gh * gw * base.size() * 4);
    for (int y = 0; y < gh; ++y)
        for (int x = 0; x < gw; ++x)
            for (auto& b : base) {
                const float fx = (float)((int64_t)x * sw), fy = (float)((int64_t)y * sh);
                out.push_back(fx + b[0]);
                out.push_back(fy + b[1]);
                out.push_back(fx + b[2]);
                out.push_back(fy + b[3]);
            }
    return out;
}

class FasterRCNN : public ResNetFPN {
  public:
    static constexpr int RPN_PRE = 1000, RPN_POST = 1000, BOX_DETS = 100;
    static constexpr int RPN_TILE = 39;  // the grouped RPN head 3x3 convs (Cout = 256): 128 x 256
    static constexpr int RPN_CHUNK = 8192;  // anchors per chunk of the chunked RPN top-k
    static constexpr double RPN_NMS = 0.7, RPN_MIN = 1e-3, RPN_SCORE = 0.0, BOX_SCORE = 0.05, BOX_NMS = 0.5,
                            BOX_MIN = 1e-2;

    FasterRCNN(const Config& c, Packer& pk) : ResNetFPN(c, pk) {}

    void pack_all() { lower(1, MIN_SIZE, MIN_SIZE, false, true); }

    std::unique_ptr<Plan> lower(int B, int H, int W, bool u8, bool pack_only = false) {
        auto Pp = std::make_unique<Plan>();
        Plan& P = *Pp;
        const int NC = cfg_.num_classes;
        Body bd = body(P, B, H, W, u8);
        const int Ho = bd.Ho, Wo = bd.Wo, Hp = bd.Hp, Wp = bd.Wp;
        const std::vector<Cur>& cs = bd.cs;

        // ---- FPN + LastLevelMaxPool
        const std::string f = "backbone.fpn.";
        Cur last = conv_bn(P, cs[3], f + "inner_blocks.3.0.weight", f + "inner_blocks.3.1", 256, 1, 1, A_NONE);
        std::vector<Cur> outs = {conv_bn(P, last, f + "layer_blocks.3.0.weight", f + "layer_blocks.3.1", 256, 3, 1, A_NONE)};
        for (int i : {2, 1, 0}) {
            const std::string si = std::to_string(i);
            last = conv_bn(P, cs[(size_t)i], f + "inner_blocks." + si + ".0.weight", f + "inner_blocks." + si + ".1", 256,
                           1, 1, A_NONE, last.x, (int)last.s[1], (int)last.s[2]);
            outs.insert(outs.begin(), conv_bn(P, last, f + "layer_blocks." + si + ".0.weight",
                                              f + "layer_blocks." + si + ".1", 256, 3, 1, A_NONE));
        }
        outs.push_back(maxpool(P, outs.back(), 1, 2, 0, "backbone.fpn.extra_blocks.pool"));
        if (pack_only) {
            for (const char* k : {"rpn.head.conv.0.0", "rpn.head.conv.1.0"})
                pk_.conv_bias(std::string(k) + ".weight", std::string(k) + ".bias", 256, 256, 3);
            pk_.conv_bias("rpn.head.cls_logits.weight", "rpn.head.cls_logits.bias", 3, 256, 1);
            pk_.conv_bias("rpn.head.bbox_pred.weight", "rpn.head.bbox_pred.bias", 12, 256, 1);
            for (int i = 0; i < 4; ++i) {
                const std::string p = "roi_heads.box_head." + std::to_string(i);
                pk_.conv_bn(p + ".0.weight", p + ".1", EPS, 256, 256, 3, false);
            }
            fc6();
            predictor();
            return Pp;
        }

        // ---- RPN head (shared over levels) + proposal filtering
        const int Aa = 3;
        std::vector<std::pair<Ref, Ref>> heads;
        std::vector<std::pair<int, int>> grids;
        // The shared 3x3 convs of the five levels as two grouped launches (EDGEDET_OP_GROUP): each 3x3
        // conv of every level in one launch on the P2 level's tile, so the small levels' workgroups fill
        // the big level's tail instead of running as eight latency-bound launches after it (round 3 ran
        // the levels one after another on the caller stream; on four stream lanes was 0.75 % slower).
        const int L5 = (int)outs.size();
        auto rpn_group = [&](const std::string& name) {
            OpRec g;
            g.kind = EDGEDET_OP_GROUP;
            g.name = name;
            g.i[0] = L5;
            P.add(g);
        };
        const bool grouped = !env_is("EDGEDET_CONV_MATH", "f32", "bf16x6");  // grouped launches: bf16x6 tiles
        std::vector<Cur> t0s, t1s;
        if (grouped) rpn_group("rpn.head.conv.0");
        for (int lvl = 0; lvl < L5; ++lvl) {
            COpt o;
            o.bias_key = "rpn.head.conv.0.0.bias";
            o.name = "rpn.head.conv.0@" + std::to_string(lvl);
            o.tile = grouped ? RPN_TILE : 0;
            t0s.push_back(conv(P, outs[(size_t)lvl], "rpn.head.conv.0.0.weight", 256, 3, 1, A_RE, o));
        }
        if (grouped) rpn_group("rpn.head.conv.1");
        for (int lvl = 0; lvl < L5; ++lvl) {
            COpt o;
            o.bias_key = "rpn.head.conv.1.0.bias";
            o.name = "rpn.head.conv.1@" + std::to_string(lvl);
            o.tile = grouped ? RPN_TILE : 0;
            t1s.push_back(conv(P, t0s[(size_t)lvl], "rpn.head.conv.1.0.weight", 256, 3, 1, A_RE, o));
        }
        for (int lvl = 0; lvl < L5; ++lvl) {
            const std::string at = "@" + std::to_string(lvl);
            const Cur& t = t1s[(size_t)lvl];
            Cur o = conv_b(P, t, "rpn.head.cls_logits", 3, 1, 1, A_NONE, "rpn.head.cls_logits" + at);
            Cur d = conv_b(P, t, "rpn.head.bbox_pred", 12, 1, 1, A_NONE, "rpn.head.bbox_pred" + at);
            heads.push_back({o.x, d.x});
            grids.push_back({(int)outs[(size_t)lvl].s[1], (int)outs[(size_t)lvl].s[2]});
        }
        std::vector<int> anchor_bufs;
        const int sizes[5] = {32, 64, 128, 256, 512};
        for (size_t l = 0; l < grids.size(); ++l) {
            auto a = grid_anchors(grids[l].first, grids[l].second, Hp, Wp, {sizes[l]});
            anchor_bufs.push_back(P.cnst(a, {(int64_t)a.size() / 4, 4}, "rpn.anchors@" + std::to_string(l)));
        }
        const int L = (int)outs.size();
        const int KM = RPN_PRE;
        const int rb = P.buf({B, L, KM, 4}, 4, "rpn.rec.box"), rs = P.buf({B, L, KM}, 4, "rpn.rec.score");
        const int rt = P.buf({B, L, KM}, I32, "rpn.rec.tb"), rl = P.buf({B, L, KM}, I32, "rpn.rec.lvl");
        const int rc = P.buf({B, L}, I32, "rpn.rec.count");
        {
            OpRec o;
            o.kind = EDGEDET_OP_RPN_LEVEL_NMS;
            o.name = "rpn.filter_proposals";
            const int64_t iv[6] = {B, L, 0, Aa, RPN_PRE, KM};
            for (int j = 0; j < 6; ++j) o.i[j] = iv[j];
            for (int l = 0; l < L; ++l) {
                o.i[6 + l] = (int64_t)grids[(size_t)l].first * grids[(size_t)l].second * Aa;
                o.p[l] = heads[(size_t)l].first;
                o.p[15 + l] = heads[(size_t)l].second;
                o.p[5 + l] = P.ref(anchor_bufs[(size_t)l]);
            }
            const int recs[5] = {rb, rs, rt, rl, rc};
            for (int j = 0; j < 5; ++j) o.p[10 + j] = P.ref(recs[j]);
            o.f[0] = (float)Ho;
            o.f[1] = (float)Wo;
            o.f[2] = (float)RPN_MIN;
            o.f[3] = (float)RPN_SCORE;
            o.d[0] = RPN_NMS;
            // chunked top-k: 8,192 anchors per chunk (P2 of an 800 x 800 image: 15 chunks per image)
            int64_t nmax = 0;
            for (int l = 0; l < L; ++l) nmax = std::max<int64_t>(nmax, o.i[6 + l]);
            const int64_t chunk = RPN_CHUNK, nch = (nmax + chunk - 1) / chunk;
            o.p[20] = P.ref(P.buf({B, L, nch, 1024}, I32, "rpn.chunk.key"));
            o.p[21] = P.ref(P.buf({B, L, nch, 1024}, I32, "rpn.chunk.idx"));
            o.p[22] = P.ref(P.buf({B, L, nch}, I32, "rpn.chunk.count"));
            o.i[16] = chunk;
            o.i[17] = nch;
            // split NMS (selection / IoU mask over many workgroups / scan): EDGEDET_RPN_SPLIT=0 keeps one
            // workgroup per (level, image) for the whole segment
            if (env_int("EDGEDET_RPN_SPLIT", 1))
                o.p[23] = P.ref(P.buf({rpn_split_bytes((int64_t)B * L)}, 1, "rpn.nms.split"));
            P.add(o);
        }
        const int R = RPN_POST;
        const int props = P.buf({B, R, 4}, 4, "proposals"), pscore = P.buf({B, R}, 4, "proposal_scores");
        const int pcount = P.buf({B}, I32, "proposal_count");
        {
            OpRec o;
            o.kind = EDGEDET_OP_MERGE_TOPK;
            o.name = "rpn.post_nms_top_n";
            const int64_t iv[4] = {B, L, KM, R};
            for (int j = 0; j < 4; ++j) o.i[j] = iv[j];
            const int recs[5] = {rb, rs, rt, rl, rc};
            for (int j = 0; j < 5; ++j) o.p[j] = P.ref(recs[j]);
            o.p[5] = Ref();
            o.p[6] = P.ref(props);
            o.p[7] = P.ref(pscore);
            o.p[8] = Ref();
            o.p[9] = P.ref(pcount);
            P.add(o);
        }

        // ---- MultiScaleRoIAlign
        const int C = 256;
        const int roi = P.buf({(int64_t)B * R, 7, 7, C}, 4, "box_roi_pool");
        {
            OpRec o;
            o.kind = EDGEDET_OP_ROI_ALIGN;
            o.name = "roi_heads.box_roi_pool";
            const int64_t iv[11] = {1, (int64_t)B * R, R, B, C, 7, 7, 2, 4, 2, 5};
            for (int j = 0; j < 11; ++j) o.i[j] = iv[j];
            o.p[4] = P.ref(props);
            o.p[5] = P.ref(pcount);
            o.p[6] = P.ref(roi);
            for (int l = 0; l < 4; ++l) {
                const int fh = (int)outs[(size_t)l].s[1], fw = (int)outs[(size_t)l].s[2];
                o.i[11 + l] = fh;
                o.i[15 + l] = fw;
                o.p[l] = outs[(size_t)l].x;
                // MultiScaleRoIAlign._infer_scale: 2 ** round(log2(feat / image)) in float32
                const float r = (float)((double)fh / (double)Ho);
                o.f[l] = (float)std::pow(2.0, (double)std::nearbyint(std::log2(r)));
            }
            P.add(o);
        }

        // ---- box head + predictor
        Cur bc{P.ref(roi), {(int64_t)B * R, 7, 7, C}};
        for (int i = 0; i < 4; ++i) {
            const std::string p = "roi_heads.box_head." + std::to_string(i);
            bc = conv_bn(P, bc, p + ".0.weight", p + ".1", 256, 3, 1, A_RE);
        }
        {
            ConvW w = fc6();
            const int fc = P.buf({(int64_t)B * R, 1024}, 4, "roi_heads.box_head.5");
            ConvArgs a;
            a.x = bc.x;
            a.xs = {(int64_t)B * R, 1, 1, 7 * 7 * C};
            a.w = w;
            a.cout = 1024;
            a.act = A_RE;
            a.y = P.ref(fc);
            a.ys = {(int64_t)B * R, 1, 1, 1024};
            a.name = "roi_heads.box_head.5";
            conv_op(P, a);
            ConvW wp = predictor();
            const int LD = 456;
            const int pred = P.buf({(int64_t)B * R, LD}, 4, "box_predictor");
            ConvArgs b;
            b.x = P.ref(fc);
            b.xs = {(int64_t)B * R, 1, 1, 1024};
            b.w = wp;
            b.cout = 5 * NC;
            b.y = P.ref(pred);
            b.ys = {(int64_t)B * R, 1, 1, 5 * NC};
            b.y_pstride = LD;
            b.y_bstride = LD;
            b.name = "roi_heads.box_predictor";
            conv_op(P, b);

            // ---- RoIHeads.postprocess_detections
            const int scores = P.buf({B, R, NC}, 4, "box_scores");
            const int bxs = P.buf({B, R, NC, 4}, 4, "box_decoded");
            OpRec o;
            o.kind = EDGEDET_OP_BOX_SCORES;
            o.name = "roi_heads.scores_decode";
            const int64_t iv[6] = {LD, B, R, NC, 4 * NC, 0};
            for (int j = 0; j < 6; ++j) o.i[j] = iv[j];
            o.p[0] = P.ref(pred);
            o.p[1] = P.ref(props);
            o.p[2] = P.ref(pcount);
            o.p[3] = P.ref(scores);
            o.p[4] = P.ref(bxs);
            o.f[0] = (float)Ho;
            o.f[1] = (float)Wo;
            P.add(o);
            const int NS = NC - 1;
            const int b0 = P.buf({B, NS, R, 4}, 4, "box.rec.box"), b1 = P.buf({B, NS, R}, 4, "box.rec.score");
            const int b2 = P.buf({B, NS, R}, I32, "box.rec.tb"), b3 = P.buf({B, NS, R}, I32, "box.rec.lbl");
            const int b4 = P.buf({B, NS}, I32, "box.rec.count");
            OpRec n;
            n.kind = EDGEDET_OP_BOX_CLASS_NMS;
            n.name = "roi_heads.class_nms";
            const int64_t nv[4] = {B, R, NC, R};
            for (int j = 0; j < 4; ++j) n.i[j] = nv[j];
            n.p[0] = P.ref(scores);
            n.p[1] = P.ref(bxs);
            n.p[2] = P.ref(pcount);
            const int brec[5] = {b0, b1, b2, b3, b4};
            for (int j = 0; j < 5; ++j) n.p[3 + j] = P.ref(brec[j]);
            n.f[0] = (float)BOX_SCORE;
            n.f[1] = (float)BOX_MIN;
            n.d[0] = BOX_NMS;
            P.add(n);
            std::vector<float> ratio;
            for (int b = 0; b < B; ++b) {
                ratio.push_back((float)W / (float)Wo);
                ratio.push_back((float)H / (float)Ho);
            }
            const int rbuf = P.cnst(ratio, {B, 2}, "ratio");
            const int N = BOX_DETS;
            P.out_box = P.buf({B, N, 4}, 4, "out.boxes");
            P.out_score = P.buf({B, N}, 4, "out.scores");
            P.out_label = P.buf({B, N}, 8, "out.labels");
            P.out_count = P.buf({B}, I32, "out.count");
            OpRec m;
            m.kind = EDGEDET_OP_MERGE_TOPK;
            m.name = "roi_heads.detections_per_img";
            const int64_t mv[4] = {B, NS, R, N};
            for (int j = 0; j < 4; ++j) m.i[j] = mv[j];
            for (int j = 0; j < 5; ++j) m.p[j] = P.ref(brec[j]);
            m.p[5] = P.ref(rbuf);
            m.p[6] = P.ref(P.out_box);
            m.p[7] = P.ref(P.out_score);
            m.p[8] = P.ref(P.out_label);
            m.p[9] = P.ref(P.out_count);
            P.add(m);
        }
        P.input = bd.inp;
        P.dets = BOX_DETS;
        return Pp;
    }

  private:
    ConvW fc6() {
        const Params& P = pk_.params();
        std::vector<float> w, b(1024, 0.f);
        if (pk_.values()) {
            const float* src = P.get("roi_heads.box_head.5.weight", (int64_t)1024 * 12544);  // (c, h, w)
            w.assign((size_t)1024 * 12544, 0.f);
            for (int o = 0; o < 1024; ++o)
                for (int c = 0; c < 256; ++c)
                    for (int hw = 0; hw < 49; ++hw) w[(size_t)o * 12544 + (size_t)hw * 256 + c] = src[(size_t)o * 12544 + (size_t)c * 49 + hw];
            std::memcpy(b.data(), P.get("roi_heads.box_head.5.bias", 1024), 4096);
        } else {
            P.check("roi_heads.box_head.5.weight", (int64_t)1024 * 12544);
        }
        return pk_.conv_given("fc6", w, b, 1024, 12544, 1);
    }
    ConvW predictor() {
        const Params& P = pk_.params();
        const int NC = cfg_.num_classes;
        std::vector<float> w, b;
        if (pk_.values()) {
            const std::string q = "roi_heads.box_predictor.";
            const float* wb = P.get(q + "bbox_pred.weight", (int64_t)4 * NC * 1024);
            const float* wc = P.get(q + "cls_score.weight", (int64_t)NC * 1024);
            w.assign(wb, wb + (size_t)4 * NC * 1024);
            w.insert(w.end(), wc, wc + (size_t)NC * 1024);
            const float* bb = P.get(q + "bbox_pred.bias", 4 * NC);
            const float* bcl = P.get(q + "cls_score.bias", NC);
            b.assign(bb, bb + 4 * NC);
            b.insert(b.end(), bcl, bcl + NC);
        } else {
            b.assign((size_t)5 * NC, 0.f);
        }
        return pk_.conv_given("pred", w, b, 5 * NC, 1024, 1);
    }

};


// retinanet_resnet50_fpn_v2 (detect.py:34-38; models.RetinaNetFPNv2): the ResNet-50 body, FPN over
// C3..C5 (convs with bias, no norm) + LastLevelP6P7 (P6 on C5, P7 on relu(P6): the ReLU applied as P7's
// conv loads its input), GroupNorm(32) head towers whose normalised tensors are never written
// (GN_STATS -> per (image, channel) scale / shift applied, with the ReLU, by the next conv's A load),
// cls / box convs storing straight into the concatenated [B, sum(HWA), K] / [B, sum(HWA), 4] tensors.
class RetinaNet : public ResNetFPN {
  public:
    static constexpr int DETS = 300, TOPK = 1000, GROUPS = 32, A = 9;
    static constexpr double SCORE = 0.05, NMS = 0.5, GN_EPS = 1e-5;
    static constexpr int64_t SELECT_CHUNK = 1 << 16;

    RetinaNet(const Config& c, Packer& pk) : ResNetFPN(c, pk) {}

    void pack_all() { lower(1, MIN_SIZE, MIN_SIZE, false, true); }

    std::unique_ptr<Plan> lower(int B, int H, int W, bool u8, bool pack_only = false) {
        auto Pp = std::make_unique<Plan>();
        Plan& P = *Pp;
        const int K = cfg_.num_classes;
        Body bd = body(P, B, H, W, u8);
        const int Ho = bd.Ho, Wo = bd.Wo, Hp = bd.Hp, Wp = bd.Wp;
        const std::string f = "backbone.fpn.";
        const Cur &c3 = bd.cs[1], &c4 = bd.cs[2], &c5 = bd.cs[3];
        Cur last = conv_b(P, c5, f + "inner_blocks.2.0", 256, 1, 1, A_NONE, f + "inner_blocks.2.0.weight");
        std::vector<Cur> outs = {conv_b(P, last, f + "layer_blocks.2.0", 256, 3, 1, A_NONE, f + "layer_blocks.2.0.weight")};
        const std::pair<int, const Cur*> lat[2] = {{1, &c4}, {0, &c3}};
        for (auto& ic : lat) {
            const std::string si = std::to_string(ic.first);
            last = conv_b(P, *ic.second, f + "inner_blocks." + si + ".0", 256, 1, 1, A_NONE,
                          f + "inner_blocks." + si + ".0.weight", last.x, (int)last.s[1], (int)last.s[2]);
            outs.insert(outs.begin(), conv_b(P, last, f + "layer_blocks." + si + ".0", 256, 3, 1, A_NONE,
                                             f + "layer_blocks." + si + ".0.weight"));
        }
        Cur p6 = conv_b(P, c5, f + "extra_blocks.p6", 256, 3, 2, A_NONE, f + "extra_blocks.p6.weight");
        Cur p7 = conv_b(P, p6, f + "extra_blocks.p7", 256, 3, 2, A_NONE, f + "extra_blocks.p7.weight", Ref(), -1, -1,
                        true);
        outs.push_back(p6);
        outs.push_back(p7);
        const char* br_name[2] = {"classification_head", "regression_head"};
        const char* last_name[2] = {"cls_logits", "bbox_reg"};
        const int kk_of[2] = {K, 4};
        if (pack_only) {
            for (int h = 0; h < 2; ++h) {
                for (int i = 0; i < 4; ++i) {
                    const std::string q = std::string("head.") + br_name[h] + ".conv." + std::to_string(i);
                    pk_.conv_nobias(q + ".0.weight", 256, 256, 3);
                    gn(q + ".1");
                }
                const std::string lp = std::string("head.") + br_name[h] + "." + last_name[h];
                pk_.conv_bias(lp + ".weight", lp + ".bias", (int64_t)A * kk_of[h], 256, 3);
            }
            return Pp;
        }

        std::vector<std::pair<int, int>> grids;
        std::vector<int64_t> na, a0;
        int64_t Atot = 0;
        for (auto& o : outs) {
            grids.push_back({(int)o.s[1], (int)o.s[2]});
            na.push_back(o.s[1] * o.s[2] * A);
            a0.push_back(Atot);
            Atot += o.s[1] * o.s[2] * A;
        }
        const int cls = P.buf({B, Atot, K}, 4, "head.cls_logits");
        const int reg = P.buf({B, Atot, 4}, 4, "head.bbox_regression");
        const int64_t C = 256;
        P.fork(3);  // the five levels' head towers are independent
        for (size_t lvl = 0; lvl < outs.size(); ++lvl) {
            P.lane((int)(lvl % 4));
            const int64_t hw = outs[lvl].s[1] * outs[lvl].s[2];
            const std::string at = "@" + std::to_string(lvl);
            for (int h = 0; h < 2; ++h) {
                const int kk = kk_of[h];
                const int dst = kk == K ? cls : reg;
                Cur t = outs[lvl];
                Ref sc, sh;
                for (int i = 0; i < 4; ++i) {
                    const std::string q = std::string("head.") + br_name[h] + ".conv." + std::to_string(i) + ".";
                    COpt o;
                    o.in_scale = sc;
                    o.in_shift = sh;
                    o.in_relu = i > 0;
                    o.name = q + "0" + at;
                    t = conv(P, t, q + "0.weight", C, 3, 1, A_NONE, o);
                    WRef g, b;
                    gn(q + "1", &g, &b);
                    const int scb = P.buf({B, C}, 4, q + "1.scale" + at), shb = P.buf({B, C}, 4, q + "1.shift" + at);
                    OpRec s;
                    s.kind = EDGEDET_OP_GN_STATS;
                    s.name = q + "1" + at;
                    s.i[0] = B;
                    s.i[1] = hw;
                    s.i[2] = C;
                    s.i[3] = GROUPS;
                    s.p[0] = t.x;
                    s.p[1] = Plan::wref(g);
                    s.p[2] = Plan::wref(b);
                    s.p[3] = P.ref(scb);
                    s.p[4] = P.ref(shb);
                    s.f[0] = (float)GN_EPS;
                    P.add(s);
                    sc = P.ref(scb);
                    sh = P.ref(shb);
                }
                const std::string lp = std::string("head.") + br_name[h] + "." + last_name[h];
                COpt o;
                o.bias_key = lp + ".bias";
                o.in_scale = sc;
                o.in_shift = sh;
                o.in_relu = true;
                o.out = dst;
                o.out_p = (int64_t)A * kk;
                o.out_b = Atot * kk;
                o.out_off = a0[lvl] * kk;
                o.name = lp + at;
                conv(P, t, lp + ".weight", (int64_t)A * kk, 3, 1, A_NONE, o);
            }
        }
        P.join();
        std::vector<float> anchors;
        for (size_t l = 0; l < grids.size(); ++l) {
            const int x = 32 << l;
            const std::vector<int> scales = {x, (int)(x * std::pow(2.0, 1.0 / 3)), (int)(x * std::pow(2.0, 2.0 / 3))};
            auto a = grid_anchors(grids[l].first, grids[l].second, Hp, Wp, scales);
            anchors.insert(anchors.end(), a.begin(), a.end());
        }
        const int anc = P.cnst(anchors, {Atot, 4}, "anchors");

        // ---- RetinaNet.postprocess_detections
        const int L = (int)outs.size(), KM = TOPK;
        const int lrec[5] = {P.buf({B, L, KM, 4}, 4, "retina.cand.box"), P.buf({B, L, KM}, 4, "retina.cand.score"),
                             P.buf({B, L, KM}, I32, "retina.cand.tb"), P.buf({B, L, KM}, I32, "retina.cand.label"),
                             P.buf({B, L}, I32, "retina.cand.count")};
        int64_t nchunk = 0;
        for (int64_t n : na) nchunk = std::max<int64_t>(nchunk, (n * K + SELECT_CHUNK - 1) / SELECT_CHUNK);
        const int ck = P.buf({B, L, nchunk, 1024}, I32, "retina.chunk.key");
        const int ci = P.buf({B, L, nchunk, 1024}, I32, "retina.chunk.idx");
        const int cc = P.buf({B, L, nchunk}, I32, "retina.chunk.count");
        {
            OpRec o;
            o.kind = EDGEDET_OP_RETINA_SELECT;
            o.name = "retina.select_topk";
            const int64_t iv[6] = {B, L, Atot, K, TOPK, KM};
            for (int j = 0; j < 6; ++j) o.i[j] = iv[j];
            o.i[16] = SELECT_CHUNK;
            o.i[17] = nchunk;
            for (int l = 0; l < L; ++l) {
                o.i[6 + l] = a0[(size_t)l];
                o.i[11 + l] = na[(size_t)l];
            }
            o.p[0] = P.ref(cls);
            o.p[1] = P.ref(reg);
            o.p[2] = P.ref(anc);
            for (int j = 0; j < 5; ++j) o.p[3 + j] = P.ref(lrec[j]);
            o.p[8] = P.ref(ck);
            o.p[9] = P.ref(ci);
            o.p[10] = P.ref(cc);
            o.f[0] = (float)Ho;
            o.f[1] = (float)Wo;
            o.f[2] = (float)SCORE;
            P.add(o);
        }
        const int N = DETS;
        const int crec[5] = {P.buf({B, K, N, 4}, 4, "retina.kept.box"), P.buf({B, K, N}, 4, "retina.kept.score"),
                             P.buf({B, K, N}, I32, "retina.kept.tb"), P.buf({B, K, N}, I32, "retina.kept.lbl"),
                             P.buf({B, K}, I32, "retina.kept.count")};
        {
            OpRec o;
            o.kind = EDGEDET_OP_RETINA_CLASS_NMS;
            o.name = "retina.batched_nms";
            const int64_t iv[5] = {B, L, KM, K, N};
            for (int j = 0; j < 5; ++j) o.i[j] = iv[j];
            for (int j = 0; j < 5; ++j) {
                o.p[j] = P.ref(lrec[j]);
                o.p[5 + j] = P.ref(crec[j]);
            }
            o.d[0] = NMS;
            P.add(o);
        }
        std::vector<float> ratio;
        for (int b = 0; b < B; ++b) {
            ratio.push_back((float)W / (float)Wo);
            ratio.push_back((float)H / (float)Ho);
        }
        const int rbuf = P.cnst(ratio, {B, 2}, "ratio");
        P.out_box = P.buf({B, N, 4}, 4, "out.boxes");
        P.out_score = P.buf({B, N}, 4, "out.scores");
        P.out_label = P.buf({B, N}, 8, "out.labels");
        P.out_count = P.buf({B}, I32, "out.count");
        {
            OpRec m;
            m.kind = EDGEDET_OP_MERGE_TOPK;
            m.name = "retina.detections_per_img";
            const int64_t mv[4] = {B, K, N, N};
            for (int j = 0; j < 4; ++j) m.i[j] = mv[j];
            for (int j = 0; j < 5; ++j) m.p[j] = P.ref(crec[j]);
            m.p[5] = P.ref(rbuf);
            m.p[6] = P.ref(P.out_box);
            m.p[7] = P.ref(P.out_score);
            m.p[8] = P.ref(P.out_label);
            m.p[9] = P.ref(P.out_count);
            P.add(m);
        }
        P.input = bd.inp;
        P.dets = DETS;
        return Pp;
    }

  private:
    void gn(const std::string& p, WRef* g = nullptr, WRef* b = nullptr) {
        const Params& Pm = pk_.params();
        std::vector<float> w(256, 0.f), bb(256, 0.f);
        if (pk_.values()) {
            std::memcpy(w.data(), Pm.get(p + ".weight", 256), 1024);
            std::memcpy(bb.data(), Pm.get(p + ".bias", 256), 1024);
        }
        WRef rg = pk_.raw("gn:" + p + ".weight", w), rb = pk_.raw("gn:" + p + ".bias", bb);
        if (g) *g = rg;
        if (b) *b = rb;
    }
};

// ------------------------------------------------------------------------------------ engine cache
struct Engine {
    Config cfg;
    Pack pack;  // layout only (values == false)
    std::unique_ptr<Packer> packer;
    Params params;
    std::unique_ptr<SSDLite> ssd;
    std::unique_ptr<FasterRCNN> frcnn;
    std::unique_ptr<RetinaNet> retina;
    std::map<std::tuple<int, int, int, bool, int64_t>, std::unique_ptr<Plan>> plans;  // (B, H, W, u8, redzone)
    uint64_t clock = 0;
};
constexpr size_t PLAN_CACHE = 64;

static std::unique_ptr<Engine> make_engine(const Config& c, const Params* values, Pack* pack_out) {
    auto e = std::make_unique<Engine>();
    e->cfg = c;
    Pack& pk = pack_out ? *pack_out : e->pack;
    pk.values = pack_out != nullptr;
    e->packer = std::make_unique<Packer>(values ? *values : e->params, pk);
    if (c.kind == 0) {
        e->ssd = std::make_unique<SSDLite>(c, *e->packer);
        e->ssd->pack_all();
    } else if (c.kind == 1) {
        e->frcnn = std::make_unique<FasterRCNN>(c, *e->packer);
        e->frcnn->pack_all();
    } else {
        e->retina = std::make_unique<RetinaNet>(c, *e->packer);
        e->retina->pack_all();
    }
    return e;
}

static std::mutex g_mu;
static std::map<std::tuple<int, int, int>, std::unique_ptr<Engine>> g_engines;

static Engine* engine(const Config& c) {
    auto key = std::make_tuple(c.kind, c.num_classes, c.reduced_tail ? 1 : 0);
    auto it = g_engines.find(key);
    if (it != g_engines.end()) return it->second.get();
    return (g_engines[key] = make_engine(c, nullptr, nullptr)).get();
}

static Plan* plan_for(Engine* e, int B, int H, int W, bool u8) {
    auto key = std::make_tuple(B, H, W, u8, g_redzone);  // a redzone layout never serves a plain lowering
    auto it = e->plans.find(key);
    if (it != e->plans.end()) {
        it->second->last_use = ++e->clock;
        return it->second.get();
    }
    if (e->plans.size() >= PLAN_CACHE) {  // evict the least recently used plan
        auto lru = e->plans.begin();
        for (auto i = e->plans.begin(); i != e->plans.end(); ++i)
            if (i->second->last_use < lru->second->last_use) lru = i;
        e->plans.erase(lru);
    }
    std::unique_ptr<Plan> p = e->cfg.kind == 0   ? e->ssd->lower(B, H, W, u8)
                              : e->cfg.kind == 1 ? e->frcnn->lower(B, H, W, u8)
                                                 : e->retina->lower(B, H, W, u8);
    p->finalize();
    p->last_use = ++e->clock;
    Plan* raw = p.get();
    e->plans[key] = std::move(p);
    return raw;
}


static std::vector<edgedet_op> records(const Plan& P, const External& x) {
    std::vector<edgedet_op> out(P.ops.size());
    std::map<int, uint64_t> ext;
    if (x.images) ext[P.input] = x.images;
    if (x.count) ext[P.out_count] = x.count;
    if (x.boxes) ext[P.out_box] = x.boxes;
    if (x.scores) ext[P.out_score] = x.scores;
    if (x.labels) ext[P.out_label] = x.labels;
    for (size_t k = 0; k < P.ops.size(); ++k) {
        const OpRec& o = P.ops[k];
        edgedet_op& r = out[k];
        std::memset(&r, 0, sizeof(r));
        r.kind = o.kind;
        for (auto& kv : o.i) r.i[kv.first] = kv.second;
        r.i[EDGEDET_OP_LANE] = o.lane;
        for (auto& kv : o.p) {
            const Ref& f = kv.second;
            uint64_t v = 0;
            if (f.kind == Ref::W) {
                v = x.weights + 4 * (uint64_t)f.byte_off;
            } else if (f.kind == Ref::BUF) {
                auto it = ext.find(f.idx);
                v = (it != ext.end() ? it->second : x.workspace + (uint64_t)P.bufs[(size_t)f.idx].off) + (uint64_t)f.byte_off;
            }
            r.p[kv.first] = v;
        }
        for (auto& kv : o.d) r.d[kv.first] = kv.second;
        for (auto& kv : o.f) r.f[kv.first] = kv.second;
    }
    return out;
}

}  // namespace lower
}  // namespace edgedet

using namespace edgedet;
using namespace edgedet::lower;

#define EDGEDET_TRY(...)                                         \
    try {                                                        \
        __VA_ARGS__                                              \
    } catch (const std::exception& ex) {                         \
        set_error(std::string("edgedet: ") + ex.what());         \
        return -1;                                               \
    }

static int config_of(int32_t kind, int32_t num_classes, int32_t reduced_tail, Config* c) {
    EDGEDET_REQUIRE(kind == EDGEDET_MODEL_SSDLITE || kind == EDGEDET_MODEL_FRCNN || kind == EDGEDET_MODEL_RETINANET,
                    "unknown model kind");
    EDGEDET_REQUIRE(num_classes >= 2 && num_classes <= 1024, "num_classes must be 2..1024");
    c->kind = kind;
    c->num_classes = num_classes;
    c->reduced_tail = kind == EDGEDET_MODEL_SSDLITE ? reduced_tail != 0 : true;
    return 0;
}

static int shape_ok(int32_t B, int32_t H, int32_t W) {
    EDGEDET_REQUIRE(B >= 1 && B <= 4096 && H >= 1 && W >= 1 && H <= 16384 && W <= 16384, "bad (B, H, W)");
    return 0;
}

extern "C" int edgedet_set_redzone(int64_t bytes) {
    EDGEDET_REQUIRE(bytes >= 0 && bytes % 256 == 0 && bytes <= (64 << 20), "set_redzone: 0..64 MiB, multiple of 256");
    std::lock_guard<std::mutex> g(g_mu);
    g_redzone = bytes;  // part of the plan cache key: every later lookup lowers (or finds) the new layout
    return 0;
}

extern "C" int64_t edgedet_model_weights_size(int32_t kind, int32_t num_classes, int32_t reduced_tail) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c)) return -1;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        return 4 * engine(c)->pack.size;
    })
}

extern "C" int edgedet_model_pack(int32_t kind, int32_t num_classes, int32_t reduced_tail, int64_t n_params,
                                  const char* const* names, const float* const* values, const int64_t* numels,
                                  void* host_blob) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c)) return -1;
    EDGEDET_REQUIRE(names && values && numels && host_blob && n_params > 0, "model_pack: null argument");
    EDGEDET_TRY({
        Params P;
        P.values = true;
        for (int64_t k = 0; k < n_params; ++k) P.m[names[k]] = {values[k], numels[k]};
        Pack pk;
        auto e = make_engine(c, &P, &pk);
        std::memcpy(host_blob, pk.blob.data(), (size_t)pk.size * 4);
        return 0;
    })
}

extern "C" int64_t edgedet_model_workspace_size(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B,
                                                int32_t H, int32_t W, int32_t input_u8) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        return plan_for(engine(c), B, H, W, input_u8 != 0)->arena;
    })
}

extern "C" int64_t edgedet_model_records(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                                         int32_t W, int32_t input_u8, uint64_t weights, uint64_t workspace,
                                         uint64_t images, uint64_t count, uint64_t boxes, uint64_t scores,
                                         uint64_t labels, edgedet_op* out, int64_t cap) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        Plan* p = plan_for(engine(c), B, H, W, input_u8 != 0);
        const int64_t n = (int64_t)p->ops.size();
        if (out && cap >= n) {
            External x{weights, workspace, images, count, boxes, scores, labels};
            auto recs = records(*p, x);
            std::memcpy(out, recs.data(), recs.size() * sizeof(edgedet_op));
        }
        return n;
    })
}

extern "C" int edgedet_model_prepare(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                                     int32_t W, int32_t input_u8, void* workspace, void* stream) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_REQUIRE(workspace, "model_prepare: null workspace");
    // what the workspace needs is copied out under the lock: once it is released another thread may
    // evict (plan_for's LRU) or release (edgedet_model_release) the cached plan and free its host memory
    int64_t arena = 0;
    std::vector<std::pair<int64_t, std::vector<uint8_t>>> consts;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        const Plan* p = plan_for(engine(c), B, H, W, input_u8 != 0);
        arena = p->arena;
        for (auto& kv : p->consts) consts.emplace_back(p->bufs[(size_t)kv.first].off, kv.second);
    })
    // zero first: every buffer starts from zero, as the Python host's arena does
    EDGEDET_CHECK_HIP(hipMemsetAsync(workspace, 0, (size_t)arena, (hipStream_t)stream));
    for (auto& kv : consts) {
        char* dst = (char*)workspace + kv.first;
        EDGEDET_CHECK_HIP(hipMemcpyAsync(dst, kv.second.data(), kv.second.size(), hipMemcpyHostToDevice,
                                         (hipStream_t)stream));
    }
    // the copies read this call's pageable host copies: complete before returning
    EDGEDET_CHECK_HIP(hipStreamSynchronize((hipStream_t)stream));
    return 0;
}

extern "C" int edgedet_model_prepare_host(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B,
                                          int32_t H, int32_t W, int32_t input_u8, void* host_workspace,
                                          int64_t bytes) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_REQUIRE(host_workspace, "model_prepare_host: null workspace");
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        Plan* p = plan_for(engine(c), B, H, W, input_u8 != 0);
        EDGEDET_REQUIRE(bytes >= p->arena, "model_prepare_host: workspace too small");
        for (auto& kv : p->consts)
            std::memcpy((char*)host_workspace + p->bufs[(size_t)kv.first].off, kv.second.data(), kv.second.size());
        return 0;
    })
}

extern "C" int edgedet_model_forward(int32_t kind, int32_t num_classes, int32_t reduced_tail, const void* weights,
                                     const void* images, int32_t B, int32_t H, int32_t W, int32_t input_u8,
                                     void* workspace, int32_t* count, float* boxes, float* scores, int64_t* labels,
                                     void* stream) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_REQUIRE(weights && images && workspace && count && boxes && scores && labels, "model_forward: null pointer");
    std::shared_ptr<const std::vector<edgedet_op>> recs;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        Plan* p = plan_for(engine(c), B, H, W, input_u8 != 0);
        External x{(uint64_t)weights, (uint64_t)workspace, (uint64_t)images, (uint64_t)count, (uint64_t)boxes,
                   (uint64_t)scores, (uint64_t)labels};
        if (!p->resolved || !(p->resolved_for == x)) {  // resolved once per set of pointers, not per call
            p->resolved = std::make_shared<const std::vector<edgedet_op>>(records(*p, x));
            p->resolved_for = x;
        }
        recs = p->resolved;
    })
    // issued outside the lock: calls on different streams run concurrently
    return edgedet_plan_run(recs->data(), (int64_t)recs->size(), stream);
}

extern "C" int64_t edgedet_model_buffers(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                                         int32_t W, int32_t input_u8, edgedet_buffer* out, int64_t cap) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        Plan* p = plan_for(engine(c), B, H, W, input_u8 != 0);
        const int64_t n = (int64_t)p->bufs.size();
        if (out && cap >= n) {
            for (int64_t k = 0; k < n; ++k) {
                const Buf& b = p->bufs[(size_t)k];
                edgedet_buffer& r = out[k];
                std::memset(&r, 0, sizeof(r));
                std::strncpy(r.name, b.name.c_str(), sizeof(r.name) - 1);
                r.offset = b.off;
                r.nbytes = b.nbytes;
                r.dtype = b.dtype;
                r.ndim = (int32_t)std::min<size_t>(b.shape.size(), 6);
                for (int j = 0; j < r.ndim; ++j) r.shape[j] = b.shape[(size_t)j];
            }
        }
        return n;
    })
}

extern "C" int64_t edgedet_model_op_names(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B,
                                          int32_t H, int32_t W, int32_t input_u8, char* out, int64_t cap) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        Plan* p = plan_for(engine(c), B, H, W, input_u8 != 0);
        std::string all;
        for (size_t k = 0; k < p->ops.size(); ++k) all += (k ? "\n" : "") + p->ops[k].name;
        const int64_t need = (int64_t)all.size() + 1;
        if (out && cap >= need) std::memcpy(out, all.c_str(), (size_t)need);
        return need;
    })
}

extern "C" int edgedet_model_release(int32_t kind, int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                                     int32_t W, int32_t input_u8) {
    Config c;
    if (config_of(kind, num_classes, reduced_tail, &c) || shape_ok(B, H, W)) return -1;
    EDGEDET_TRY({
        std::lock_guard<std::mutex> g(g_mu);
        engine(c)->plans.erase(std::make_tuple(B, H, W, input_u8 != 0, g_redzone));
        return 0;
    })
}

extern "C" int edgedet_model_max_detections(int32_t kind) {
    return kind == EDGEDET_MODEL_SSDLITE     ? SSDLite::DETS
           : kind == EDGEDET_MODEL_FRCNN     ? FasterRCNN::BOX_DETS
           : kind == EDGEDET_MODEL_RETINANET ? RetinaNet::DETS
                                             : -1;
}

// ---- the per-model names of SURVEY.md §8(b)
extern "C" int64_t edgedet_ssdlite_workspace_size(int32_t num_classes, int32_t reduced_tail, int32_t B, int32_t H,
                                                  int32_t W, int32_t input_u8) {
    return edgedet_model_workspace_size(EDGEDET_MODEL_SSDLITE, num_classes, reduced_tail, B, H, W, input_u8);
}
extern "C" int edgedet_ssdlite_forward(const void* weights, int32_t num_classes, int32_t reduced_tail,
                                       const void* images, int32_t B, int32_t H, int32_t W, int32_t input_u8,
                                       void* workspace, int32_t* count, float* boxes, float* scores, int64_t* labels,
                                       void* stream) {
    return edgedet_model_forward(EDGEDET_MODEL_SSDLITE, num_classes, reduced_tail, weights, images, B, H, W, input_u8,
                                 workspace, count, boxes, scores, labels, stream);
}
extern "C" int64_t edgedet_frcnn_workspace_size(int32_t num_classes, int32_t B, int32_t H, int32_t W,
                                                int32_t input_u8) {
    return edgedet_model_workspace_size(EDGEDET_MODEL_FRCNN, num_classes, 1, B, H, W, input_u8);
}
extern "C" int edgedet_frcnn_forward(const void* weights, int32_t num_classes, const void* images, int32_t B, int32_t H,
                                     int32_t W, int32_t input_u8, void* workspace, int32_t* count, float* boxes,
                                     float* scores, int64_t* labels, void* stream) {
    return edgedet_model_forward(EDGEDET_MODEL_FRCNN, num_classes, 1, weights, images, B, H, W, input_u8, workspace,
                                 count, boxes, scores, labels, stream);
}
