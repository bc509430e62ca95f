// Geometry-aware family (reference src/models/geometry_aware_network.h):
//   GeometryAwareNetworkImpl(3, f, 4, max_depth, use_pcl, use_attention)   :201-347 (6 levels)
//   LightweightGeometryNetworkImpl(3, f, 4, max_depth)                      :355-440 (5 levels)
//
//   level l (H/2^l, C_l = f 2^l):
//     enc1      RayEnhancedConv(3, f, 4, rays): cat(rgb, rays) -> conv-BN-ReLU-FiLM-conv-BN-ReLU  (:17-65)
//     enc2..    GeometryEncoderBlock: MaxPool2d(2) -> RayEnhancedConv(no rays) -> CBAM              (:74-104)
//     bottleneck  the same at the deepest level
//     decN      GeometryDecoderBlock: ConvT 2x2/2 -> PCL -> cat{skip, up} -> RayEnhancedConv -> CBAM  (:112-170)
//     out_conv  1x1, sigmoid * max_depth
//   (getDownsampledRays feeds only PCL's unused ray argument, pcl_layer.h:76-111: not computed.)
//
// Arithmetic: the process-wide GEMM engine (default S3: fp32-accurate split-bf16 MFMA) through the
// plain NHWC fp32 conv / ConvT launchers; BN statistics from the conv epilogues; FiLM, CBAM and PCL
// kernels fp32 (attn_kernels.hip, film_kernels.hip).  Parity: pinned to fixtures the reference code
// writes (oracle/ref_harness.cpp --model geo|geolite; tests/test_gpu_geonet.py).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/cad/cad.h"
#include "../kernels/kernels.hpp"

namespace cad {
void set_last_error(const std::string& msg);   // cad_api.cpp (cad_last_error)
}

namespace {

struct GError : std::runtime_error {
    cad_status st;
    GError(cad_status s, const std::string& m) : std::runtime_error(m), st(s) {}
};
#define GCHK(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            throw GError(e_ == hipErrorOutOfMemory ? CAD_ERR_OOM : CAD_ERR_HIP,                 \
                         std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)
void need(bool c, const std::string& m, cad_status s = CAD_ERR_INVALID) {
    if (!c) throw GError(s, m);
}
template <class F>
cad_status gguard(F&& f) {
    try {
        f();
        return CAD_OK;
    } catch (const GError& e) {
        cad::set_last_error(e.what());
        return e.st;
    } catch (const std::exception& e) {
        cad::set_last_error(e.what());
        return CAD_ERR_INVALID;
    }
}
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

struct Arena {
    char* base = nullptr;
    size_t off = 0;
    void* take(size_t bytes) {
        off = (off + 255) & ~size_t(255);
        void* p = base ? base + off : nullptr;
        off += bytes;
        return p;
    }
    float* f(int64_t n) { return static_cast<float*>(take(sizeof(float) * (size_t)std::max<int64_t>(n, 1))); }
    double* d(int64_t n) { return static_cast<double*>(take(sizeof(double) * (size_t)std::max<int64_t>(n, 1))); }
    int* i(int64_t n) { return static_cast<int*>(take(sizeof(int) * (size_t)std::max<int64_t>(n, 1))); }
    uint8_t* u8(int64_t n) { return static_cast<uint8_t*>(take((size_t)std::max<int64_t>(n, 1))); }
};

// parameter kinds: internal layouts and the reference module's default initialisation
enum GKind {
    G_CONV3,                                   // [co][tap][ci_pad] internal; kaiming_uniform(a=sqrt5)
    G_BNW, G_BNB,                              // 1 / 0
    G_CONVT_W, G_CONVT_B,                      // [ci][q][co] internal
    G_FC_W, G_FC_B,                            // torch::nn::Linear defaults
    G_FILM_HEAD_W, G_FILM_GAMMA_B, G_FILM_BETA_B,   // film_layer.h:68-71
    G_PCL_T_W, G_PCL_T_B,                      // fc_transform: zeros / identity (pcl_layer.h:61-63)
    G_SCONV,                                   // CBAM spatial conv (1, 2, 7, 7)
    G_HEAD_W, G_HEAD_B
};
struct GParam {
    std::string name;
    int ndim;
    int64_t shape[4];
    GKind kind;
    int64_t off = 0, n_int = 0, n_ref = 0;
    int cin_ref = 0, cin_int = 0, cout = 0;
    int fan_in = 1;   // of the weight this parameter belongs to (default init bound 1/sqrt(fan_in))
};
struct GBuf {
    std::string name;
    int64_t C;
    float* ptr;
};
struct GBN {
    int C = 0, widx = -1, bidx = -1;
    float *rm = nullptr, *rv = nullptr, *mean = nullptr, *invstd = nullptr, *scale = nullptr, *shift = nullptr,
          *coef = nullptr;
};
struct GConv {
    int pidx = -1, cin = 0, cout = 0;
    float* wd = nullptr;   // dgrad repack [ci][tap][co]
};
struct GFilm {
    int p0 = -1;
    float *rm1, *rv1, *rm2, *rv2, *xh1, *h1, *xh2, *h2, *is1, *is2, *gam, *bet, *dgam, *dbet, *dh2, *dh1;
};
// RayEnhancedConv (+ CBAM when cb0 >= 0)
struct GBlock {
    int level = 0;
    GConv c1, c2;
    GBN b1, b2;
    GFilm film;
    int cb0 = -1;              // index of attention.channel_attention.fc1.weight (fc1.b, fc2.w, fc2.b, sconv follow)
    int Cr = 0;
    cad::Cbam A{};             // state pointers (parameters filled per use: the slabs may move)
    float *y1 = nullptr, *a1 = nullptr, *y2 = nullptr, *z = nullptr;   // z: relu(bn2(y2)), the CBAM input
    int first_param = 0, last_param = 0;
};
struct GDec {
    int up_w = -1, up_b = -1, cin = 0, cout = 0;
    float* wf = nullptr;       // ConvT forward repack
    int pcl0 = -1;             // index of pcl.loc_fc1.weight (5 parameters follow)
    cad::Pcl P{};
    float* u = nullptr;        // ConvT output [M][C] (PCL input)
    float* x = nullptr;        // block output [M][C]
    GBlock blk;
};

}  // namespace

struct cad_geonet {
    int device = 0, variant = CAD_GEONET_FULL, nl = 6, f = 64, Bmax = 1, H = 0, W = 0;
    bool use_pcl = true, use_attention = true;
    float max_depth = 10.f;
    bool train = true, have_fwd = false;
    int fwd_B = 0;
    int64_t nbt = 0, nbt_film = 0;
    std::vector<GParam> params;
    std::vector<GBuf> bufs;
    int64_t n_flat = 0;
    float *flat_p = nullptr, *flat_g = nullptr, *adam_m = nullptr, *adam_v = nullptr;
    int64_t adam_t = 0;
    float* norm_coef = nullptr;
    void* base = nullptr;
    GBlock enc[6];
    GDec dec[5];               // index = output level
    int head_w = -1, head_b = -1;
    float *x0 = nullptr, *camn = nullptr, *sig = nullptr, *bott = nullptr;
    float* cat[5] = {};
    float* pool[6] = {};
    uint8_t* pidx[6] = {};
    float* dcat[5] = {};
    float *Sa = nullptr, *Sb = nullptr, *Sc = nullptr, *Sd = nullptr, *Su = nullptr, *Sx = nullptr;
    float* stats = nullptr;
    double* dscr = nullptr;
    float* slab = nullptr;
    int64_t slab_cap = 0;
    int Hl(int l) const { return H >> l; }
    int Wl(int l) const { return W >> l; }
    int Cl(int l) const { return f << l; }
    int64_t Ml(int l, int B) const { return (int64_t)B * Hl(l) * Wl(l); }
    float* P(int i) const { return flat_p + params[i].off; }
    float* G(int i) const { return flat_g + params[i].off; }
    std::vector<std::pair<int64_t, int64_t>> stage_range;   // staged backward: each stage's slab range
};

namespace {

int add_param(cad_geonet* h, const std::string& name, std::vector<int64_t> shape, GKind kind, int fan_in,
              int cin_ref = 0, int cin_int = 0, int cout = 0) {
    GParam p;
    p.name = name;
    p.ndim = (int)shape.size();
    p.n_ref = 1;
    for (int i = 0; i < 4; ++i) p.shape[i] = i < p.ndim ? shape[i] : 1;
    for (int i = 0; i < p.ndim; ++i) p.n_ref *= shape[i];
    p.kind = kind;
    p.fan_in = fan_in;
    p.cin_ref = cin_ref; p.cin_int = cin_int; p.cout = cout;
    p.n_int = kind == G_CONV3 ? (int64_t)cout * 9 * cin_int : p.n_ref;
    h->n_flat = (h->n_flat + 63) & ~int64_t(63);
    p.off = h->n_flat;
    h->n_flat += p.n_int;
    h->params.push_back(p);
    return (int)h->params.size() - 1;
}

// RayEnhancedConvImpl ctor (geometry_aware_network.h:25-45): conv1, bn1, conv2, bn2, film
void add_block(cad_geonet* h, GBlock& b, const std::string& pre, int cin_ref, int cin_int, int cout, int level) {
    b.level = level;
    b.first_param = (int)h->params.size();
    b.c1 = GConv{add_param(h, pre + "conv1.weight", {cout, cin_ref, 3, 3}, G_CONV3, cin_ref * 9, cin_ref, cin_int, cout),
                 cin_int, cout, nullptr};
    b.b1.C = cout;
    b.b1.widx = add_param(h, pre + "bn1.weight", {cout}, G_BNW, 1);
    b.b1.bidx = add_param(h, pre + "bn1.bias", {cout}, G_BNB, 1);
    b.c2 = GConv{add_param(h, pre + "conv2.weight", {cout, cout, 3, 3}, G_CONV3, cout * 9, cout, cout, cout), cout,
                 cout, nullptr};
    b.b2.C = cout;
    b.b2.widx = add_param(h, pre + "bn2.weight", {cout}, G_BNW, 1);
    b.b2.bidx = add_param(h, pre + "bn2.bias", {cout}, G_BNB, 1);
    // FiLMLayerImpl(4, C) (film_layer.h:55-66): fc1, fc2, fc_gamma, fc_beta, bn1, bn2
    const std::string fp = pre + "film.";
    const int H1 = cad::kFilmH1, H2 = cad::kFilmH2;
    b.film.p0 = add_param(h, fp + "fc1.weight", {H1, 4}, G_FC_W, 4);
    add_param(h, fp + "fc1.bias", {H1}, G_FC_B, 4);
    add_param(h, fp + "fc2.weight", {H2, H1}, G_FC_W, H1);
    add_param(h, fp + "fc2.bias", {H2}, G_FC_B, H1);
    add_param(h, fp + "fc_gamma.weight", {cout, H2}, G_FILM_HEAD_W, H2);
    add_param(h, fp + "fc_gamma.bias", {cout}, G_FILM_GAMMA_B, H2);
    add_param(h, fp + "fc_beta.weight", {cout, H2}, G_FILM_HEAD_W, H2);
    add_param(h, fp + "fc_beta.bias", {cout}, G_FILM_BETA_B, H2);
    add_param(h, fp + "bn1.weight", {H1}, G_BNW, 1);
    add_param(h, fp + "bn1.bias", {H1}, G_BNB, 1);
    add_param(h, fp + "bn2.weight", {H2}, G_BNW, 1);
    add_param(h, fp + "bn2.bias", {H2}, G_BNB, 1);
    b.last_param = (int)h->params.size() - 1;
}

// CBAMImpl(C) (spatial_attention.h:150-157): channel_attention.{fc1, fc2}, spatial_attention.conv
void add_cbam(cad_geonet* h, GBlock& b, const std::string& pre) {
    const int C = b.c2.cout, Cr = std::max(1, C / 16);
    b.Cr = Cr;
    b.cb0 = add_param(h, pre + "channel_attention.fc1.weight", {Cr, C}, G_FC_W, C);
    add_param(h, pre + "channel_attention.fc1.bias", {Cr}, G_FC_B, C);
    add_param(h, pre + "channel_attention.fc2.weight", {C, Cr}, G_FC_W, Cr);
    add_param(h, pre + "channel_attention.fc2.bias", {C}, G_FC_B, Cr);
    add_param(h, pre + "spatial_attention.conv.weight", {1, 2, 7, 7}, G_SCONV, 98);
    b.last_param = (int)h->params.size() - 1;
}

void build(cad_geonet* h) {
    const int f = h->f, nl = h->nl;
    // GeometryAwareNetworkImpl / LightweightGeometryNetworkImpl ctor registration order
    add_block(h, h->enc[0], "enc1.", 3 + 3, 8, f, 0);   // RayEnhancedConv(3, f, 4, true): NHWC8 input
    for (int l = 1; l < nl; ++l) {
        const std::string pre = l == nl - 1 ? std::string("bottleneck.") : "enc" + std::to_string(l + 1) + ".";
        add_block(h, h->enc[l], pre + "conv.", h->Cl(l - 1), h->Cl(l - 1), h->Cl(l), l);
        if (h->use_attention) add_cbam(h, h->enc[l], pre + "attention.");
    }
    for (int l = nl - 2; l >= 0; --l) {
        GDec& d = h->dec[l];
        const std::string pre = "dec" + std::to_string(l + 1) + ".";
        d.cin = h->Cl(l + 1);
        d.cout = h->Cl(l);
        d.up_w = add_param(h, pre + "up.weight", {d.cin, d.cout, 2, 2}, G_CONVT_W, d.cout * 4);
        d.up_b = add_param(h, pre + "up.bias", {d.cout}, G_CONVT_B, d.cout * 4);
        add_block(h, d.blk, pre + "conv.", d.cin, d.cin, d.cout, l);
        d.blk.first_param = d.up_w;
        if (h->use_pcl) {   // PerspectiveCorrectionLayerImpl(C, 4, 128) (pcl_layer.h:45-63)
            const int K1 = d.cout + 4, Hd = cad::kPclHidden;
            d.pcl0 = add_param(h, pre + "pcl.loc_fc1.weight", {Hd, K1}, G_FC_W, K1);
            add_param(h, pre + "pcl.loc_fc1.bias", {Hd}, G_FC_B, K1);
            add_param(h, pre + "pcl.loc_fc2.weight", {Hd, Hd}, G_FC_W, Hd);
            add_param(h, pre + "pcl.loc_fc2.bias", {Hd}, G_FC_B, Hd);
            add_param(h, pre + "pcl.fc_transform.weight", {6, Hd}, G_PCL_T_W, Hd);
            add_param(h, pre + "pcl.fc_transform.bias", {6}, G_PCL_T_B, Hd);
            d.blk.last_param = (int)h->params.size() - 1;
        }
        if (h->use_attention) add_cbam(h, d.blk, pre + "attention.");
    }
    h->head_w = add_param(h, "out_conv.weight", {1, f, 1, 1}, G_HEAD_W, f);
    h->head_b = add_param(h, "out_conv.bias", {1}, G_HEAD_B, f);
    h->n_flat = (h->n_flat + 63) & ~int64_t(63);
}

void bn_alloc(Arena& a, GBN& b) {
    b.rm = a.f(b.C); b.rv = a.f(b.C);
    b.mean = a.f(b.C); b.invstd = a.f(b.C); b.scale = a.f(b.C); b.shift = a.f(b.C); b.coef = a.f(3 * b.C);
}

void block_alloc(cad_geonet* h, Arena& a, GBlock& b, int B) {
    const int l = b.level, C = b.c2.cout;
    const int64_t M = h->Ml(l, B), MC = M * C;
    bn_alloc(a, b.b1);
    bn_alloc(a, b.b2);
    b.y1 = a.f(MC); b.a1 = a.f(MC); b.y2 = a.f(MC);
    if (b.level > 0 || &b != &h->enc[0]) b.c1.wd = a.f((int64_t)b.c1.cout * 9 * b.c1.cin);
    b.c2.wd = a.f((int64_t)C * 9 * C);
    GFilm& F = b.film;
    const int H1 = cad::kFilmH1, H2 = cad::kFilmH2;
    F.rm1 = a.f(H1); F.rv1 = a.f(H1); F.rm2 = a.f(H2); F.rv2 = a.f(H2);
    F.xh1 = a.f((int64_t)B * H1); F.h1 = a.f((int64_t)B * H1); F.dh1 = a.f((int64_t)B * H1);
    F.xh2 = a.f((int64_t)B * H2); F.h2 = a.f((int64_t)B * H2); F.dh2 = a.f((int64_t)B * H2);
    F.is1 = a.f(H1); F.is2 = a.f(H2);
    F.gam = a.f((int64_t)B * C); F.bet = a.f((int64_t)B * C);
    F.dgam = a.f((int64_t)B * C); F.dbet = a.f((int64_t)B * C);
    if (b.cb0 >= 0) {
        b.z = a.f(MC);
        cad::Cbam& A = b.A;
        const int Cr = b.Cr;
        A.C = C; A.Cr = Cr;
        A.avg = a.f((int64_t)B * C); A.mx = a.f((int64_t)B * C); A.amax = a.i((int64_t)B * C);
        A.ha = a.f((int64_t)B * Cr); A.hm = a.f((int64_t)B * Cr); A.att = a.f((int64_t)B * C);
        A.s = a.f(2 * M); A.sidx = a.i(M); A.sa = a.f(M);
        A.dlog = a.f(M); A.ds = a.f(2 * M);
        A.dO = a.f((int64_t)B * C); A.dha = a.f((int64_t)B * Cr); A.dhm = a.f((int64_t)B * Cr);
        A.dva = a.f((int64_t)B * C); A.dvm = a.f((int64_t)B * C);
    }
}

void layout(cad_geonet* h, Arena& a) {
    const int B = h->Bmax, nl = h->nl;
    h->flat_p = a.f(h->n_flat);
    h->flat_g = a.f(h->n_flat);
    h->adam_m = a.f(h->n_flat);
    h->adam_v = a.f(h->n_flat);
    h->norm_coef = a.f(4);
    h->camn = a.f((int64_t)B * 4);
    h->x0 = a.f(h->Ml(0, B) * 8);
    h->sig = a.f(h->Ml(0, B));
    for (int l = 0; l < nl; ++l) {
        block_alloc(h, a, h->enc[l], B);
        if (l > 0) {
            h->pool[l] = a.f(h->Ml(l, B) * h->Cl(l - 1));
            h->pidx[l] = a.u8(h->Ml(l, B) * h->Cl(l - 1));
        }
        if (l < nl - 1) {
            h->cat[l] = a.f(2 * h->Ml(l, B) * h->Cl(l));
            h->dcat[l] = a.f(2 * h->Ml(l, B) * h->Cl(l));
        }
    }
    h->bott = a.f(h->Ml(nl - 1, B) * h->Cl(nl - 1));
    for (int l = nl - 2; l >= 0; --l) {
        GDec& d = h->dec[l];
        const int64_t MC = h->Ml(l, B) * d.cout;
        block_alloc(h, a, d.blk, B);
        d.wf = a.f((int64_t)4 * d.cout * d.cin);
        d.u = a.f(MC);
        d.x = a.f(MC);
        if (d.pcl0 >= 0) {
            cad::Pcl& P = d.P;
            const int Hd = cad::kPclHidden;
            P.C = d.cout;
            P.pooled = a.f((int64_t)B * d.cout);
            P.h1 = a.f((int64_t)B * Hd); P.h2 = a.f((int64_t)B * Hd);
            P.tp = a.f((int64_t)B * 6); P.theta = a.f((int64_t)B * 6);
            P.dgrid = a.f(2 * h->Ml(l, B));
            P.dtp = a.f((int64_t)B * 6); P.dh1 = a.f((int64_t)B * Hd); P.dh2 = a.f((int64_t)B * Hd);
            P.dpooled = a.f((int64_t)B * d.cout);
        }
    }
    const int64_t M0C0 = h->Ml(0, B) * h->Cl(0);
    h->Sa = a.f(M0C0); h->Sb = a.f(M0C0); h->Sd = a.f(M0C0); h->Su = a.f(M0C0); h->Sx = a.f(M0C0);
    h->Sc = a.f(h->Ml(1, B) * h->Cl(0));
    int64_t st = 0, dscr = 8192;
    int64_t sl = 0;
    for (int l = 0; l < nl; ++l) {
        const int64_t M = h->Ml(l, B), HW = (int64_t)h->Hl(l) * h->Wl(l);
        const int C = h->Cl(l);
        st = std::max<int64_t>(st, (M + 63) / 64 * (2 * C + 1));   // BN tile partials + counts
        dscr = std::max(dscr, (int64_t)(cad::colsum_slices(M) + 2) * 4 * C + 4 * C + 8192);
        dscr = std::max(dscr, cad::film_reduce_doubles(B, HW, C) + 8192);
        dscr = std::max(dscr, cad::attn_scratch_doubles(B, HW, C) + 8192);
        sl = std::max(sl, cad::wgrad_slab_floats(C, 9 * C * 2, (int)std::min<int64_t>(M, INT32_MAX)));
    }
    h->stats = a.f(st);
    h->dscr = a.d(dscr);
    h->slab_cap = std::min<int64_t>(sl, (int64_t)64 << 20);
    h->slab = a.f(h->slab_cap);
    // named_buffers() order (float buffers): per RayEnhancedConv bn1, bn2, film.bn1, film.bn2
    h->bufs.clear();
    auto add_bufs = [&](const std::string& pre, GBlock& b) {
        h->bufs.push_back({pre + "bn1.running_mean", b.b1.C, b.b1.rm});
        h->bufs.push_back({pre + "bn1.running_var", b.b1.C, b.b1.rv});
        h->bufs.push_back({pre + "bn2.running_mean", b.b2.C, b.b2.rm});
        h->bufs.push_back({pre + "bn2.running_var", b.b2.C, b.b2.rv});
        h->bufs.push_back({pre + "film.bn1.running_mean", cad::kFilmH1, b.film.rm1});
        h->bufs.push_back({pre + "film.bn1.running_var", cad::kFilmH1, b.film.rv1});
        h->bufs.push_back({pre + "film.bn2.running_mean", cad::kFilmH2, b.film.rm2});
        h->bufs.push_back({pre + "film.bn2.running_var", cad::kFilmH2, b.film.rv2});
    };
    add_bufs("enc1.", h->enc[0]);
    for (int l = 1; l < nl; ++l)
        add_bufs(l == nl - 1 ? std::string("bottleneck.conv.") : "enc" + std::to_string(l + 1) + ".conv.", h->enc[l]);
    for (int l = nl - 2; l >= 0; --l) add_bufs("dec" + std::to_string(l + 1) + ".conv.", h->dec[l].blk);
}

// ------------------------------------------------------------------------------------------
// parameter views (rebuilt per use: pointers into the current slabs)
// ------------------------------------------------------------------------------------------
cad::FilmLayer film_view(const cad_geonet* h, const GBlock& b) {
    const GFilm& F = b.film;
    const int i = F.p0;
    cad::FilmLayer L;
    L.C = b.c2.cout;
    L.w1 = h->P(i); L.b1 = h->P(i + 1); L.w2 = h->P(i + 2); L.b2 = h->P(i + 3);
    L.wg = h->P(i + 4); L.bg = h->P(i + 5); L.wb = h->P(i + 6); L.bb = h->P(i + 7);
    L.g1 = h->P(i + 8); L.be1 = h->P(i + 9); L.g2 = h->P(i + 10); L.be2 = h->P(i + 11);
    L.rm1 = F.rm1; L.rv1 = F.rv1; L.rm2 = F.rm2; L.rv2 = F.rv2;
    L.xh1 = F.xh1; L.h1 = F.h1; L.xh2 = F.xh2; L.h2 = F.h2; L.is1 = F.is1; L.is2 = F.is2;
    L.gam = F.gam; L.bet = F.bet; L.dgam = F.dgam; L.dbet = F.dbet; L.dh2 = F.dh2; L.dh1 = F.dh1;
    L.gw1 = h->G(i); L.gb1 = h->G(i + 1); L.gw2 = h->G(i + 2); L.gb2 = h->G(i + 3);
    L.gwg = h->G(i + 4); L.gbg = h->G(i + 5); L.gwb = h->G(i + 6); L.gbb = h->G(i + 7);
    L.gg1 = h->G(i + 8); L.gbe1 = h->G(i + 9); L.gg2 = h->G(i + 10); L.gbe2 = h->G(i + 11);
    return L;
}
cad::Cbam cbam_view(const cad_geonet* h, const GBlock& b) {
    cad::Cbam A = b.A;
    const int i = b.cb0;
    A.w1 = h->P(i); A.b1 = h->P(i + 1); A.w2 = h->P(i + 2); A.b2 = h->P(i + 3); A.wsp = h->P(i + 4);
    A.gw1 = h->G(i); A.gb1 = h->G(i + 1); A.gw2 = h->G(i + 2); A.gb2 = h->G(i + 3); A.gwsp = h->G(i + 4);
    return A;
}
cad::Pcl pcl_view(const cad_geonet* h, const GDec& d) {
    cad::Pcl P = d.P;
    const int i = d.pcl0;
    P.w1 = h->P(i); P.b1 = h->P(i + 1); P.w2 = h->P(i + 2); P.b2 = h->P(i + 3); P.w3 = h->P(i + 4); P.b3 = h->P(i + 5);
    P.gw1 = h->G(i); P.gb1 = h->G(i + 1); P.gw2 = h->G(i + 2); P.gb2 = h->G(i + 3); P.gw3 = h->G(i + 4);
    P.gb3 = h->G(i + 5);
    return P;
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// RayEnhancedConvImpl::forward (geometry_aware_network.h:47-64) [+ CBAMImpl::forward]: output rows ldo at ocoff
void block_fwd(cad_geonet* h, GBlock& b, const float* in, int64_t ldin, int B, float* out, int64_t ldo, int ocoff,
               hipStream_t st) {
    const int l = b.level, Hh = h->Hl(l), Ww = h->Wl(l), C = b.c2.cout;
    const int64_t M = h->Ml(l, B), HW = (int64_t)Hh * Ww;
    const bool tr = h->train;
    auto bn = [&](GBN& n, int cin) {
        const int rows = cad::conv3x3_stats_rows(cin, B, Hh, Ww, C, false);
        if (tr)
            cad::bn_fwd_finalize(h->stats, rows, C, M, h->P(n.widx), h->P(n.bidx), n.rm, n.rv, 0.1f, 1e-5f, h->dscr,
                                 n.mean, n.invstd, n.scale, n.shift, st);
        else
            cad::bn_eval_coeffs(h->P(n.widx), h->P(n.bidx), n.rm, n.rv, C, 1e-5f, n.mean, n.invstd, n.scale, n.shift, st);
    };
    float* stats = tr ? h->stats : nullptr;
    cad::conv3x3_fwd(in, ldin, 0, b.c1.cin, h->P(b.c1.pidx), C, b.y1, C, 0, B, Hh, Ww, stats, st);
    bn(b.b1, b.c1.cin);
    cad::film_apply(b.y1, C, b.b1.scale, b.b1.shift, b.film.gam, b.film.bet, B, HW, b.a1, st);
    cad::conv3x3_fwd(b.a1, C, 0, C, h->P(b.c2.pidx), C, b.y2, C, 0, B, Hh, Ww, stats, st);
    bn(b.b2, C);
    if (b.cb0 >= 0) {
        cad::bn_relu_fwd(b.y2, C, b.b2.scale, b.b2.shift, b.z, C, 0, M, st);
        cad::cbam_fwd(cbam_view(h, b), b.z, B, Hh, Ww, out, ldo, ocoff, h->dscr, st);
    } else {
        cad::bn_relu_fwd(b.y2, C, b.b2.scale, b.b2.shift, out, ldo, ocoff, M, st);
    }
}

void forward(cad_geonet* h, const float* rgb, const float* rays, const float* cam4, float* depth, int B,
             hipStream_t st) {
    const int nl = h->nl;
    cad::camera_normalize(cam4, B, h->H, h->W, h->camn, st);   // normalizeCameraIntrinsics (:327-345)
    for (int l = 0; l < nl; ++l) cad::film_mlp_fwd(film_view(h, h->enc[l]), h->camn, B, h->train, st);
    for (int l = nl - 2; l >= 0; --l) {
        cad::film_mlp_fwd(film_view(h, h->dec[l].blk), h->camn, B, h->train, st);
        cad::repack_convT_fwd(h->P(h->dec[l].up_w), h->dec[l].wf, h->dec[l].cin, h->dec[l].cout, st);
    }
    cad::pack_rgb_rays(rgb, rays, B, h->H, h->W, h->x0, st);
    block_fwd(h, h->enc[0], h->x0, 8, B, h->cat[0], 2 * h->Cl(0), 0, st);
    for (int l = 1; l < nl; ++l) {
        const int Cp = h->Cl(l - 1);
        cad::maxpool_fwd(h->cat[l - 1], 2 * Cp, Cp, B, h->Hl(l - 1), h->Wl(l - 1), h->pool[l], h->pidx[l], st);
        if (l < nl - 1)
            block_fwd(h, h->enc[l], h->pool[l], Cp, B, h->cat[l], 2 * h->Cl(l), 0, st);
        else
            block_fwd(h, h->enc[l], h->pool[l], Cp, B, h->bott, h->Cl(l), 0, st);
    }
    for (int l = nl - 2; l >= 0; --l) {
        GDec& d = h->dec[l];
        const int C = d.cout;
        const float* in = l == nl - 2 ? h->bott : h->dec[l + 1].x;
        if (d.pcl0 >= 0) {
            cad::convT_fwd(in, d.cin, d.cin, d.wf, h->P(d.up_b), C, d.u, C, 0, B, h->Hl(l + 1), h->Wl(l + 1), st);
            cad::pcl_fwd(pcl_view(h, d), d.u, h->camn, B, h->Hl(l), h->Wl(l), h->cat[l], 2 * C, C, h->dscr, st);
        } else {
            cad::convT_fwd(in, d.cin, d.cin, d.wf, h->P(d.up_b), C, h->cat[l], 2 * C, C, B, h->Hl(l + 1), h->Wl(l + 1),
                           st);
        }
        block_fwd(h, d.blk, h->cat[l], 2 * C, B, d.x, C, 0, st);
    }
    cad::head_fwd(h->dec[0].x, h->f, h->P(h->head_w), h->P(h->head_b), h->max_depth, h->sig, depth, h->Ml(0, B), st);
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// g: grad of the block output (ld ldg, offset gcoff); in: the block input; din: conv1's dgrad (nullable)
void block_bwd(cad_geonet* h, GBlock& b, const float* g, int64_t ldg, int gcoff, const float* in, int64_t ldin, int B,
               float* din, int64_t lddin, hipStream_t st) {
    const int l = b.level, Hh = h->Hl(l), Ww = h->Wl(l), C = b.c2.cout;
    const int64_t M = h->Ml(l, B), HW = (int64_t)Hh * Ww;
    if (b.cb0 >= 0) {
        cad::cbam_bwd(cbam_view(h, b), b.z, g, ldg, gcoff, B, Hh, Ww, h->Sd, h->dscr, st);
        g = h->Sd; ldg = C; gcoff = 0;
    }
    float* dY = h->Sb;
    float* dA1 = h->Sa;
    cad::bn_relu_bwd(g, ldg, gcoff, b.y2, C, b.b2.mean, b.b2.invstd, b.b2.scale, b.b2.shift, h->P(b.b2.widx), M, h->dscr,
                     b.b2.coef, h->G(b.b2.widx), h->G(b.b2.bidx), dY, st);
    cad::conv3x3_wgrad(dY, C, b.a1, C, 0, C, h->G(b.c2.pidx), B, Hh, Ww, h->slab, h->slab_cap, st);
    cad::conv3x3_dgrad(dY, C, b.c2.wd, C, dA1, C, B, Hh, Ww, st);
    cad::film_affine_bwd(dA1, b.y1, C, b.b1.scale, b.b1.shift, B, HW, h->dscr, b.film.dgam, b.film.dbet, st);
    cad::bn_relu_bwd(dA1, C, 0, b.y1, C, b.b1.mean, b.b1.invstd, b.b1.scale, b.b1.shift, h->P(b.b1.widx), M, h->dscr,
                     b.b1.coef, h->G(b.b1.widx), h->G(b.b1.bidx), dY, st, b.film.gam, HW);
    cad::film_mlp_bwd(film_view(h, b), h->camn, B, st);
    cad::conv3x3_wgrad(dY, C, in, ldin, 0, b.c1.cin, h->G(b.c1.pidx), B, Hh, Ww, h->slab, h->slab_cap, st);
    if (din) cad::conv3x3_dgrad(dY, C, b.c1.wd, b.c1.cin, din, lddin, B, Hh, Ww, st);
}

// Backward in stages whose parameter gradients are contiguous, decreasing-offset slab ranges
// (registration order enc1, enc2.., bottleneck, dec<nl-1>..dec1, out_conv): 0 head, 1..nl-1 the
// decoders dec1..dec<nl-1>, then the encoders bottleneck..enc2, last enc1 — the data-parallel
// exchange (dp.cpp) all-reduces a finished range while the later stages run.
int num_stages(const cad_geonet* h) { return 1 + (h->nl - 1) + (h->nl - 1) + 1; }

void backward_stage(cad_geonet* h, int stage, const float* dpred, hipStream_t st) {
    const int B = h->fwd_B, nl = h->nl;
    if (stage == 0) {
        auto rp = [&](GConv& c) { cad::repack_conv_dgrad(h->P(c.pidx), c.wd, c.cout, c.cin, st); };
        for (int l = 0; l < nl; ++l) {
            if (l > 0) rp(h->enc[l].c1);
            rp(h->enc[l].c2);
        }
        for (int l = 0; l <= nl - 2; ++l) { rp(h->dec[l].blk.c1); rp(h->dec[l].blk.c2); }
        cad::head_bwd(h->dec[0].x, h->f, h->P(h->head_w), dpred, h->sig, h->max_depth, h->Sx, h->Ml(0, B), h->dscr,
                      h->G(h->head_w), h->G(h->head_b), st);
        return;
    }
    if (stage <= nl - 1) {   // decoder level l = stage - 1; Sx = grad of dec[l].x
        const int l = stage - 1;
        GDec& d = h->dec[l];
        const int C = d.cout;
        const int64_t M = h->Ml(l, B);
        block_bwd(h, d.blk, h->Sx, C, 0, h->cat[l], 2 * C, B, h->dcat[l], 2 * C, st);
        const float* gu = h->dcat[l];
        int64_t ldgu = 2 * C;
        int gcu = C;
        if (d.pcl0 >= 0) {
            cad::pcl_bwd(pcl_view(h, d), d.u, h->camn, h->dcat[l], 2 * C, C, B, h->Hl(l), h->Wl(l), h->Su, h->dscr, st);
            gu = h->Su; ldgu = C; gcu = 0;
        }
        const float* in = l == nl - 2 ? h->bott : h->dec[l + 1].x;
        cad::convT_wgrad(in, d.cin, gu, ldgu, gcu, C, h->G(d.up_w), B, h->Hl(l + 1), h->Wl(l + 1), h->slab, h->slab_cap,
                         st);
        cad::colsum(gu, ldgu, gcu, M, C, h->dscr, st);
        cad::colsum_finalize(h->dscr, cad::colsum_slices(M), C, h->G(d.up_b), 1.f, st);
        cad::convT_dgrad(gu, ldgu, gcu, C, h->P(d.up_w), d.cin, h->Sx, B, h->Hl(l + 1), h->Wl(l + 1), st);
        return;
    }
    const int l = nl - 1 - (stage - nl);   // encoders: bottleneck (nl - 1) .. enc2 (1), then enc1 (0)
    if (l >= 1) {
        GBlock& e = h->enc[l];
        const int C = h->Cl(l), Cp = h->Cl(l - 1);
        const float* g = l == nl - 1 ? h->Sx : h->dcat[l];
        block_bwd(h, e, g, l == nl - 1 ? C : 2 * C, 0, h->pool[l], Cp, B, h->Sc, Cp, st);
        cad::maxpool_bwd(h->Sc, h->pidx[l], Cp, B, h->Hl(l - 1), h->Wl(l - 1), h->dcat[l - 1], 2 * Cp, st);
        return;
    }
    block_bwd(h, h->enc[0], h->dcat[0], 2 * h->Cl(0), 0, h->x0, 8, B, nullptr, 0, st);
}

void backward(cad_geonet* h, const float* dpred, hipStream_t st) {
    for (int s = 0; s < num_stages(h); ++s) backward_stage(h, s, dpred, st);
}

void compute_stage_ranges(cad_geonet* h) {
    const int nl = h->nl;
    std::vector<std::string> pre = {"out_conv."};
    for (int l = 0; l <= nl - 2; ++l) pre.push_back("dec" + std::to_string(l + 1) + ".");
    for (int l = nl - 1; l >= 0; --l)
        pre.push_back(l == 0 ? std::string("enc1.") : l == nl - 1 ? std::string("bottleneck.")
                                                                    : "enc" + std::to_string(l + 1) + ".");
    h->stage_range.clear();
    std::vector<int> owner(h->params.size(), -1);
    for (size_t s = 0; s < pre.size(); ++s) {
        int64_t lo = INT64_MAX, hi = -1;
        for (size_t i = 0; i < h->params.size(); ++i)
            if (h->params[i].name.compare(0, pre[s].size(), pre[s]) == 0) {
                if (owner[i] >= 0) throw std::logic_error("parameter in two backward stages: " + h->params[i].name);
                owner[i] = (int)s;
                lo = std::min(lo, h->params[i].off);
                hi = std::max(hi, h->params[i].off + h->params[i].n_int);
            }
        if (hi < 0) throw std::logic_error("empty backward stage " + pre[s]);
        h->stage_range.push_back({lo, hi - lo});
    }
    for (size_t i = 0; i < h->params.size(); ++i) {
        if (owner[i] < 0) throw std::logic_error("parameter in no backward stage: " + h->params[i].name);
        for (size_t s = 0; s < pre.size(); ++s)
            if ((int)s != owner[i] && h->params[i].off < h->stage_range[s].first + h->stage_range[s].second &&
                h->params[i].off + h->params[i].n_int > h->stage_range[s].first)
                throw std::logic_error("backward stage ranges overlap at " + h->params[i].name);
    }
}

// ------------------------------------------------------------------------------------------
// reference layout <-> internal, default init
// ------------------------------------------------------------------------------------------
void ref_to_int(const GParam& p, const float* src, std::vector<float>& dst) {
    dst.assign(p.n_int, 0.f);
    if (p.kind == G_CONV3) {   // (co, ci, ky, kx) -> [co][tap][ci_pad]
        for (int co = 0; co < p.cout; ++co)
            for (int ci = 0; ci < p.cin_ref; ++ci)
                for (int t = 0; t < 9; ++t)
                    dst[((int64_t)co * 9 + t) * p.cin_int + ci] = src[((int64_t)co * p.cin_ref + ci) * 9 + t];
    } else if (p.kind == G_CONVT_W) {   // (ci, co, dy, dx) -> [ci][q][co]
        const int64_t ci_n = p.shape[0], co_n = p.shape[1];
        for (int64_t ci = 0; ci < ci_n; ++ci)
            for (int64_t co = 0; co < co_n; ++co)
                for (int q = 0; q < 4; ++q) dst[(ci * 4 + q) * co_n + co] = src[(ci * co_n + co) * 4 + q];
    } else {
        std::memcpy(dst.data(), src, sizeof(float) * p.n_ref);
    }
}
void int_to_ref(const GParam& p, const float* src, float* dst) {
    if (p.kind == G_CONV3) {
        for (int co = 0; co < p.cout; ++co)
            for (int ci = 0; ci < p.cin_ref; ++ci)
                for (int t = 0; t < 9; ++t)
                    dst[((int64_t)co * p.cin_ref + ci) * 9 + t] = src[((int64_t)co * 9 + t) * p.cin_int + ci];
    } else if (p.kind == G_CONVT_W) {
        const int64_t ci_n = p.shape[0], co_n = p.shape[1];
        for (int64_t ci = 0; ci < ci_n; ++ci)
            for (int64_t co = 0; co < co_n; ++co)
                for (int q = 0; q < 4; ++q) dst[(ci * co_n + co) * 4 + q] = src[(ci * 4 + q) * co_n + co];
    } else {
        std::memcpy(dst, src, sizeof(float) * p.n_ref);
    }
}

// reference module defaults (same distributions; deterministic host stream, seed 42)
void default_init(cad_geonet* h) {
    uint64_t s = 0x2545F4914F6CDD1Dull ^ 42;
    auto rnd = [&]() {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        return (float)((s >> 40) * (1.0 / 16777216.0));
    };
    auto normal = [&]() {
        const float u1 = std::max(rnd(), 1e-7f), u2 = rnd();
        return std::sqrt(-2.f * std::log(u1)) * std::cos(6.2831853f * u2);
    };
    std::vector<float> ref, inter;
    for (const GParam& p : h->params) {
        ref.assign(p.n_ref, 0.f);
        switch (p.kind) {
            case G_BNW: case G_FILM_GAMMA_B: std::fill(ref.begin(), ref.end(), 1.f); break;
            case G_BNB: case G_FILM_BETA_B: case G_PCL_T_W: break;
            case G_PCL_T_B: ref[0] = 1.f; ref[1] = 1.f; break;   // identity transform
            case G_FILM_HEAD_W: for (auto& x : ref) x = 0.01f * normal(); break;
            default: {
                const float bound = 1.f / std::sqrt((float)p.fan_in);
                for (auto& x : ref) x = (rnd() * 2.f - 1.f) * bound;
            }
        }
        ref_to_int(p, ref.data(), inter);
        GCHK(hipMemcpy(h->flat_p + p.off, inter.data(), sizeof(float) * p.n_int, hipMemcpyHostToDevice));
    }
    for (const GBuf& b : h->bufs) {
        std::vector<float> v(b.C, b.name.find("running_var") != std::string::npos ? 1.f : 0.f);
        GCHK(hipMemcpy(b.ptr, v.data(), sizeof(float) * b.C, hipMemcpyHostToDevice));
    }
}

void geo_get(const cad_geonet* h, const float* slab, int idx, float* host, int64_t numel) {
    need(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
    const GParam& p = h->params[idx];
    need(numel == p.n_ref, "numel mismatch for " + p.name);
    std::vector<float> inter(p.n_int);
    GCHK(hipMemcpy(inter.data(), slab + p.off, sizeof(float) * p.n_int, hipMemcpyDeviceToHost));
    int_to_ref(p, inter.data(), host);
}

}  // namespace

// ============================================================================================
// C ABI (cad.h: geometry-aware family)
// ============================================================================================
extern "C" {

cad_status cad_geonet_create(const cad_geonet_desc* d, int device, cad_geonet** out) {
    return gguard([&] {
        need(d && out, "null argument");
        need(d->variant == CAD_GEONET_FULL || d->variant == CAD_GEONET_LIGHT, "unknown geonet variant");
        need(d->in_channels == 3, "in_channels must be 3");
        need(d->camera_dim == 4, "camera_dim must be 4");
        need(d->init_features >= 4 && d->init_features % 4 == 0, "init_features must be a positive multiple of 4");
        const int nl = d->variant == CAD_GEONET_FULL ? 6 : 5;
        const int div = 1 << (nl - 1);
        need(d->height > 0 && d->width > 0 && d->height % div == 0 && d->width % div == 0,
             "height/width must be positive multiples of " + std::to_string(div) +
                 " (the reference's pad branch is then a no-op)");
        need(d->max_batch >= 1, "max_batch must be >= 1");
        GCHK(hipSetDevice(device));
        auto h = std::make_unique<cad_geonet>();
        h->device = device;
        h->variant = d->variant;
        h->nl = nl;
        h->f = d->init_features;
        h->Bmax = d->max_batch;
        h->H = d->height;
        h->W = d->width;
        h->max_depth = d->max_depth;
        h->use_pcl = d->variant == CAD_GEONET_LIGHT ? true : d->use_pcl != 0;
        h->use_attention = d->variant == CAD_GEONET_LIGHT ? true : d->use_attention != 0;
        build(h.get());
        compute_stage_ranges(h.get());
        Arena sz;
        layout(h.get(), sz);
        void* base = nullptr;
        GCHK(hipMalloc(&base, sz.off + 4096));
        GCHK(hipMemset(base, 0, sz.off + 4096));
        h->base = base;
        Arena real;
        real.base = static_cast<char*>(base);
        layout(h.get(), real);
        need(real.off == sz.off, "internal: layout differs between passes", CAD_ERR_STATE);
        default_init(h.get());
        GCHK(hipDeviceSynchronize());
        *out = h.release();
    });
}

void cad_geonet_destroy(cad_geonet* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    (void)hipFree(h->base);
    delete h;
}

int64_t cad_geonet_count_parameters(const cad_geonet* h) {
    int64_t n = 0;
    for (const GParam& p : h->params) n += p.n_ref;
    return n;
}
int cad_geonet_num_tensors(const cad_geonet* h, int kind) { return kind == 0 ? (int)h->params.size() : (int)h->bufs.size(); }

cad_status cad_geonet_tensor_info(const cad_geonet* h, int kind, int idx, const char** name, int* ndim,
                                  int64_t shape[4]) {
    return gguard([&] {
        if (kind == 0) {
            need(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
            const GParam& p = h->params[idx];
            if (name) *name = p.name.c_str();
            if (ndim) *ndim = p.ndim;
            if (shape) for (int i = 0; i < 4; ++i) shape[i] = p.shape[i];
        } else {
            need(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            if (name) *name = h->bufs[idx].name.c_str();
            if (ndim) *ndim = 1;
            if (shape) { shape[0] = h->bufs[idx].C; shape[1] = shape[2] = shape[3] = 1; }
        }
    });
}

cad_status cad_geonet_set_tensor(cad_geonet* h, int kind, int idx, const float* host, int64_t numel) {
    return gguard([&] {
        GCHK(hipSetDevice(h->device));
        if (kind == 0) {
            need(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
            const GParam& p = h->params[idx];
            need(numel == p.n_ref, "numel mismatch for " + p.name);
            std::vector<float> inter;
            ref_to_int(p, host, inter);
            GCHK(hipMemcpy(h->flat_p + p.off, inter.data(), sizeof(float) * p.n_int, hipMemcpyHostToDevice));
        } else {
            need(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            need(numel == h->bufs[idx].C, "numel mismatch for " + h->bufs[idx].name);
            GCHK(hipMemcpy(h->bufs[idx].ptr, host, sizeof(float) * numel, hipMemcpyHostToDevice));
        }
    });
}

cad_status cad_geonet_get_tensor(const cad_geonet* h, int kind, int idx, float* host, int64_t numel) {
    return gguard([&] {
        GCHK(hipSetDevice(h->device));
        GCHK(hipDeviceSynchronize());
        if (kind == 0) {
            geo_get(h, h->flat_p, idx, host, numel);
        } else {
            need(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            need(numel == h->bufs[idx].C, "numel mismatch");
            GCHK(hipMemcpy(host, h->bufs[idx].ptr, sizeof(float) * numel, hipMemcpyDeviceToHost));
        }
    });
}

cad_status cad_geonet_get_grad(const cad_geonet* h, int idx, float* host, int64_t numel) {
    return gguard([&] {
        GCHK(hipSetDevice(h->device));
        GCHK(hipDeviceSynchronize());
        geo_get(h, h->flat_g, idx, host, numel);
    });
}

cad_status cad_geonet_train(cad_geonet* h, int train) {
    return gguard([&] { h->train = train != 0; });
}

cad_status cad_geonet_flat(cad_geonet* h, float** params, float** grads, int64_t* n) {
    return gguard([&] {
        if (params) *params = h->flat_p;
        if (grads) *grads = h->flat_g;
        if (n) *n = h->n_flat;
    });
}

cad_status cad_geonet_forward(cad_geonet* h, const float* rgb, const float* rays, const float* cam4, float* depth,
                              int B, void* stream) {
    return gguard([&] {
        need(rgb && rays && cam4 && depth, "null tensor");
        need(B >= 1 && B <= h->Bmax, "batch size out of range");
        GCHK(hipSetDevice(h->device));
        forward(h, rgb, rays, cam4, depth, B, S(stream));
        h->fwd_B = B;
        h->have_fwd = h->train;
        if (h->train) {
            ++h->nbt;
            if (B > 1) ++h->nbt_film;
        }
        GCHK(hipGetLastError());
    });
}

cad_status cad_geonet_backward(cad_geonet* h, const float* ddepth, void* stream) {
    return gguard([&] {
        need(h->have_fwd, "backward needs a train-mode forward first", CAD_ERR_STATE);
        GCHK(hipSetDevice(h->device));
        backward(h, ddepth, S(stream));
        GCHK(hipGetLastError());
    });
}

int cad_geonet_num_stages(const cad_geonet* h) { return h ? num_stages(h) : -1; }

cad_status cad_geonet_grad_layout(const cad_geonet_desc* d, int* nstages, int64_t stage_off[16], int64_t stage_cnt[16],
                                  int64_t* n_flat) {
    return gguard([&] {
        need(d && (d->variant == CAD_GEONET_FULL || d->variant == CAD_GEONET_LIGHT), "unknown geonet variant");
        need(d->in_channels == 3 && d->init_features >= 4 && d->init_features % 4 == 0, "bad model description");
        cad_geonet t;   // tables only: no device memory is touched
        t.variant = d->variant;
        t.nl = d->variant == CAD_GEONET_FULL ? 6 : 5;
        t.f = d->init_features;
        t.H = t.W = 1 << t.nl;
        t.use_pcl = d->variant == CAD_GEONET_LIGHT ? true : d->use_pcl != 0;
        t.use_attention = d->variant == CAD_GEONET_LIGHT ? true : d->use_attention != 0;
        build(&t);
        compute_stage_ranges(&t);
        need((int)t.stage_range.size() <= 16, "too many stages");
        if (nstages) *nstages = (int)t.stage_range.size();
        for (size_t s = 0; s < t.stage_range.size(); ++s) {
            if (stage_off) stage_off[s] = t.stage_range[s].first;
            if (stage_cnt) stage_cnt[s] = t.stage_range[s].second;
        }
        if (n_flat) *n_flat = t.n_flat;
    });
}

cad_status cad_geonet_stage_grad_range(const cad_geonet* h, int stage, int64_t* offset, int64_t* count) {
    return gguard([&] {
        need(h && stage >= 0 && stage < (int)h->stage_range.size(), "stage out of range");
        if (offset) *offset = h->stage_range[(size_t)stage].first;
        if (count) *count = h->stage_range[(size_t)stage].second;
    });
}

cad_status cad_geonet_backward_stage(cad_geonet* h, int stage, const float* ddepth, void* stream) {
    return gguard([&] {
        need(h->have_fwd, "backward needs a train-mode forward first", CAD_ERR_STATE);
        need(stage >= 0 && stage < num_stages(h), "stage out of range");
        GCHK(hipSetDevice(h->device));
        backward_stage(h, stage, ddepth, S(stream));
        GCHK(hipGetLastError());
    });
}

cad_status cad_geonet_clip_grad_norm(cad_geonet* h, float max_norm, float prescale, void* stream) {
    return gguard([&] {
        GCHK(hipSetDevice(h->device));
        cad::grad_norm_clip(h->flat_g, h->n_flat, max_norm, prescale, h->dscr, h->norm_coef, S(stream));
    });
}

cad_status cad_geonet_last_grad_norm(cad_geonet* h, float* total_norm, void* stream) {
    return gguard([&] {
        GCHK(hipStreamSynchronize(S(stream)));
        GCHK(hipMemcpy(total_norm, h->norm_coef, sizeof(float), hipMemcpyDeviceToHost));
    });
}

cad_status cad_geonet_adam_step(cad_geonet* h, float lr, float beta1, float beta2, float eps, float weight_decay,
                                void* stream) {
    return gguard([&] {
        GCHK(hipSetDevice(h->device));
        ++h->adam_t;
        cad::adam_step(h->flat_p, h->flat_g, h->adam_m, h->adam_v, h->n_flat, h->norm_coef, lr, beta1, beta2, eps,
                       weight_decay, (int)h->adam_t, S(stream));
    });
}

int64_t cad_geonet_num_batches_tracked(const cad_geonet* h, int film) { return h ? (film ? h->nbt_film : h->nbt) : -1; }

// ---- operator-level entry points (tests): one CBAM / one PCL forward + backward on device tensors.
// Parameters and gradients packed in the reference's registration order; state is allocated per
// call (test use only).
cad_status cad_op_cbam(const float* x, const float* g, const float* params, int B, int H, int W, int C, float* out,
                       float* dx, float* grads, void* stream) {
    return gguard([&] {
        need(x && g && params && out && dx && grads && B > 0 && H > 0 && W > 0 && C > 0, "bad argument");
        const int Cr = std::max(1, C / 16);
        const int64_t M = (int64_t)B * H * W, HW = (int64_t)H * W;
        Arena sz, real;
        cad::Cbam A{};
        auto lay = [&](Arena& a) {
            A.C = C; A.Cr = Cr;
            A.avg = a.f((int64_t)B * C); A.mx = a.f((int64_t)B * C); A.amax = a.i((int64_t)B * C);
            A.ha = a.f((int64_t)B * Cr); A.hm = a.f((int64_t)B * Cr); A.att = a.f((int64_t)B * C);
            A.s = a.f(2 * M); A.sidx = a.i(M); A.sa = a.f(M); A.dlog = a.f(M); A.ds = a.f(2 * M);
            A.dO = a.f((int64_t)B * C); A.dha = a.f((int64_t)B * Cr); A.dhm = a.f((int64_t)B * Cr);
            A.dva = a.f((int64_t)B * C); A.dvm = a.f((int64_t)B * C);
            return a.d(cad::attn_scratch_doubles(B, HW, C));
        };
        lay(sz);
        void* base = nullptr;
        GCHK(hipMalloc(&base, sz.off + 4096));
        real.base = static_cast<char*>(base);
        double* scr = lay(real);
        const int64_t o1 = (int64_t)Cr * C, o2 = o1 + Cr, o3 = o2 + (int64_t)C * Cr, o4 = o3 + C;
        A.w1 = params; A.b1 = params + o1; A.w2 = params + o2; A.b2 = params + o3; A.wsp = params + o4;
        A.gw1 = grads; A.gb1 = grads + o1; A.gw2 = grads + o2; A.gb2 = grads + o3; A.gwsp = grads + o4;
        cad::cbam_fwd(A, x, B, H, W, out, C, 0, scr, S(stream));
        cad::cbam_bwd(A, x, g, C, 0, B, H, W, dx, scr, S(stream));
        const hipError_t e = hipStreamSynchronize(S(stream));
        (void)hipFree(base);
        GCHK(e);
    });
}

cad_status cad_op_pcl(const float* u, const float* camn, const float* g, const float* params, int B, int H, int W,
                      int C, float* out, float* du, float* grads, float* theta, void* stream) {
    return gguard([&] {
        need(u && camn && g && params && out && du && grads && B > 0 && H > 0 && W > 0 && C > 0, "bad argument");
        const int Hd = cad::kPclHidden;
        const int64_t M = (int64_t)B * H * W, HW = (int64_t)H * W;
        Arena sz, real;
        cad::Pcl P{};
        auto lay = [&](Arena& a) {
            P.C = C;
            P.pooled = a.f((int64_t)B * C); P.h1 = a.f((int64_t)B * Hd); P.h2 = a.f((int64_t)B * Hd);
            P.tp = a.f((int64_t)B * 6); P.theta = a.f((int64_t)B * 6); P.dgrid = a.f(2 * M);
            P.dtp = a.f((int64_t)B * 6); P.dh1 = a.f((int64_t)B * Hd); P.dh2 = a.f((int64_t)B * Hd);
            P.dpooled = a.f((int64_t)B * C);
            return a.d(cad::attn_scratch_doubles(B, HW, C));
        };
        lay(sz);
        void* base = nullptr;
        GCHK(hipMalloc(&base, sz.off + 4096));
        real.base = static_cast<char*>(base);
        double* scr = lay(real);
        const int64_t K1 = C + 4, o1 = (int64_t)Hd * K1, o2 = o1 + Hd, o3 = o2 + (int64_t)Hd * Hd, o4 = o3 + Hd,
                      o5 = o4 + 6 * Hd;
        P.w1 = params; P.b1 = params + o1; P.w2 = params + o2; P.b2 = params + o3; P.w3 = params + o4; P.b3 = params + o5;
        P.gw1 = grads; P.gb1 = grads + o1; P.gw2 = grads + o2; P.gb2 = grads + o3; P.gw3 = grads + o4; P.gb3 = grads + o5;
        cad::pcl_fwd(P, u, camn, B, H, W, out, C, 0, scr, S(stream));
        cad::pcl_bwd(P, u, camn, g, C, 0, B, H, W, du, scr, S(stream));
        if (theta) (void)hipMemcpyAsync(theta, P.theta, sizeof(float) * 6 * B, hipMemcpyDeviceToDevice, S(stream));
        const hipError_t e = hipStreamSynchronize(S(stream));
        (void)hipFree(base);
        GCHK(e);
    });
}

// test hook: copies a buffer of the last step to the host (NHWC rows; int32 buffers bit-copied).
//   "cat<l>" [M][2C] decoder concat, "dcat<l>" its gradient, "x<l>" decoder output, "u<l>" ConvT output,
//   "z<l>" encoder CBAM input; CBAM decisions of encoder ("e") / decoder ("d") block l:
//   "amax<e|d><l>" [B][C] argmax pixel of the channel max-pool, "sidx<e|d><l>" [M] argmax channel;
//   "y1<e|d><l>" / "y2<e|d><l>" [M][C] the block's pre-BN conv outputs (the values BN normalised)
// returns the element count (host == nullptr: count only), -1 if unknown
int64_t cad_geonet_debug_buffer(cad_geonet* h, const char* name, float* host, int64_t numel) {
    if (!h || !name) return -1;
    const std::string n(name);
    const int B = h->fwd_B;
    if (n.size() < 2) return -1;
    const int l = n.back() - '0';
    if (l < 0 || l >= h->nl) return -1;
    std::string key = n.substr(0, n.size() - 1);
    const void* src = nullptr;
    int64_t cnt = 0;
    if (key == "amaxe" || key == "amaxd" || key == "sidxe" || key == "sidxd") {
        const bool enc = key.back() == 'e';
        if (!enc && l > h->nl - 2) return -1;
        const GBlock& b = enc ? h->enc[l] : h->dec[l].blk;
        if (b.cb0 < 0) return -1;
        if (key[0] == 'a') { src = b.A.amax; cnt = (int64_t)B * b.A.C; }
        else { src = b.A.sidx; cnt = h->Ml(l, B); }
    } else if (key == "y1e" || key == "y2e" || key == "y1d" || key == "y2d") {
        const bool enc = key.back() == 'e';
        if (!enc && l > h->nl - 2) return -1;
        const GBlock& b = enc ? h->enc[l] : h->dec[l].blk;
        src = key[1] == '1' ? b.y1 : b.y2;
        cnt = h->Ml(l, B) * h->Cl(l);
    } else if (key == "cat" && l < h->nl - 1) { src = h->cat[l]; cnt = 2 * h->Ml(l, B) * h->Cl(l); }
    else if (key == "dcat" && l < h->nl - 1) { src = h->dcat[l]; cnt = 2 * h->Ml(l, B) * h->Cl(l); }
    else if (key == "x" && l < h->nl - 1) { src = h->dec[l].x; cnt = h->Ml(l, B) * h->Cl(l); }
    else if (key == "u" && l < h->nl - 1) { src = h->dec[l].u; cnt = h->Ml(l, B) * h->Cl(l); }
    else if (key == "z" && l > 0 && h->enc[l].z) { src = h->enc[l].z; cnt = h->Ml(l, B) * h->Cl(l); }
    else return -1;
    if (!host) return cnt;
    if (numel < cnt || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(host, src, sizeof(float) * cnt, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return cnt;
}

}  // extern "C"
