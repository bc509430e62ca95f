// Config-5 network (BASELINE.json configs[4]): ResNet-50 encoder + U-Net decoder, trained with bf16
// operands on the MI355X matrix cores.  The reference has no such model:
// the architecture is defined here and checked against a torch fp32 restatement of
// the same modules (oracle/resunet_oracle.py) — parity unpinned.
//
//   encoder (torchvision ResNet-50 v1.5 layout and parameter names, prefix "encoder."):
//     conv1 7x7/2 (3 -> 64) + bn1 + relu            x1   /2    64
//     maxpool 3x3/2 p1
//     layer1 3 x Bottleneck(w 64,  out 256)          x2   /4   256
//     layer2 4 x Bottleneck(w 128, out 512, s 2)     x3   /8   512
//     layer3 6 x Bottleneck(w 256, out 1024, s 2)    x4   /16 1024
//     layer4 3 x Bottleneck(w 512, out 2048, s 2)    x5   /32 2048
//     Bottleneck: conv1 1x1, conv2 3x3 (stride s), conv3 1x1, BN after each, projection shortcut
//     (1x1 stride s + BN) on the first block, out = relu(bn3 + shortcut)
//   decoder (the baseline U-Net's stages: ConvTranspose2d(2, 2) up, cat {skip, up}, DoubleConv):
//     dec4: up 2048 -> 512, cat x4 -> DC(1536 -> 512)   /16
//     dec3: up 512 -> 256,  cat x3 -> DC(768 -> 256)    /8
//     dec2: up 256 -> 128,  cat x2 -> DC(384 -> 128)    /4
//     dec1: up 128 -> 64,   cat x1 -> DC(128 -> 64)     /2
//     dec0: up 64 -> 32            -> DC(32 -> 32)      /1
//     out_conv 1x1 (32 -> 1), sigmoid * max_depth
//
// Contractions (all on the B1 pre-split engine: bf16 operand twins, fp32 accumulation; the pre-BN
// conv outputs are stored as bf16, their BN statistics taken from the stored values):
//   3x3 stride-1 convolutions: the window kernels (conv3x3_*_ps, gemm_win.hpp / gemm_ps.hpp);
//   1x1 convolutions: dense GEMMs straight on the activation twins (stride 2: subsampled twin);
//   7x7/2 stem and 3x3/2 convolutions: im2col twin + dense GEMM, col2im gather for the dgrad;
//   ConvTranspose2d: the U-Net's kernels.  BN statistics come from the GEMM epilogues.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
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

struct RError : std::runtime_error {
    cad_status st;
    RError(cad_status s, const std::string& m) : std::runtime_error(m), st(s) {}
};
#define RCHK(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            throw RError(e_ == hipErrorOutOfMemory ? CAD_ERR_OOM : CAD_ERR_HIP,                 \
                         std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)
void need(bool c, const std::string& m, cad_status s = CAD_ERR_INVALID) {
    if (!c) throw RError(s, m);
}
template <class F>
cad_status rguard(F&& f) {
    try {
        f();
        return CAD_OK;
    } catch (const RError& e) {
        cad::set_last_error(e.what());
        return e.st;
    } catch (const std::exception& e) {
        cad::set_last_error(e.what());
        return CAD_ERR_INVALID;
    }
}
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t up8(int64_t x) { return (x + 7) & ~int64_t(7); }

// the model runs on the B1 (bf16 operand) engine whatever the process-wide engine is (the window
// kernels' block shapes, and so the BN partial counts, depend on it: layout runs under it too)
struct EngineScope {
    int prev;
    EngineScope() : prev(cad::gemm_engine()) { cad::set_gemm_engine(2); }
    ~EngineScope() { cad::set_gemm_engine(prev); }
};

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
    uint8_t* u8(int64_t n) { return static_cast<uint8_t*>(take((size_t)std::max<int64_t>(n, 1))); }
    void* tw(int64_t elems) { return take(2 * (size_t)std::max<int64_t>(elems, 1)); }   // bf16 twin
};

enum RKind { R_CONV, R_BNW, R_BNB, R_CONVT_W, R_CONVT_B, R_HEAD_W, R_HEAD_B };
struct RParam {
    std::string name;
    int ndim;
    int64_t shape[4];
    RKind kind;
    int64_t off, n_int, n_ref;
    int k = 0, cin_ref = 0, cin_int = 0, cout = 0, Kp = 0;   // convolutions
};
struct RBuf {
    std::string name;
    int64_t C;
    float* ptr;
};

struct RBN {
    int C = 0, widx = -1, bidx = -1;
    float *rm = nullptr, *rv = nullptr, *mean = nullptr, *invstd = nullptr, *scale = nullptr, *shift = nullptr,
          *coef = nullptr;
};
struct RConv {
    int pidx = -1, cin = 0, cout = 0, k = 1, s = 1, p = 0, Kp = 0;
    bool win = false;          // 3x3 stride 1: window kernels
    void *ws = nullptr;        // forward weight twin [cout][Kp]
    void *wts = nullptr;       // dgrad twin: window [cin][9][cout] repack, else W^T [Kp][cout]
    float* wd = nullptr;       // fp32 repack scratch of the window dgrad
    // MX-fp8 forward (cad_resunet_set_fp8): eligible contractions read MXFP8 operands
    bool x8 = false;
    uint8_t *wq = nullptr, *wsc = nullptr;   // forward weights [cout][ldq] e4m3 + [cout][ldq / 32] e8m0
    int64_t ldq = 0;
};
struct Unit {   // conv + BN (+ its pre-BN output y)
    RConv c;
    RBN b;
    float* y = nullptr;
};
struct Bott {
    std::string prefix;        // "encoder.layer<L>.<i>."
    Unit u1, u2, u3, ud;
    bool down = false;
    int s = 1, cin = 0, w = 0, cout = 0, H = 0, W = 0, Ho = 0, Wo = 0;   // input geometry
    void *t1s = nullptr, *t2s = nullptr, *col2 = nullptr, *xs = nullptr;
    float* out = nullptr;
    void* outs = nullptr;
};
struct Dec {
    int l = 0;                 // "dec<l>." (output at 1/2^l)
    int up_w = -1, up_b = -1, cin_up = 0, cout_up = 0, skipC = 0, C = 0, H = 0, W = 0;   // output geometry
    Unit u1, u2;
    void* cats = nullptr;      // twin [M][skipC + cout_up]
    void* a1s = nullptr;
    float* out = nullptr;
    void* outs = nullptr;
    float* dcat = nullptr;     // backward [M][Ccat]
    void *wfs = nullptr, *wms = nullptr;
    float* wf = nullptr;
};

}  // namespace

struct cad_resunet {
    int device = 0, Bmax = 1, H = 0, W = 0;
    float max_depth = 10.f;
    bool train = true;
    int fwd_B = 0;
    bool have_fwd = false;
    bool fp8 = false;          // forward conv-GEMMs on MX-fp8 operands where eligible (x8 units)
    uint8_t *xq = nullptr, *xsc = nullptr;   // MX scratch of the current contraction's A operand
    int64_t xq_cap = 0;
    // the MX copy a BN-apply pass writes of its output for the next contraction (consumed by it before
    // the next such pass runs: one buffer serves the whole forward)
    uint8_t *xqp = nullptr, *xscp = nullptr;
    int64_t nbt = 0;
    std::vector<RParam> params;
    std::vector<RBuf> bufs;
    int64_t n_flat = 0;
    float *flat_p = nullptr, *flat_g = nullptr, *adam_m = nullptr, *adam_v = nullptr;
    int64_t adam_t = 0;
    float* norm_coef = nullptr;
    void* base = nullptr;
    // encoder
    Unit stem;
    void* stem_col = nullptr;
    float* x0 = nullptr;
    float* s_out = nullptr;    // relu(bn1(conv1)) fp32 [M1][64]
    void* s_outs = nullptr;
    float* pool = nullptr;
    void* pools = nullptr;
    uint8_t* pidx = nullptr;
    std::vector<Bott> blocks;
    int stage_end[4] = {};     // blocks [stage_end[i-1], stage_end[i]) form layer i+1
    std::vector<Dec> dec;      // dec4 .. dec0
    int head_w = -1, head_b = -1;
    float* sig = nullptr;
    // scratch
    float* stats = nullptr;
    double* dscr = nullptr;
    float *slab = nullptr;
    int64_t slab_cap = 0;
    float *gA = nullptr, *gB = nullptr, *gS = nullptr, *dT = nullptr, *dcol = nullptr;
    void* dYs = nullptr;
    // staged backward (data-parallel exchange, dp.cpp): the gradient of the current stage's output,
    // and each stage's contiguous slab range [off, off + cnt)
    float* bwd_g = nullptr;
    bool bwd_masked = false;   // bwd_g already carries the ReLU mask of the block whose output it is
    bool bwd_skip_added = false;   // ... and the decoder concat's skip gradient
    std::vector<std::pair<int64_t, int64_t>> stage_range;
    float* P(int i) const { return flat_p + params[i].off; }
    float* G(int i) const { return flat_g + params[i].off; }
    int64_t M(int B, int h, int w) const { return (int64_t)B * h * w; }
};

namespace {

void add_param(cad_resunet* h, const std::string& name, std::vector<int64_t> shape, RKind kind, int k = 0,
               int cin_ref = 0, int cin_int = 0, int cout = 0, int Kp = 0) {
    RParam p;
    p.name = name;
    p.ndim = (int)shape.size();
    p.n_ref = 1;
    for (int i = 0; i < 4; ++i) p.shape[i] = i < p.ndim ? shape[i] : 1;
    for (int i = 0; i < p.ndim; ++i) p.n_ref *= shape[i];
    p.kind = kind;
    p.k = k; p.cin_ref = cin_ref; p.cin_int = cin_int; p.cout = cout; p.Kp = Kp;
    p.n_int = kind == R_CONV ? (int64_t)cout * Kp : p.n_ref;
    h->n_flat = (h->n_flat + 63) & ~int64_t(63);
    p.off = h->n_flat;
    h->n_flat += p.n_int;
    h->params.push_back(p);
}

// conv (no bias) + BN: k x k, stride s, padding k/2; cin_int = channels of the stored input rows
Unit add_unit(cad_resunet* h, const std::string& conv_name, const std::string& bn_name, int cin_ref, int cin_int,
              int cout, int k, int s) {
    Unit u;
    u.c.cin = cin_int; u.c.cout = cout; u.c.k = k; u.c.s = s; u.c.p = k / 2;
    u.c.win = k == 3 && s == 1 && cin_int % 8 == 0;
    u.c.Kp = (int)up8((int64_t)k * k * cin_int);
    add_param(h, conv_name, {cout, cin_ref, k, k}, R_CONV, k, cin_ref, cin_int, cout, u.c.Kp);
    u.c.pidx = (int)h->params.size() - 1;
    add_param(h, bn_name + ".weight", {cout}, R_BNW);
    add_param(h, bn_name + ".bias", {cout}, R_BNB);
    u.b.C = cout; u.b.widx = (int)h->params.size() - 2; u.b.bidx = (int)h->params.size() - 1;
    return u;
}

void build(cad_resunet* h) {
    // stem: the NHWC4 input (rgb + a zero channel)
    h->stem = add_unit(h, "encoder.conv1.weight", "encoder.bn1", 3, 4, 64, 7, 2);
    const int widths[4] = {64, 128, 256, 512}, nblocks[4] = {3, 4, 6, 3};
    int cin = 64, Hh = (h->H - 1) / 2 + 1, Ww = (h->W - 1) / 2 + 1;   // after conv1
    Hh = (Hh - 1) / 2 + 1; Ww = (Ww - 1) / 2 + 1;                      // after the max-pool
    for (int L = 0; L < 4; ++L) {
        for (int i = 0; i < nblocks[L]; ++i) {
            Bott b;
            const std::string pre = "encoder.layer" + std::to_string(L + 1) + "." + std::to_string(i) + ".";
            b.prefix = pre;
            b.s = (L > 0 && i == 0) ? 2 : 1;
            b.cin = cin; b.w = widths[L]; b.cout = 4 * widths[L];
            b.down = i == 0;
            b.H = Hh; b.W = Ww;
            b.Ho = (Hh - 1) / b.s + 1; b.Wo = (Ww - 1) / b.s + 1;
            b.u1 = add_unit(h, pre + "conv1.weight", pre + "bn1", cin, cin, b.w, 1, 1);
            b.u2 = add_unit(h, pre + "conv2.weight", pre + "bn2", b.w, b.w, b.w, 3, b.s);
            b.u3 = add_unit(h, pre + "conv3.weight", pre + "bn3", b.w, b.w, b.cout, 1, 1);
            if (b.down) b.ud = add_unit(h, pre + "downsample.0.weight", pre + "downsample.1", cin, cin, b.cout, 1, b.s);
            h->blocks.push_back(b);
            cin = b.cout; Hh = b.Ho; Ww = b.Wo;
        }
        h->stage_end[L] = (int)h->blocks.size();
    }
    // decoder
    const int skipC[5] = {1024, 512, 256, 64, 0}, outC[5] = {512, 256, 128, 64, 32};
    int cup = 2048;
    for (int j = 0; j < 5; ++j) {
        const int l = 4 - j;   // dec4 .. dec0, output at 1/2^l
        Dec d;
        d.l = l;
        const std::string pre = "dec" + std::to_string(l) + ".";
        d.cin_up = cup; d.cout_up = outC[j]; d.skipC = skipC[j]; d.C = outC[j];
        d.H = h->H >> l; d.W = h->W >> l;
        add_param(h, pre + "up.weight", {cup, outC[j], 2, 2}, R_CONVT_W);
        add_param(h, pre + "up.bias", {outC[j]}, R_CONVT_B);
        d.up_w = (int)h->params.size() - 2; d.up_b = (int)h->params.size() - 1;
        const int cc = skipC[j] + outC[j];
        d.u1 = add_unit(h, pre + "conv.conv1.weight", pre + "conv.bn1", cc, cc, outC[j], 3, 1);
        d.u2 = add_unit(h, pre + "conv.conv2.weight", pre + "conv.bn2", outC[j], outC[j], outC[j], 3, 1);
        h->dec.push_back(d);
        cup = outC[j];
    }
    add_param(h, "out_conv.weight", {1, 32, 1, 1}, R_HEAD_W);
    add_param(h, "out_conv.bias", {1}, R_HEAD_B);
    h->head_w = (int)h->params.size() - 2;
    h->head_b = (int)h->params.size() - 1;
    h->n_flat = (h->n_flat + 63) & ~int64_t(63);
}

inline int64_t up128(int64_t x) { return (x + 127) & ~int64_t(127); }

// MX-fp8 eligibility of a forward contraction (input width Win): the window kernel for the 3x3
// stride-1 convolutions, the dense GEMM for the 1x1 / im2col ones (K = Kp)
bool x8_eligible(const RConv& c, int Win) {
    if (c.win) return cad::conv3x3_x8_ok(c.cin, Win, c.cout);
    return c.Kp % 32 == 0 && cad::dense_x8_ok(c.Kp, c.cout);
}
// rows and channels of the A operand the contraction reads (window: the input; dense: the input,
// its stride-2 subsample or its im2col rows)
void x8_operand_shape(const RConv& c, int B, int Hin, int Win, int64_t& rows, int& chans) {
    const int Ho = (Hin + 2 * c.p - c.k) / c.s + 1, Wo = (Win + 2 * c.p - c.k) / c.s + 1;
    if (c.win) { rows = (int64_t)B * Hin * Win; chans = c.cin; }
    else if (c.k == 1) { rows = (int64_t)B * Ho * Wo; chans = c.cin; }
    else { rows = (int64_t)B * Ho * Wo; chans = c.Kp; }
}

void bn_alloc(Arena& a, RBN& b) {
    b.rm = a.f(b.C); b.rv = a.f(b.C);
    b.mean = a.f(b.C); b.invstd = a.f(b.C); b.scale = a.f(b.C); b.shift = a.f(b.C); b.coef = a.f(3 * b.C);
}
void conv_alloc(Arena& a, RConv& c) {
    c.ws = a.tw((int64_t)c.cout * c.Kp);
    if (c.win) {
        c.wd = a.f((int64_t)c.cout * c.Kp);
        c.wts = a.tw((int64_t)c.cout * c.Kp);
    } else {
        c.wts = a.tw((int64_t)c.cout * c.Kp);
    }
}

void layout(cad_resunet* h, Arena& a) {
    const int B = h->Bmax;
    h->flat_p = a.f(h->n_flat);
    h->flat_g = a.f(h->n_flat);
    h->adam_m = a.f(h->n_flat);
    h->adam_v = a.f(h->n_flat);
    h->norm_coef = a.f(4);
    const int H1 = (h->H - 1) / 2 + 1, W1 = (h->W - 1) / 2 + 1;
    const int64_t M0 = h->M(B, h->H, h->W), M1 = h->M(B, H1, W1);
    int64_t maxMC = 0, maxRows2C = 0, maxCol = 0, maxX8 = 0;
    auto track = [&](int64_t M, int C) { maxMC = std::max(maxMC, M * C); };
    // MX-fp8 forward of a unit on a B x Hin x Win input: weights, A-operand scratch, BN partial rows
    auto x8_prep = [&](Unit& u, int Hin, int Win) {
        RConv& c = u.c;
        c.x8 = x8_eligible(c, Win);
        if (!c.x8) return;
        c.ldq = up128(c.Kp);
        c.wq = a.u8((int64_t)c.cout * c.ldq);
        c.wsc = a.u8((int64_t)c.cout * (c.ldq >> 5));
        int64_t rows = 0;
        int chans = 0;
        x8_operand_shape(c, B, Hin, Win, rows, chans);
        maxX8 = std::max(maxX8, rows * up128(chans));
        const int Ho = (Hin + 2 * c.p - c.k) / c.s + 1, Wo = (Win + 2 * c.p - c.k) / c.s + 1;
        const int srows = c.win ? cad::conv3x3_x8_stats_rows(c.cin, B, Hin, Win, c.cout)
                                : cad::dense_x8_stats_rows(h->M(B, Ho, Wo), c.cout);
        maxRows2C = std::max<int64_t>(maxRows2C, (int64_t)srows * (2 * c.cout + 1));
    };
    // stem
    h->x0 = a.f(M0 * 4);
    RConv& sc = h->stem.c;
    conv_alloc(a, sc);
    bn_alloc(a, h->stem.b);
    h->stem_col = a.tw(M1 * sc.Kp);
    h->stem.y = a.f(M1 * 64);
    h->s_out = a.f(M1 * 64);
    h->s_outs = a.tw(M1 * 64);
    const int H2 = (H1 - 1) / 2 + 1, W2 = (W1 - 1) / 2 + 1;
    const int64_t M2 = h->M(B, H2, W2);
    h->pool = a.f(M2 * 64);
    h->pools = a.tw(M2 * 64);
    h->pidx = a.u8(M2 * 64);
    track(M1, 64);
    maxRows2C = std::max<int64_t>(maxRows2C, (int64_t)cad::dense_stats_rows(M1, 64) * 129);
    for (Bott& b : h->blocks) {
        const int64_t Mi = h->M(B, b.H, b.W), Mo = h->M(B, b.Ho, b.Wo);
        for (Unit* u : {&b.u1, &b.u2, &b.u3, &b.ud}) {
            if (u->c.pidx < 0) continue;
            conv_alloc(a, u->c);
            bn_alloc(a, u->b);
            x8_prep(*u, u == &b.u3 ? b.Ho : b.H, u == &b.u3 ? b.Wo : b.W);
        }
        b.u1.y = a.f(Mi * b.w);
        b.t1s = a.tw(Mi * b.w);
        if (!b.u2.c.win) {
            b.col2 = a.tw(Mo * b.u2.c.Kp);
            maxCol = std::max<int64_t>(maxCol, Mo * b.u2.c.Kp);
        }
        b.u2.y = a.f(Mo * b.w);
        b.t2s = a.tw(Mo * b.w);
        b.u3.y = a.f(Mo * b.cout);
        if (b.down) {
            b.ud.y = a.f(Mo * b.cout);
            if (b.s == 2) b.xs = a.tw(Mo * b.cin);
        }
        b.out = a.f(Mo * b.cout);
        b.outs = a.tw(Mo * b.cout);
        track(Mi, std::max(b.w, b.cin));
        track(Mo, b.cout);
        for (const Unit* u : {&b.u1, &b.u2, &b.u3, &b.ud}) {
            if (u->c.pidx < 0) continue;
            const int64_t Mu = u == &b.u1 ? Mi : Mo;
            maxRows2C = std::max<int64_t>(maxRows2C, (int64_t)cad::dense_stats_rows(Mu, u->c.cout) * (2 * u->c.cout + 1));
            maxRows2C = std::max<int64_t>(
                maxRows2C, (int64_t)cad::conv3x3_stats_rows(u->c.cin, B, b.H, b.W, u->c.cout, true) * (2 * u->c.cout + 1));
        }
    }
    for (Dec& d : h->dec) {
        const int64_t Md = h->M(B, d.H, d.W);
        const int cc = d.skipC + d.cout_up;
        d.cats = a.tw(Md * cc);
        d.wf = a.f((int64_t)4 * d.cout_up * d.cin_up);
        d.wfs = a.tw((int64_t)4 * d.cout_up * d.cin_up);
        d.wms = a.tw((int64_t)4 * d.cout_up * d.cin_up);
        for (Unit* u : {&d.u1, &d.u2}) {
            conv_alloc(a, u->c);
            bn_alloc(a, u->b);
            x8_prep(*u, d.H, d.W);
            u->y = a.f(Md * d.C);
            maxRows2C = std::max<int64_t>(
                maxRows2C, (int64_t)cad::conv3x3_stats_rows(u->c.cin, B, d.H, d.W, d.C, true) * (2 * d.C + 1));
            maxRows2C = std::max<int64_t>(maxRows2C, (int64_t)cad::dense_stats_rows(Md, d.C) * (2 * d.C + 1));
        }
        d.a1s = a.tw(Md * d.C);
        d.out = a.f(Md * d.C);
        d.outs = a.tw(Md * d.C);
        d.dcat = a.f(Md * cc);
        track(Md, cc);
    }
    h->sig = a.f(M0);
    h->stats = a.f(maxRows2C);
    h->dscr = a.d((int64_t)(cad::colsum_slices(M0) + 2) * 4 * 2048 + 4 * 2048 + 8192);
    h->gA = a.f(maxMC);
    h->gB = a.f(maxMC);
    h->gS = a.f(maxMC);
    h->dT = a.f(maxMC);
    h->dYs = a.tw(maxMC);
    h->dcol = a.f(std::max<int64_t>(maxCol, 1));
    h->xq_cap = maxX8;
    h->xq = a.u8(maxX8);
    h->xsc = a.u8(maxX8 / 32);
    h->xqp = a.u8(maxX8);
    h->xscp = a.u8(maxX8 / 32);
    int64_t sl = 0;
    for (const RParam& p : h->params)
        if (p.kind == R_CONV) sl = std::max<int64_t>(sl, (int64_t)p.cout * p.Kp * 64);
    h->slab_cap = std::min<int64_t>(std::max<int64_t>(sl, 1 << 20), (int64_t)64 << 20);
    h->slab = a.f(h->slab_cap);
    // buffers: running statistics in parameter order of the BNs
    h->bufs.clear();
    for (const RParam& p : h->params)
        if (p.kind == R_BNW) {
            const std::string pre = p.name.substr(0, p.name.size() - 6);   // strip "weight"
            // find the BN struct owning this parameter
            RBN* bn = nullptr;
            auto chk = [&](Unit& u) { if (u.b.widx >= 0 && h->params[u.b.widx].name == p.name) bn = &u.b; };
            chk(h->stem);
            for (Bott& b : h->blocks) { chk(b.u1); chk(b.u2); chk(b.u3); chk(b.ud); }
            for (Dec& d : h->dec) { chk(d.u1); chk(d.u2); }
            h->bufs.push_back({pre + "running_mean", p.shape[0], bn ? bn->rm : nullptr});
            h->bufs.push_back({pre + "running_var", p.shape[0], bn ? bn->rv : nullptr});
        }
}

// reference <-> internal layouts
void ref_to_int(const RParam& p, const float* src, std::vector<float>& dst) {
    dst.assign(p.n_int, 0.f);
    if (p.kind == R_CONV) {   // (co, ci, ky, kx) -> [co][(ky*k + kx)*cin_int + ci], zero pad
        const int kk = p.k * p.k;
        for (int co = 0; co < p.cout; ++co)
            for (int ci = 0; ci < p.cin_ref; ++ci)
                for (int t = 0; t < kk; ++t)
                    dst[(int64_t)co * p.Kp + (int64_t)t * p.cin_int + ci] = src[((int64_t)co * p.cin_ref + ci) * kk + t];
    } else if (p.kind == R_CONVT_W) {   // (ci, co, dy, dx) -> [ci][q][co]
        const int64_t ci_n = p.shape[0], co_n = p.shape[1];
        for (int64_t ci = 0; ci < ci_n; ++ci)
            for (int64_t co = 0; co < co_n; ++co)
                for (int q = 0; q < 4; ++q) dst[(ci * 4 + q) * co_n + co] = src[(ci * co_n + co) * 4 + q];
    } else {
        std::memcpy(dst.data(), src, sizeof(float) * p.n_ref);
    }
}
void int_to_ref(const RParam& p, const float* src, float* dst) {
    if (p.kind == R_CONV) {
        const int kk = p.k * p.k;
        for (int co = 0; co < p.cout; ++co)
            for (int ci = 0; ci < p.cin_ref; ++ci)
                for (int t = 0; t < kk; ++t)
                    dst[((int64_t)co * p.cin_ref + ci) * kk + t] = src[(int64_t)co * p.Kp + (int64_t)t * p.cin_int + ci];
    } else if (p.kind == R_CONVT_W) {
        const int64_t ci_n = p.shape[0], co_n = p.shape[1];
        for (int64_t ci = 0; ci < ci_n; ++ci)
            for (int64_t co = 0; co < co_n; ++co)
                for (int q = 0; q < 4; ++q) dst[(ci * co_n + co) * 4 + q] = src[(ci * 4 + q) * co_n + co];
    } else {
        std::memcpy(dst, src, sizeof(float) * p.n_ref);
    }
}

// torch module defaults: conv / ConvT / Linear weights and biases U(+-1/sqrt(fan_in)), BN 1 / 0,
// running stats 0 / 1 (deterministic host stream)
void default_init(cad_resunet* h) {
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        return (float)((s >> 40) * (1.0 / 16777216.0));
    };
    std::vector<float> ref, inter;
    for (size_t i = 0; i < h->params.size(); ++i) {
        const RParam& p = h->params[i];
        ref.assign(p.n_ref, 0.f);
        if (p.kind == R_BNW) std::fill(ref.begin(), ref.end(), 1.f);
        else if (p.kind != R_BNB) {
            int64_t fan_in;
            if (p.kind == R_CONV) fan_in = (int64_t)p.cin_ref * p.k * p.k;
            else if (p.kind == R_CONVT_W) fan_in = p.shape[1] * 4;
            else if (p.kind == R_CONVT_B) fan_in = h->params[i - 1].shape[1] * 4;
            else fan_in = 32;
            const float bound = 1.f / std::sqrt((float)fan_in);
            for (auto& x : ref) x = (rnd() * 2.f - 1.f) * bound;
        }
        ref_to_int(p, ref.data(), inter);
        RCHK(hipMemcpy(h->flat_p + p.off, inter.data(), sizeof(float) * p.n_int, hipMemcpyHostToDevice));
    }
    for (const RBuf& b : h->bufs) {
        std::vector<float> v(b.C, b.name.find("running_var") != std::string::npos ? 1.f : 0.f);
        RCHK(hipMemcpy(b.ptr, v.data(), sizeof(float) * b.C, hipMemcpyHostToDevice));
    }
}

cad::Split tw(const void* p, int64_t ld, int coff = 0) {
    cad::Split v;
    v.p = p; v.ld = ld; v.coff = coff;
    return v;
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// conv of unit u on input twin `in` (B x Hin x Win, ld ldin, coff); y = pre-BN output [Mo][cout]
// (+ BN partials in train mode), then the BN coefficients.  col: im2col buffer (k > 1 or s > 1 and
// not the window path); xs: the stride-2 1x1 input subsample buffer.
// the MX-fp8 copy of unit u's input that its producer pass can write (nullptr: u quantises itself —
// not fp8, or its A operand is an im2col / subsampled copy of the input); C = the input's channels
// CAD_MXPREQ=0: every fp8 contraction quantises its operand itself (mx8_quantize), none is written
// by the producing pass (A/B switch; bit-identical: tests/test_gpu_resunet_switches.py)
bool mx_preq_on() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_MXPREQ");
        return !(e && e[0] == '0');
    }();
    return on;
}
const cad::Mx8* preq_for(cad_resunet* h, const Unit& u, int64_t rows, cad::Mx8& m) {
    const RConv& c = u.c;
    if (!mx_preq_on() || !h->fp8 || !c.x8 || !(c.win || (c.k == 1 && c.s == 1)) || c.cin % 32 || rows * up128(c.cin) > h->xq_cap)
        return nullptr;
    m.q = h->xqp; m.s = h->xscp; m.ld = up128(c.cin); m.coff = 0;
    return &m;
}

// preq: the input's MX copy, already written by the producing pass (preq_for)
void unit_fwd(cad_resunet* h, Unit& u, cad::Split in, int B, int Hin, int Win, void* col, void* xs, hipStream_t st,
              const cad::Mx8* preq = nullptr) {
    RConv& c = u.c;
    const int Ho = (Hin + 2 * c.p - c.k) / c.s + 1, Wo = (Win + 2 * c.p - c.k) / c.s + 1;
    const int64_t Mo = h->M(B, Ho, Wo);
    float* stats = h->train ? h->stats : nullptr;
    int rows = 0;
    if (h->fp8 && c.x8) {   // MX-fp8 operand (quantised from the bf16 twin), fp8 MFMA contraction
        cad::Split a = in;
        int64_t arows = 0;
        int chans = 0;
        x8_operand_shape(c, B, Hin, Win, arows, chans);
        if (!c.win && c.s > 1) {
            if (c.k == 1) {
                cad::copy_twin(in, c.cin, B, Hin, Win, c.s, xs, c.cin, 0, st);
                a = tw(xs, c.cin);
            } else {
                cad::im2col_ps(in, c.cin, B, Hin, Win, c.k, c.k, c.s, c.p, col, c.Kp, st);
                a = tw(col, c.Kp);
            }
        }
        cad::Mx8 xa, wa;
        xa.q = h->xq; xa.s = h->xsc; xa.ld = up128(chans);
        wa.q = c.wq; wa.s = c.wsc; wa.ld = c.ldq;
        if (arows * xa.ld > h->xq_cap) throw RError(CAD_ERR_INVALID, "MX-fp8 scratch too small");
        if (preq && (c.win || (c.k == 1 && c.s == 1)) && preq->ld == xa.ld) xa = *preq;
        else cad::mx8_quantize(a.p, true, a.ld, a.coff, chans, arows, xa, st);
        if (c.win) {
            cad::conv3x3_fwd_x8(xa, c.cin, wa, c.cout, u.y, c.cout, 0, B, Hin, Win, stats, st, true);
            rows = cad::conv3x3_x8_stats_rows(c.cin, B, Hin, Win, c.cout);
        } else {
            cad::dense_fwd_x8(xa, c.Kp, wa, c.cout, u.y, c.cout, 0, Mo, stats, st, true);
            rows = cad::dense_x8_stats_rows(Mo, c.cout);
        }
    } else if (c.win) {
        cad::conv3x3_fwd_ps(in, c.cin, tw(c.ws, c.Kp), c.cout, u.y, c.cout, 0, B, Hin, Win, stats, st, true);
        rows = cad::conv3x3_stats_rows(c.cin, B, Hin, Win, c.cout, true);
    } else {
        cad::Split a = in;
        if (c.k > 1 || c.s > 1) {
            if (c.k == 1) {   // 1x1 stride 2: subsampled twin
                cad::copy_twin(in, c.cin, B, Hin, Win, c.s, xs, c.cin, 0, st);
                a = tw(xs, c.cin);
            } else if (col) {
                cad::im2col_ps(in, c.cin, B, Hin, Win, c.k, c.k, c.s, c.p, col, c.Kp, st);
                a = tw(col, c.Kp);
            }
        }
        cad::dense_fwd_ps(a, c.Kp, tw(c.ws, c.Kp), c.cout, u.y, c.cout, 0, Mo, stats, st, true);
        rows = cad::dense_stats_rows(Mo, c.cout);
    }
    RBN& b = u.b;
    if (h->train)
        cad::bn_fwd_finalize(h->stats, rows, b.C, Mo, h->P(b.widx), h->P(b.bidx), b.rm, b.rv, 0.1f, 1e-5f, h->dscr, b.mean,
                             b.invstd, b.scale, b.shift, st);
    else
        cad::bn_eval_coeffs(h->P(b.widx), h->P(b.bidx), b.rm, b.rv, b.C, 1e-5f, b.mean, b.invstd, b.scale, b.shift, st);
}

// the per-step weight conversions (bf16 twins, dgrad / ConvT repacks, transposes) batched into
// k_weight_prep launches of up to kWPrepMaxJobs tensors each (one launch per tensor before: ~70 small
// launches per forward and per backward)
// CAD_WPREPBATCH=0: one k_weight_prep launch per tensor (A/B switch; bit-identical:
// tests/test_gpu_resunet_switches.py)
int wprep_batch() {
    static const int n = [] {
        const char* e = std::getenv("CAD_WPREPBATCH");
        return (e && e[0] == '0') ? 1 : cad::kWPrepMaxJobs;
    }();
    return n;
}
struct PrepBatch {
    cad::WPrepList L{};
    hipStream_t st;
    explicit PrepBatch(hipStream_t s) : st(s) {}
    void add(int kind, const float* src, float* d32, void* d16, int cout, int cin, int64_t n) {
        if (L.njobs == wprep_batch()) flush();
        cad::WPrepJob& j = L.job[L.njobs++];
        j.src = src; j.d32 = d32; j.d16 = d16; j.kind = kind; j.cout = cout; j.cin = cin; j.n = n;
    }
    void flush() {
        if (L.njobs) cad::weight_prep(L, st);
        L.njobs = 0;
    }
    // the owner flushes explicitly; unwinding from an exception drops the pending jobs (a destructor
    // must not launch, nor throw: weight_prep can)
    ~PrepBatch() = default;
};

void prep_weights_fwd(cad_resunet* h, hipStream_t st) {
    PrepBatch pb(st);
    cad::Mx8WList xl;   // the fp8 weights, quantised from the fp32 parameters in one launch
    auto sw = [&](RConv& c) {   // bf16 twin of [cout][Kp] (split_rows' rounding)
        pb.add(cad::WPREP_SPLIT, h->P(c.pidx), nullptr, c.ws, c.cout, c.Kp, (int64_t)c.cout * c.Kp);
        if (h->fp8 && c.x8) {
            if (xl.njobs == cad::kMx8WMaxJobs) {
                cad::mx8_quantize_weights(xl, st);
                xl.njobs = 0;
            }
            cad::Mx8WJob& j = xl.job[xl.njobs++];
            j.src = h->P(c.pidx); j.q = c.wq; j.s = c.wsc; j.ldq = c.ldq; j.rows = c.cout; j.C = c.Kp; j.blk0 = 0;
        }
    };
    sw(h->stem.c);
    for (Bott& b : h->blocks)
        for (Unit* u : {&b.u1, &b.u2, &b.u3, &b.ud})
            if (u->c.pidx >= 0) sw(u->c);
    for (Dec& d : h->dec) {
        sw(d.u1.c);
        sw(d.u2.c);
        // repack_convT_fwd + its twin
        pb.add(cad::WPREP_CONVT, h->P(d.up_w), d.wf, d.wfs, d.cout_up, d.cin_up, (int64_t)4 * d.cout_up * d.cin_up);
    }
    pb.flush();
    cad::mx8_quantize_weights(xl, st);
}

void forward(cad_resunet* h, const float* rgb, float* depth, int B, hipStream_t st) {
    prep_weights_fwd(h, st);
    const int H1 = (h->H - 1) / 2 + 1, W1 = (h->W - 1) / 2 + 1;
    const int64_t M1 = h->M(B, H1, W1);
    // stem: conv1 (im2col of the NHWC4 fp32 input) + bn1 + relu, max-pool
    cad::rgb_to_nhwc4(rgb, h->x0, B, h->H, h->W, st);
    RConv& sc = h->stem.c;
    cad::im2col_f32(h->x0, 4, 0, 4, B, h->H, h->W, 7, 7, 2, 3, h->stem_col, sc.Kp, st);
    {
        float* stats = h->train ? h->stats : nullptr;
        cad::dense_fwd_ps(tw(h->stem_col, sc.Kp), sc.Kp, tw(sc.ws, sc.Kp), 64, h->stem.y, 64, 0, M1, stats, st, true);
        RBN& b = h->stem.b;
        if (h->train)
            cad::bn_fwd_finalize(h->stats, cad::dense_stats_rows(M1, 64), 64, M1, h->P(b.widx), h->P(b.bidx), b.rm, b.rv,
                                 0.1f, 1e-5f, h->dscr, b.mean, b.invstd, b.scale, b.shift, st);
        else
            cad::bn_eval_coeffs(h->P(b.widx), h->P(b.bidx), b.rm, b.rv, 64, 1e-5f, b.mean, b.invstd, b.scale, b.shift, st);
        cad::bn_relu_fwd(h->stem.y, 64, b.scale, b.shift, h->s_out, 64, 0, M1, st, h->s_outs, 64, 0, true);
    }
    cad::maxpool3s2_fwd(h->s_out, 64, B, H1, W1, h->pool, h->pidx, h->pools, st);
    // bottlenecks
    const float* xf = h->pool;
    const void* xsw = h->pools;
    // in fp8 mode each BN-apply pass also writes the MX copy its consumer contracts (preq_for): the
    // bytes mx8_quantize would write from the twin, without re-reading it
    const cad::Mx8* pq = nullptr;   // the MX copy of the next block's input, written by bn_add_relu
    cad::Mx8 mnext;
    for (size_t bi = 0; bi < h->blocks.size(); ++bi) {
        Bott& b = h->blocks[bi];
        const int64_t Mi = h->M(B, b.H, b.W), Mo = h->M(B, b.Ho, b.Wo);
        cad::Mx8 m2, m3;
        unit_fwd(h, b.u1, tw(xsw, b.cin), B, b.H, b.W, nullptr, nullptr, st, pq);
        const cad::Mx8* q2 = preq_for(h, b.u2, Mi, m2);
        cad::bn_relu_fwd(b.u1.y, b.w, b.u1.b.scale, b.u1.b.shift, nullptr, b.w, 0, Mi, st, b.t1s, b.w, 0, true, q2);
        unit_fwd(h, b.u2, tw(b.t1s, b.w), B, b.H, b.W, b.col2, nullptr, st, q2);
        const cad::Mx8* q3 = preq_for(h, b.u3, Mo, m3);
        cad::bn_relu_fwd(b.u2.y, b.w, b.u2.b.scale, b.u2.b.shift, nullptr, b.w, 0, Mo, st, b.t2s, b.w, 0, true, q3);
        unit_fwd(h, b.u3, tw(b.t2s, b.w), B, b.Ho, b.Wo, nullptr, nullptr, st, q3);
        if (b.down) unit_fwd(h, b.ud, tw(xsw, b.cin), B, b.H, b.W, nullptr, b.xs, st);
        pq = bi + 1 < h->blocks.size() ? preq_for(h, h->blocks[bi + 1].u1, Mo, mnext) : nullptr;
        cad::bn_add_relu(b.u3.y, b.u3.b.scale, b.u3.b.shift, b.down ? b.ud.y : nullptr, b.ud.b.scale, b.ud.b.shift, xf,
                         b.cin, b.cout, Mo, b.out, b.outs, st, true, pq);
        xf = b.out;
        xsw = b.outs;
    }
    // decoder
    const void* skips[5] = {h->blocks[h->stage_end[2] - 1].outs, h->blocks[h->stage_end[1] - 1].outs,
                            h->blocks[h->stage_end[0] - 1].outs, h->s_outs, nullptr};
    const void* prev = h->blocks.back().outs;
    for (size_t j = 0; j < h->dec.size(); ++j) {
        Dec& d = h->dec[j];
        const int cc = d.skipC + d.cout_up;
        const int64_t Md = h->M(B, d.H, d.W);
        cad::convT_fwd_ps(tw(prev, d.cin_up), d.cin_up, tw(d.wfs, d.cin_up), h->P(d.up_b), d.cout_up,
                          static_cast<float*>(d.cats), cc, d.skipC, B, d.H / 2, d.W / 2, st, true);
        if (d.skipC) cad::copy_twin(tw(skips[j], d.skipC), d.skipC, B, d.H, d.W, 1, d.cats, cc, 0, st);
        unit_fwd(h, d.u1, tw(d.cats, cc), B, d.H, d.W, nullptr, nullptr, st);
        cad::Mx8 m2;
        const cad::Mx8* q2 = preq_for(h, d.u2, Md, m2);
        cad::bn_relu_fwd(d.u1.y, d.C, d.u1.b.scale, d.u1.b.shift, nullptr, d.C, 0, Md, st, d.a1s, d.C, 0, true, q2);
        unit_fwd(h, d.u2, tw(d.a1s, d.C), B, d.H, d.W, nullptr, nullptr, st, q2);
        cad::bn_relu_fwd(d.u2.y, d.C, d.u2.b.scale, d.u2.b.shift, d.out, d.C, 0, Md, st, d.outs, d.C, 0, true);
        prev = d.outs;
    }
    cad::head_fwd(h->dec.back().out, 32, h->P(h->head_w), h->P(h->head_b), h->max_depth, h->sig, depth,
                  h->M(B, h->H, h->W), st);
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
void prep_weights_bwd(cad_resunet* h, hipStream_t st) {
    PrepBatch pb(st);
    auto dw = [&](RConv& c) {
        if (c.win)   // repack_conv_dgrad + its twin
            pb.add(cad::WPREP_DGRAD, h->P(c.pidx), c.wd, c.wts, c.cout, c.cin, (int64_t)c.cout * 9 * c.cin);
        else         // transpose_split: [cout][Kp] -> bf16 [Kp][cout]
            pb.add(cad::WPREP_TRANSPOSE, h->P(c.pidx), nullptr, c.wts, c.cout, c.Kp, (int64_t)c.cout * c.Kp);
    };
    for (Bott& b : h->blocks)
        for (Unit* u : {&b.u1, &b.u2, &b.u3, &b.ud})
            if (u->c.pidx >= 0) dw(u->c);
    for (Dec& d : h->dec) {
        dw(d.u1.c);
        dw(d.u2.c);
        pb.add(cad::WPREP_SPLIT, h->P(d.up_w), nullptr, d.wms, d.cout_up, d.cin_up, (int64_t)4 * d.cout_up * d.cin_up);
    }
    pb.flush();
}

// BN (+ReLU) backward of unit u: g (ld ldg, coff) -> dYs twin; then the conv's wgrad from the
// input twin `in` (or its col / subsample) and, if dx, its dgrad into dx (ld lddx, overwritten)
// add: a matrix added to the 1x1 stride-1 dgrad output (the identity shortcut's gradient)
// g_bf16: g is bf16 rows (ldg elements); dx_bf16: dx is written as bf16 rows (window / 1x1 stride-1
// dgrads only) — the input gradients of a bottleneck's conv2 / conv3 and of a decoder's conv2, which
// only the BN backward of the unit below reads
// hi / ldhi / split_n: the window dgrad's split store (columns >= split_n as bf16 rows of hi); returns
// whether it ran
bool unit_bwd(cad_resunet* h, Unit& u, const float* g, int64_t ldg, int gcoff, bool relu, cad::Split in, int B,
              int Hin, int Win, const void* col, const void* xs, float* dx, int64_t lddx, hipStream_t st,
              const float* add = nullptr, bool g_bf16 = false, bool dx_bf16 = false, const float* mask = nullptr,
              int64_t ldadd = 0, void* hi = nullptr, int64_t ldhi = 0, int split_n = 0) {
    RConv& c = u.c;
    const int Ho = (Hin + 2 * c.p - c.k) / c.s + 1, Wo = (Win + 2 * c.p - c.k) / c.s + 1;
    const int64_t Mo = h->M(B, Ho, Wo);
    RBN& b = u.b;
    cad::bn_relu_bwd(g, ldg, gcoff, u.y, b.C, b.mean, b.invstd, b.scale, b.shift, h->P(b.widx), Mo, h->dscr, b.coef,
                     h->G(b.widx), h->G(b.bidx), nullptr, st, nullptr, 1, h->dYs, relu, true, nullptr, g_bf16);
    const cad::Split dz = tw(h->dYs, c.cout);
    need(!dx_bf16 || !add, "unit_bwd: a bf16 input gradient with an added matrix");
    if (c.win) {
        cad::conv3x3_wgrad_ps(dz, c.cout, in, c.cin, h->G(c.pidx), B, Hin, Win, h->slab, h->slab_cap, st);
        return dx && cad::conv3x3_dgrad_ps(dz, c.cout, tw(c.wts, 9 * c.cout), c.cin, dx, lddx, B, Hin, Win, st, dx_bf16,
                                           hi, ldhi, split_n);
    }
    cad::Split a = in;
    if (c.k == 1 && c.s > 1) a = tw(xs, c.cin);
    else if (c.k > 1 || c.s > 1) a = tw(col, c.Kp);
    cad::dense_wgrad_ps(dz, c.cout, a, c.Kp, h->G(c.pidx), c.Kp, Mo, h->slab, h->slab_cap, st);
    if (!dx) return false;
    if (c.k == 1 && c.s == 1) {
        cad::dense_fwd_ps(dz, c.cout, tw(c.wts, c.cout), c.cin, dx, lddx, 0, Mo, nullptr, st, dx_bf16, add, mask, ldadd);
        return false;
    }
    need(!dx_bf16 && !mask, "unit_bwd: bf16 / masked input gradient of a strided / im2col convolution");
    if (c.k == 1) {   // stride-2 1x1: dgrad on the subsampled grid, scattered by the caller
        cad::dense_fwd_ps(dz, c.cout, tw(c.wts, c.cout), c.cin, dx, c.cin, 0, Mo, nullptr, st);
    } else {
        cad::dense_fwd_ps(dz, c.cout, tw(c.wts, c.cout), c.Kp, h->dcol, c.Kp, 0, Mo, nullptr, st);
        cad::col2im(h->dcol, c.Kp, c.cin, B, Hin, Win, c.k, c.k, c.s, c.p, dx, lddx, st);
    }
    return false;
}

// Backward in stages whose parameter gradients are contiguous, decreasing-offset slab ranges (the
// registration order is stem, layer1..layer4, dec4..dec0, head): 0 head, 1..5 dec0..dec4, then the
// bottleneck blocks from layer4's last to layer1's first, last the stem.  A stage writes only its own
// range, so the data-parallel exchange can all-reduce a finished range while later stages run.
int num_stages(const cad_resunet* h) { return 6 + (int)h->blocks.size() + 1; }

// CAD_MASKFUSE=0: the separate k_relu_mask pass for every block (A/B switch; bit-identical)
bool mask_fuse_on() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_MASKFUSE");
        return !(e && e[0] == '0');
    }();
    return on;
}

// CAD_UPSPLIT=0: the decoder conv1 input gradient's up half split into the ConvT operand by a pass
// (A/B switch; bit-identical)
bool up_split_on() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_UPSPLIT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// CAD_SKIPFUSE=0: the decoder skip gradients and the stride-1 projection's dgrad added by separate
// passes (A/B switch; the skip gradient's add order differs: fp32 rounding)
bool fuse_skip_on() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_SKIPFUSE");
        return !(e && e[0] == '0');
    }();
    return on;
}

void backward_stage(cad_resunet* h, int stage, const float* ddepth, hipStream_t st) {
    const int B = h->fwd_B;
    const int nb = (int)h->blocks.size();
    if (stage == 0) {   // head
        prep_weights_bwd(h, st);
        Dec& d0 = h->dec.back();
        h->bwd_g = h->gA;
        h->bwd_masked = h->bwd_skip_added = false;
        cad::head_bwd(d0.out, 32, h->P(h->head_w), ddepth, h->sig, h->max_depth, h->bwd_g, h->M(B, h->H, h->W),
                      h->dscr, h->G(h->head_w), h->G(h->head_b), st);
        return;
    }
    float* g = h->bwd_g;
    if (stage <= 5) {   // decoder: h->dec[4] (dec0) first
        const int j = 5 - stage;
        Dec& d = h->dec[j];
        const void* prev = j == 0 ? h->blocks.back().outs : h->dec[j - 1].outs;
        const int cc = d.skipC + d.cout_up;
        const int64_t Md = h->M(B, d.H, d.W);
        unit_bwd(h, d.u2, g, d.C, 0, true, tw(d.a1s, d.C), B, d.H, d.W, nullptr, nullptr, h->dT, d.C, st, nullptr,
                 false, true);
        // conv1's input gradient: the skip half fp32 into dcat (the encoder's skip adds read it), the up half
        // straight into the ConvT's bf16 operand (the window dgrad's split store; dec0, all up half: the
        // dgrad's bf16 output), else split from dcat by a pass (split_rows' rounding, the same values).
        // The operand goes to dT — free once bn1's backward has read conv2's input gradient from it — not
        // to dYs, which the dgrad itself reads (its dz)
        void* dup = h->dT;
        bool up_done;
        if (d.skipC == 0 && up_split_on()) {
            unit_bwd(h, d.u1, h->dT, d.C, 0, true, tw(d.cats, cc), B, d.H, d.W, nullptr, nullptr,
                     static_cast<float*>(dup), d.cout_up, st, nullptr, true, true);
            up_done = true;
        } else {
            up_done = unit_bwd(h, d.u1, h->dT, d.C, 0, true, tw(d.cats, cc), B, d.H, d.W, nullptr, nullptr, d.dcat, cc, st,
                               nullptr, true, false, nullptr, 0, up_split_on() ? dup : nullptr, d.cout_up, d.skipC);
        }
        if (!up_done) cad::split_rows(d.dcat, cc, d.skipC, d.cout_up, Md, dup, d.cout_up, 0, st);
        // ConvTranspose backward on the up half; its bias gradient sums the same bf16 gradient
        cad::convT_wgrad_ps(tw(prev, d.cin_up), d.cin_up, tw(dup, d.cout_up), d.cout_up, h->G(d.up_w), B, d.H / 2,
                            d.W / 2, h->slab, h->slab_cap, st);
        cad::colsum_bf16(dup, d.cout_up, 0, Md, d.cout_up, h->dscr, st);
        cad::colsum_finalize(h->dscr, cad::colsum_slices(Md), d.cout_up, h->G(d.up_b), 1.f, st);
        float* gn = g == h->gA ? h->gB : h->gA;
        cad::convT_dgrad_ps(tw(dup, d.cout_up), d.cout_up, tw(d.wms, 4 * d.cout_up), d.cin_up, gn, B, d.H / 2,
                            d.W / 2, st);
        h->bwd_g = gn;
        h->bwd_masked = h->bwd_skip_added = false;
        return;
    }
    if (stage < 6 + nb) {   // encoder bottleneck block bi; g = gradient of its output
        const int bi = nb - 1 - (stage - 6);
        Bott& b = h->blocks[bi];
        const int stage_last[3] = {h->stage_end[0] - 1, h->stage_end[1] - 1, h->stage_end[2] - 1};
        // skip gradients of the decoder concat (x4 = layer3, x3 = layer2, x2 = layer1 outputs)
        for (int L = 0; L < 3; ++L)
            if (bi == stage_last[L] && !h->bwd_skip_added) {
                need(!h->bwd_masked, "resunet backward: a masked gradient at a skip block");
                const Dec& d = h->dec[2 - L];
                cad::add_strided(g, b.cout, d.dcat, d.skipC + d.cout_up, 0, b.cout, B, b.Ho, b.Wo, 1, st);
            }
        const void* xsw = bi ? h->blocks[bi - 1].outs : h->pools;
        const int64_t Mo = h->M(B, b.Ho, b.Wo);
        // gS = g [out > 0]: already so when the next block's conv1 dgrad epilogue applied the mask
        float* gS = h->bwd_masked ? g : h->gS;
        if (!h->bwd_masked) cad::relu_mask(g, b.cout, 0, b.out, b.cout, Mo, h->gS, st);
        float* gn = g == h->gA ? h->gB : h->gA;   // gradient of the block input
        // identity shortcut (bi > 0: the input is block bi - 1's output, no skip add lands on it — a
        // layer's last block is followed by a projection block): the conv1 dgrad epilogue adds gS and
        // applies block bi - 1's ReLU mask (k_relu_mask fused)
        const bool fuse_mask = !b.down && bi > 0 && mask_fuse_on();
        const float* mask = fuse_mask ? h->blocks[bi - 1].out : nullptr;
        // a projection block after a layer's last block (bi - 1): the decoder concat's skip gradient of
        // that block's output added in this block's conv1 dgrad epilogue (its own row stride)
        const float* skip = nullptr;
        int64_t ldskip = 0;
        for (int L = 0; L < 3; ++L)
            if (b.down && bi - 1 == stage_last[L] && fuse_skip_on()) {
                const Dec& d = h->dec[2 - L];
                skip = d.dcat;
                ldskip = d.skipC + d.cout_up;
            }
        // conv3's and (stride 1) conv2's input gradients stored as bf16 (unit_bwd)
        const bool g2 = b.u2.c.win;
        unit_bwd(h, b.u3, gS, b.cout, 0, false, tw(b.t2s, b.w), B, b.Ho, b.Wo, nullptr, nullptr, h->dT, b.w, st,
                 nullptr, false, true);
        unit_bwd(h, b.u2, h->dT, b.w, 0, true, tw(b.t1s, b.w), B, b.H, b.W, b.col2, nullptr, h->dT, b.w, st, nullptr,
                 true, g2);
        // identity shortcut: its gradient gS is added inside conv1's dgrad epilogue
        unit_bwd(h, b.u1, h->dT, b.w, 0, true, tw(xsw, b.cin), B, b.H, b.W, nullptr, nullptr, gn, b.cin, st,
                 b.down ? skip : gS, g2, false, mask, ldskip);
        if (b.down && b.s == 1 && fuse_skip_on()) {   // the projection's dgrad added to gn in place
            unit_bwd(h, b.ud, gS, b.cout, 0, false, tw(xsw, b.cin), B, b.H, b.W, nullptr, b.xs, gn, b.cin, st, gn);
        } else if (b.down) {
            unit_bwd(h, b.ud, gS, b.cout, 0, false, tw(xsw, b.cin), B, b.H, b.W, nullptr, b.xs, h->dT, b.cin, st);
            cad::add_strided(gn, b.cin, h->dT, b.cin, 0, b.cin, B, b.H, b.W, b.s, st);
        }
        h->bwd_g = gn;
        h->bwd_masked = fuse_mask;
        h->bwd_skip_added = skip != nullptr;
        return;
    }
    // stem: max-pool backward, the dec1 skip gradient (x1), bn1 + relu, conv1 weight gradient
    const int H1 = (h->H - 1) / 2 + 1, W1 = (h->W - 1) / 2 + 1;
    const int64_t M1 = h->M(B, H1, W1);
    float* gs = g == h->gA ? h->gB : h->gA;
    const Dec& d1 = h->dec[3];
    if (fuse_skip_on()) {   // the dec1 skip gradient added in the gather (the same single add per element)
        cad::maxpool3s2_bwd(g, h->pidx, 64, B, H1, W1, gs, st, d1.dcat, d1.skipC + d1.cout_up);
    } else {
        cad::maxpool3s2_bwd(g, h->pidx, 64, B, H1, W1, gs, st);
        cad::add_strided(gs, 64, d1.dcat, d1.skipC + d1.cout_up, 0, 64, B, H1, W1, 1, st);
    }
    RBN& sb = h->stem.b;
    cad::bn_relu_bwd(gs, 64, 0, h->stem.y, 64, sb.mean, sb.invstd, sb.scale, sb.shift, h->P(sb.widx), M1, h->dscr, sb.coef,
                     h->G(sb.widx), h->G(sb.bidx), nullptr, st, nullptr, 1, h->dYs, true, true);
    cad::dense_wgrad_ps(tw(h->dYs, 64), 64, tw(h->stem_col, h->stem.c.Kp), h->stem.c.Kp, h->G(h->stem.c.pidx),
                        h->stem.c.Kp, M1, h->slab, h->slab_cap, st);
}

void backward(cad_resunet* h, const float* ddepth, hipStream_t st) {
    for (int s = 0; s < num_stages(h); ++s) backward_stage(h, s, ddepth, st);
}

// the slab range of each stage, from the parameter names (checked contiguous: no other stage's
// parameter inside it)
void compute_stage_ranges(cad_resunet* h) {
    std::vector<std::vector<std::string>> pre;
    pre.push_back({"out_conv."});
    for (int j = 4; j >= 0; --j) pre.push_back({"dec" + std::to_string(h->dec[j].l) + "."});
    for (int bi = (int)h->blocks.size() - 1; bi >= 0; --bi) pre.push_back({h->blocks[bi].prefix});
    pre.push_back({"encoder.conv1.", "encoder.bn1."});
    h->stage_range.clear();
    std::vector<int> owner(h->params.size(), -1);
    for (size_t s = 0; s < pre.size(); ++s) {
        int64_t lo = INT64_MAX, hi = -1;
        for (size_t i = 0; i < h->params.size(); ++i)
            for (const std::string& p : pre[s])
                if (h->params[i].name.compare(0, p.size(), p) == 0) {
                    if (owner[i] >= 0) throw std::logic_error("parameter in two backward stages: " + h->params[i].name);
                    owner[i] = (int)s;
                    lo = std::min(lo, h->params[i].off);
                    hi = std::max(hi, h->params[i].off + h->params[i].n_int);
                }
        if (hi < 0) throw std::logic_error("empty backward stage");
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

}  // namespace

// ============================================================================================
// C ABI (cad.h: config-5 network)
// ============================================================================================
extern "C" {

cad_status cad_resunet_create(const cad_resunet_desc* d, int device, cad_resunet** out) {
    return rguard([&] {
        need(d && out, "null argument");
        need(d->in_channels == 3, "in_channels must be 3");
        need(d->height > 0 && d->width > 0 && d->height % 32 == 0 && d->width % 32 == 0,
             "height/width must be positive multiples of 32");
        need(d->max_batch >= 1, "max_batch must be >= 1");
        RCHK(hipSetDevice(device));
        auto h = std::make_unique<cad_resunet>();
        h->device = device;
        h->Bmax = d->max_batch;
        h->H = d->height;
        h->W = d->width;
        h->max_depth = d->max_depth;
        EngineScope es;
        build(h.get());
        compute_stage_ranges(h.get());
        Arena sz;
        layout(h.get(), sz);
        void* base = nullptr;
        RCHK(hipMalloc(&base, sz.off + 4096));
        RCHK(hipMemset(base, 0, sz.off + 4096));
        h->base = base;
        Arena real;
        real.base = static_cast<char*>(base);
        layout(h.get(), real);
        need(real.off == sz.off, "internal: layout differs between passes", CAD_ERR_STATE);
        default_init(h.get());
        RCHK(hipDeviceSynchronize());
        *out = h.release();
    });
}

void cad_resunet_destroy(cad_resunet* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    (void)hipFree(h->base);
    delete h;
}

int64_t cad_resunet_count_parameters(const cad_resunet* h) {
    int64_t n = 0;
    for (const RParam& p : h->params) n += p.n_ref;
    return n;
}
int cad_resunet_num_tensors(const cad_resunet* h, int kind) { return kind == 0 ? (int)h->params.size() : (int)h->bufs.size(); }

cad_status cad_resunet_tensor_info(const cad_resunet* h, int kind, int idx, const char** name, int* ndim,
                                   int64_t shape[4]) {
    return rguard([&] {
        if (kind == 0) {
            need(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
            const RParam& p = h->params[idx];
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

cad_status cad_resunet_set_tensor(cad_resunet* h, int kind, int idx, const float* host, int64_t numel) {
    return rguard([&] {
        RCHK(hipSetDevice(h->device));
        if (kind == 0) {
            need(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
            const RParam& p = h->params[idx];
            need(numel == p.n_ref, "numel mismatch for " + p.name);
            std::vector<float> inter;
            ref_to_int(p, host, inter);
            RCHK(hipMemcpy(h->flat_p + p.off, inter.data(), sizeof(float) * p.n_int, hipMemcpyHostToDevice));
        } else {
            need(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            need(numel == h->bufs[idx].C, "numel mismatch for " + h->bufs[idx].name);
            RCHK(hipMemcpy(h->bufs[idx].ptr, host, sizeof(float) * numel, hipMemcpyHostToDevice));
        }
    });
}

static void res_get(const cad_resunet* h, const float* slab, int idx, float* host, int64_t numel) {
    need(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
    const RParam& p = h->params[idx];
    need(numel == p.n_ref, "numel mismatch for " + p.name);
    std::vector<float> inter(p.n_int);
    RCHK(hipMemcpy(inter.data(), slab + p.off, sizeof(float) * p.n_int, hipMemcpyDeviceToHost));
    int_to_ref(p, inter.data(), host);
}

cad_status cad_resunet_get_tensor(const cad_resunet* h, int kind, int idx, float* host, int64_t numel) {
    return rguard([&] {
        RCHK(hipSetDevice(h->device));
        RCHK(hipDeviceSynchronize());
        if (kind == 0) {
            res_get(h, h->flat_p, idx, host, numel);
        } else {
            need(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            need(numel == h->bufs[idx].C, "numel mismatch");
            RCHK(hipMemcpy(host, h->bufs[idx].ptr, sizeof(float) * numel, hipMemcpyDeviceToHost));
        }
    });
}

cad_status cad_resunet_get_grad(const cad_resunet* h, int idx, float* host, int64_t numel) {
    return rguard([&] {
        RCHK(hipSetDevice(h->device));
        RCHK(hipDeviceSynchronize());
        res_get(h, h->flat_g, idx, host, numel);
    });
}

cad_status cad_resunet_train(cad_resunet* h, int train) {
    return rguard([&] { h->train = train != 0; });
}

cad_status cad_resunet_set_fp8(cad_resunet* h, int on) {
    return rguard([&] {
        need(h, "null network");
        h->fp8 = on != 0;
    });
}

int cad_resunet_fp8_units(const cad_resunet* h) {
    if (!h) return -1;
    int n = 0;
    auto cnt = [&](const Unit& u) { n += u.c.pidx >= 0 && u.c.x8; };
    cnt(h->stem);
    for (const Bott& b : h->blocks) { cnt(b.u1); cnt(b.u2); cnt(b.u3); cnt(b.ud); }
    for (const Dec& d : h->dec) { cnt(d.u1); cnt(d.u2); }
    return n;
}

cad_status cad_resunet_flat(cad_resunet* h, float** params, float** grads, int64_t* n) {
    return rguard([&] {
        if (params) *params = h->flat_p;
        if (grads) *grads = h->flat_g;
        if (n) *n = h->n_flat;
    });
}

cad_status cad_resunet_forward(cad_resunet* h, const float* rgb, float* depth, int B, void* stream) {
    return rguard([&] {
        need(B >= 1 && B <= h->Bmax, "batch size out of range");
        RCHK(hipSetDevice(h->device));
        EngineScope es;
        forward(h, rgb, depth, B, S(stream));
        h->fwd_B = B;
        h->have_fwd = h->train;
        if (h->train) ++h->nbt;
        RCHK(hipGetLastError());
    });
}

cad_status cad_resunet_backward(cad_resunet* h, const float* ddepth, void* stream) {
    return rguard([&] {
        need(h->have_fwd, "backward needs a train-mode forward first", CAD_ERR_STATE);
        RCHK(hipSetDevice(h->device));
        EngineScope es;
        backward(h, ddepth, S(stream));
        RCHK(hipGetLastError());
    });
}

// Test hook (tests/test_gpu_fullsize_bf16.py): a buffer of the last train-mode forward as fp32 rows.
//   "y:<conv>"      the pre-BN output of convolution <conv> ("encoder.conv1", "encoder.layer2.0.conv2",
//                   "encoder.layer1.0.downsample.0", "dec3.conv.conv1", ...): the stored bf16 values, widened
//   "scale:<bn>" / "shift:<bn>"  the BN-apply coefficients of BatchNorm <bn> ("encoder.layer1.0.bn1", ...):
//                   a BN-ReLU's decision is fma(y, scale, shift) > 0, as k_bn_relu_fwd / _bwd evaluate it
//   "out:<block>"   a bottleneck's output relu(bn3 + shortcut) ("encoder.layer1.0"), "out:encoder.stem"
//                   relu(bn1(conv1)), "out:dec<l>" a decoder block's output (fp32)
// Returns the element count (host == nullptr: only the count), -1 for an unknown name.
int64_t cad_resunet_debug_buffer(cad_resunet* h, const char* name, float* host, int64_t numel) {
    int64_t cnt = -1;
    cad_status st = rguard([&] {
        need(h && name, "null argument");
        const std::string n(name);
        const int B = h->fwd_B > 0 ? h->fwd_B : h->Bmax;
        const int H1 = (h->H - 1) / 2 + 1, W1 = (h->W - 1) / 2 + 1;
        const void* p = nullptr;
        bool bf16 = false;
        auto conv_name = [&](const Unit& u) {
            const std::string& w = h->params[u.c.pidx].name;
            return w.substr(0, w.size() - 7);   // strip ".weight"
        };
        auto bn_name = [&](const Unit& u) {
            const std::string& w = h->params[u.b.widx].name;
            return w.substr(0, w.size() - 7);
        };
        auto unit = [&](const Unit& u, int64_t M) {
            if (u.c.pidx < 0) return;
            if (n == "y:" + conv_name(u)) { p = u.y; bf16 = true; cnt = M * u.c.cout; }
            else if (n == "scale:" + bn_name(u)) { p = u.b.scale; cnt = u.b.C; }
            else if (n == "shift:" + bn_name(u)) { p = u.b.shift; cnt = u.b.C; }
        };
        unit(h->stem, h->M(B, H1, W1));
        if (n == "out:encoder.stem") { p = h->s_out; cnt = h->M(B, H1, W1) * 64; }
        for (const Bott& b : h->blocks) {
            unit(b.u1, h->M(B, b.H, b.W));
            for (const Unit* u : {&b.u2, &b.u3, &b.ud}) unit(*u, h->M(B, b.Ho, b.Wo));
            if (n == "out:" + b.prefix.substr(0, b.prefix.size() - 1)) { p = b.out; cnt = h->M(B, b.Ho, b.Wo) * b.cout; }
        }
        for (const Dec& d : h->dec) {
            unit(d.u1, h->M(B, d.H, d.W));
            unit(d.u2, h->M(B, d.H, d.W));
            if (n == "out:dec" + std::to_string(d.l)) { p = d.out; cnt = h->M(B, d.H, d.W) * d.C; }
            if (n == "cat:dec" + std::to_string(d.l)) { p = d.cats; bf16 = true; cnt = h->M(B, d.H, d.W) * (d.skipC + d.cout_up); }
        }
        need(p != nullptr, "unknown debug buffer '" + n + "'");
        if (!host) return;
        need(numel >= cnt, "debug buffer: host array too small");
        RCHK(hipSetDevice(h->device));
        RCHK(hipDeviceSynchronize());
        if (bf16) {
            std::vector<uint16_t> tmp((size_t)cnt);
            RCHK(hipMemcpy(tmp.data(), p, sizeof(uint16_t) * cnt, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < cnt; ++i) {
                const uint32_t u = (uint32_t)tmp[(size_t)i] << 16;
                std::memcpy(host + i, &u, 4);
            }
        } else {
            RCHK(hipMemcpy(host, p, sizeof(float) * cnt, hipMemcpyDeviceToHost));
        }
    });
    return st == CAD_OK ? cnt : -1;
}

int cad_resunet_num_stages(const cad_resunet* h) { return h ? num_stages(h) : -1; }

cad_status cad_resunet_grad_layout(int* nstages, int64_t stage_off[32], int64_t stage_cnt[32], int64_t* n_flat) {
    return rguard([&] {
        cad_resunet t;   // tables only: no device memory is touched
        t.H = t.W = 64;
        build(&t);
        compute_stage_ranges(&t);
        need((int)t.stage_range.size() <= 32, "too many stages");
        if (nstages) *nstages = (int)t.stage_range.size();
        for (size_t s = 0; s < t.stage_range.size(); ++s) {
            if (stage_off) stage_off[s] = t.stage_range[s].first;
            if (stage_cnt) stage_cnt[s] = t.stage_range[s].second;
        }
        if (n_flat) *n_flat = t.n_flat;
    });
}

cad_status cad_resunet_stage_grad_range(const cad_resunet* h, int stage, int64_t* offset, int64_t* count) {
    return rguard([&] {
        need(h && stage >= 0 && stage < (int)h->stage_range.size(), "stage out of range");
        if (offset) *offset = h->stage_range[(size_t)stage].first;
        if (count) *count = h->stage_range[(size_t)stage].second;
    });
}

cad_status cad_resunet_backward_stage(cad_resunet* h, int stage, const float* ddepth, void* stream) {
    return rguard([&] {
        need(h->have_fwd, "backward needs a train-mode forward first", CAD_ERR_STATE);
        need(stage >= 0 && stage < num_stages(h), "stage out of range");
        RCHK(hipSetDevice(h->device));
        EngineScope es;
        backward_stage(h, stage, ddepth, S(stream));
        RCHK(hipGetLastError());
    });
}

cad_status cad_resunet_clip_grad_norm(cad_resunet* h, float max_norm, float prescale, void* stream) {
    return rguard([&] {
        RCHK(hipSetDevice(h->device));
        cad::grad_norm_clip(h->flat_g, h->n_flat, max_norm, prescale, h->dscr, h->norm_coef, S(stream));
    });
}

cad_status cad_resunet_last_grad_norm(cad_resunet* h, float* total_norm, void* stream) {
    return rguard([&] {
        RCHK(hipStreamSynchronize(S(stream)));
        RCHK(hipMemcpy(total_norm, h->norm_coef, sizeof(float), hipMemcpyDeviceToHost));
    });
}

// torch::optim::Adam step (coupled L2), moments owned by the model; uses the clip coefficient of the
// last cad_resunet_clip_grad_norm
cad_status cad_resunet_adam_step(cad_resunet* h, float lr, float beta1, float beta2, float eps, float weight_decay,
                                 void* stream) {
    return rguard([&] {
        RCHK(hipSetDevice(h->device));
        ++h->adam_t;
        cad::adam_step(h->flat_p, h->flat_g, h->adam_m, h->adam_v, h->n_flat, h->norm_coef, lr, beta1, beta2, eps,
                       weight_decay, (int)h->adam_t, S(stream));
    });
}

}  // extern "C"
