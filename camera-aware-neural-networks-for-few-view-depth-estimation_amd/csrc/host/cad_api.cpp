// libcad_hip.so — host runtime behind include/cad/cad.h.
//
// Owns the U-Net's device state (flat parameter/gradient slabs, BN buffers, activation arena sized
// at create time — no allocation inside a step, so a step is hipGraph-capturable) and sequences the
// HIP kernels of csrc/kernels for BaselineUNetImpl::forward (baseline_unet.h:174-195), its
// backward, CombinedDepthLoss (depth_loss.h:366-433), clip_grad_norm_ and Adam
// (tensorboard_trainer_enhanced.h:287-304).
//
// Activation layout per level l (H_l = H >> l, C_l = f << l), NHWC fp32:
//   enc/bottleneck: y1, a1, y2 [M_l][C_l] (conv outputs pre-BN and a1 = relu(bn1(y1)) feeding
//         conv2); output written straight into cat_l[:, 0:C_l]
//   cat_l [M_l][2 C_l] = decoder concat buffer {skip | up} (baseline_unet.h:98, skip first) — the
//         encoder writes the skip half, the ConvTranspose epilogue writes the up half: no cat/pad.
//   pool_l [M_l][C_{l-1}] + uint8 argmax; dec: y1d, a1d, y2d, d_l [M_l][C_l].
// Backward scratch: S_a, S_b [M_0][C_0], S_c [M_1][C_0]; dcat_l [M_l][2 C_l].
//
// Config-3 models (cad_unet_create_model): every DoubleConv also owns a FiLMLayer (film_layer.h);
// its a1 = FiLM(relu(bn1(y1))) is materialised [M_l][C_l] (conv2 reads it, conv2's wgrad too), and
// the FiLM MLPs of all nine blocks run at the start of the forward (they only see the camera).
// RAY_FILM's enc1 reads NHWC8 [rgb | rays | 0 0] built on device from the intrinsics.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/cad/cad.h"
#include "../kernels/kernels.hpp"

namespace {

thread_local std::string g_err;

struct CadError : std::runtime_error {
    cad_status st;
    CadError(cad_status s, const std::string& m) : std::runtime_error(m), st(s) {}
};

#define HIPCHK(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            throw CadError(e_ == hipErrorOutOfMemory ? CAD_ERR_OOM : CAD_ERR_HIP,               \
                           std::string(#expr) + ": " + hipGetErrorString(e_));                 \
    } while (0)

void require(bool c, const std::string& m, cad_status s = CAD_ERR_INVALID) {
    if (!c) throw CadError(s, m);
}

template <class F>
cad_status guard(F&& f) {
    try {
        f();
        return CAD_OK;
    } catch (const CadError& e) {
        g_err = e.what();
        return e.st;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CAD_ERR_INVALID;
    }
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// bump allocator over one hipMalloc; run once with base == nullptr to size it
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
};

enum PKind {
    P_CONV3, P_BNW, P_BNB, P_CONVT_W, P_CONVT_B, P_HEAD_W, P_HEAD_B,
    P_FC_W, P_FC_B,                                  // FiLM fc1 / fc2 (torch::nn::Linear defaults)
    P_FILM_HEAD_W, P_FILM_GAMMA_B, P_FILM_BETA_B     // fc_gamma / fc_beta (film_layer.h:68-71)
};

struct PInfo {
    std::string name;
    int ndim;
    int64_t shape[4];
    PKind kind;
    int64_t off;      // offset in the flat slab (floats)
    int64_t n_int;    // internal element count
    int64_t n_ref;    // reference element count
    int cin_ref = 0, cin_int = 0, cout = 0;
};

struct BufInfo {
    std::string name;
    int64_t C;
    float* ptr;
};

struct BN {
    int C = 0, widx = -1, bidx = -1;
    float *rm = nullptr, *rv = nullptr;
    float *mean = nullptr, *invstd = nullptr, *scale = nullptr, *shift = nullptr, *coef = nullptr;
};
struct Conv {
    int pidx = -1, cin = 0, cout = 0;
    float* wd = nullptr;   // dgrad repack
    void *ws = nullptr, *wds = nullptr;   // pre-split weights / dgrad repack (cin % 8 == 0 only)
};
struct Film {
    int p0 = -1;   // index of film.fc1.weight; the 12 FiLM parameters follow in registration order
    float *rm1, *rv1, *rm2, *rv2;
    float *xh1, *h1, *xh2, *h2, *is1, *is2, *gam, *bet, *dgam, *dbet, *dh2, *dh1;
};
struct DoubleConv {
    Conv c1, c2;
    BN b1, b2;
    Film film;     // film.p0 < 0: plain DoubleConv
    int level = 0;
    float *y1 = nullptr, *a1 = nullptr, *y2 = nullptr;
    bool y1b = false, y2b = false;   // y1 / y2 hold bf16 values (bf16 engine, pre-split conv of the last forward)
    // conv1 keeps fp32 outputs on the bf16 engine: enc1 on the raw (non-negative) rgb, whose BN mean is
    // many standard deviations from zero, so bf16-stored values would cost x-hat several % (measured:
    // enc1.bn1 gradients 5x further from fp64 than the fp32 oracle's)
    bool y1_f32 = false;
    void* a1s = nullptr;   // pre-split a1 (gemm_ps.hpp)
    int first_param = 0, last_param = 0;   // [first, last] indices in named_parameters()
    bool has_film() const { return film.p0 >= 0; }
};
struct Up {
    int widx = -1, bidx = -1, cin = 0, cout = 0;
    float* wf = nullptr;   // forward repack [q][co][ci]
    void *wfs = nullptr, *wms = nullptr;   // pre-split forward repack / weights [ci][q][co]
};

}  // namespace

namespace cad {
void set_last_error(const std::string& msg) { g_err = msg; }
}  // namespace cad

struct cad_unet {
    int device = 0;
    int model = CAD_MODEL_BASELINE;
    int in_ch = 3, f = 64, Bmax = 1, H = 0, W = 0;
    int x0_ld = 8;               // NHWC8: rgb + zero channels (baseline, film) or rgb + rays (ray_film)
    float* camn = nullptr;       // normalised intrinsics (Bmax x 4) of the last forward
    float max_depth = 10.f;
    bool train = true;
    bool have_fwd = false;
    // BatchNorm num_batches_tracked (torch::save state): the BatchNorm2d layers count every
    // train-mode forward, FiLM's BatchNorm1d only those with B > 1 (film_layer.h:85,91)
    int64_t nbt = 0, nbt_film = 0;
    int fwd_B = 0;
    std::vector<PInfo> params;
    std::vector<BufInfo> bufs;
    int64_t n_flat = 0;
    float *flat_p = nullptr, *flat_g = nullptr;
    float* norm_coef = nullptr;   // [norm, coef]
    void* arena_base = nullptr;
    // The backward's parameter-gradient work — FiLM MLP backwards always, conv2 / conv1 / ConvT weight
    // gradients and the ConvT bias sums on the S3 engine (wgrad_stream) — runs on `side`, forked from the
    // step's stream as soon as its operands exist, beside the chain dgrad -> BN backward -> dgrad that the
    // next stage waits on (it writes only parameter gradients and its own scratch: slab, dscr2).  bn2 / bn1 of a block write their dL/dz into
    // two buffer pairs (Sb / dYs, Sb2 / dYs2); before rewriting a pair the step's stream waits for the
    // side's last reader of it (evA, evB).  Joined at the end of every stage, or once at the end of a
    // whole backward (cad_unet_backward; the staged API and the DP exchange need each stage complete).
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, evA = nullptr, evB = nullptr, ev_tail = nullptr;
    bool defer_join = false;
    float* Sb2 = nullptr;
    void* dYs2 = nullptr;
    double* dscr2 = nullptr;
    // model structure
    DoubleConv enc[5];   // enc1..enc4 = levels 0..3, bottleneck = level 4
    DoubleConv dec[4];   // dec1..dec4 at levels 0..3 (index = level)
    Up up[4];            // dec_l.up: level l+1 -> l
    int head_w = -1, head_b = -1;
    // activations
    float* x0 = nullptr;
    float* cat[4] = {};
    float* pool[5] = {};
    uint8_t* pidx[5] = {};
    float* a2_bott = nullptr;
    float* dout[4] = {};   // decoder outputs d_l
    float* sig = nullptr;
    // pre-split operand twins (gemm_ps.hpp, bf16): written by their producer on the B1 engine, read by
    // the pre-split GEMMs; fwd_np = planes of the last forward (0: fp32 operands only)
    void* x0s = nullptr;          // the NHWC8 input's twin (enc1.conv1 on the pre-split kernels)
    void* cats[4] = {};
    void* pools[5] = {};
    void* botts = nullptr;
    void* douts[4] = {};          // l = 1..3 (dout[0] feeds only the head)
    void* dcats[4] = {};          // up half of dcat, [M_l][C_l]
    void* dskips[4] = {};         // skip half of dcat, [M_l][C_l] (the bf16 engine's encoder bn2 gradient)
    void* dYs = nullptr;          // split dL/dz scratch (largest level)
    int fwd_np = 0;
    // the last forward ran decoder level 0's bn2 + ReLU fused with the head (head_fusable): dout[0]
    // was not written, the backward rebuilds the head's input gradient per row
    bool head_fused = false;
    // backward
    float* dcat[4] = {};
    float *Sa = nullptr, *Sb = nullptr, *Sc = nullptr;
    float* stats = nullptr;    // conv-epilogue BN partials
    double* dscr = nullptr;    // column-reduction scratch
    float* slab = nullptr;
    int64_t slab_cap = 0;
    // per-tile BN-backward sums of bn1 from conv2's input-gradient epilogue (conv3x3_dgrad_*_bnsums):
    // tiles of >= 128 rows at any level fit its 64-row level-0 sizing; reduced right after the GEMM
    // that writes it
    double* rc_part = nullptr;
    int64_t part_cap = 0;
    // stage grad ranges
    std::vector<std::pair<int64_t, int64_t>> stage_range;

    int Hl(int l) const { return H >> l; }
    int Wl(int l) const { return W >> l; }
    int Cl(int l) const { return f << l; }
    int64_t Ml(int l, int B) const { return (int64_t)B * Hl(l) * Wl(l); }
    float* P(int i) const { return flat_p + params[i].off; }
    float* G(int i) const { return flat_g + params[i].off; }
};

struct cad_loss {
    int device = 0, Bmax = 0, H = 0, W = 0;
    float w[4];
    cad::LossWorkspace ws{};
    float* out5 = nullptr;
    void* base = nullptr;
};

struct cad_adam {
    cad_unet* model = nullptr;
    cad_adam_opts o{};
    float *m = nullptr, *v = nullptr;
    int64_t step = 0;
};

namespace {

// ------------------------------------------------------------------------------------------
// model construction: parameter table in named_parameters() order (baseline_unet.h:147-165)
// ------------------------------------------------------------------------------------------
void add_param(cad_unet* h, const std::string& name, std::vector<int64_t> shape, PKind kind, int cin_ref = 0,
               int cin_int = 0, int cout = 0) {
    PInfo p;
    p.name = name;
    p.ndim = (int)shape.size();
    p.n_ref = 1;
    for (int i = 0; i < 4; ++i) p.shape[i] = i < p.ndim ? shape[i] : 1;
    for (int i = 0; i < p.ndim; ++i) p.n_ref *= shape[i];
    p.kind = kind;
    p.cin_ref = cin_ref; p.cin_int = cin_int; p.cout = cout;
    p.n_int = kind == P_CONV3 ? (int64_t)cout * 9 * cin_int : p.n_ref;
    h->n_flat = (h->n_flat + 63) & ~int64_t(63);
    p.off = h->n_flat;
    h->n_flat += p.n_int;
    h->params.push_back(p);
}

void add_film(cad_unet* h, DoubleConv& dc, const std::string& pre, int C) {
    // FiLMLayerImpl ctor registration order (film_layer.h:55-66): fc1, fc2, fc_gamma, fc_beta, bn1, bn2
    const int H1 = cad::kFilmH1, H2 = cad::kFilmH2;
    dc.film.p0 = (int)h->params.size();
    add_param(h, pre + "fc1.weight", {H1, 4}, P_FC_W);
    add_param(h, pre + "fc1.bias", {H1}, P_FC_B);
    add_param(h, pre + "fc2.weight", {H2, H1}, P_FC_W);
    add_param(h, pre + "fc2.bias", {H2}, P_FC_B);
    add_param(h, pre + "fc_gamma.weight", {C, H2}, P_FILM_HEAD_W);
    add_param(h, pre + "fc_gamma.bias", {C}, P_FILM_GAMMA_B);
    add_param(h, pre + "fc_beta.weight", {C, H2}, P_FILM_HEAD_W);
    add_param(h, pre + "fc_beta.bias", {C}, P_FILM_BETA_B);
    add_param(h, pre + "bn1.weight", {H1}, P_BNW);
    add_param(h, pre + "bn1.bias", {H1}, P_BNB);
    add_param(h, pre + "bn2.weight", {H2}, P_BNW);
    add_param(h, pre + "bn2.bias", {H2}, P_BNB);
}

void add_double_conv(cad_unet* h, DoubleConv& dc, const std::string& pre, int cin_ref, int cin_int, int cout, int level) {
    dc.level = level;
    dc.first_param = (int)h->params.size();
    add_param(h, pre + "conv1.weight", {cout, cin_ref, 3, 3}, P_CONV3, cin_ref, cin_int, cout);
    dc.c1 = Conv{(int)h->params.size() - 1, cin_int, cout, nullptr};
    add_param(h, pre + "bn1.weight", {cout}, P_BNW);
    add_param(h, pre + "bn1.bias", {cout}, P_BNB);
    dc.b1.C = cout; dc.b1.widx = (int)h->params.size() - 2; dc.b1.bidx = (int)h->params.size() - 1;
    add_param(h, pre + "conv2.weight", {cout, cout, 3, 3}, P_CONV3, cout, cout, cout);
    dc.c2 = Conv{(int)h->params.size() - 1, cout, cout, nullptr};
    add_param(h, pre + "bn2.weight", {cout}, P_BNW);
    add_param(h, pre + "bn2.bias", {cout}, P_BNB);
    dc.b2.C = cout; dc.b2.widx = (int)h->params.size() - 2; dc.b2.bidx = (int)h->params.size() - 1;
    if (h->model != CAD_MODEL_BASELINE) add_film(h, dc, pre + "film.", cout);   // intrinsics_unet.h:34
    dc.last_param = (int)h->params.size() - 1;
}

void build_tables(cad_unet* h) {
    const int f = h->f;
    // enc1.conv1 runs on 8 internal input channels (zero-padded weights and input): the pre-split
    // kernels' 16-B pieces, so its forward and weight gradient read bf16 twins like the rest
    if (h->model == CAD_MODEL_RAY_FILM)   // RayEnhancedConv(3, f, 4, true): conv1 sees rgb + rays
        add_double_conv(h, h->enc[0], "enc1.", h->in_ch + 3, 8, f, 0);
    else
        add_double_conv(h, h->enc[0], "enc1.", h->in_ch, 8, f, 0);
    h->enc[0].y1_f32 = h->model != CAD_MODEL_RAY_FILM;
    const char* enames[4] = {"enc2", "enc3", "enc4", "bottleneck"};
    for (int i = 0; i < 4; ++i)
        add_double_conv(h, h->enc[i + 1], std::string(enames[i]) + ".conv.", f << i, f << i, f << (i + 1), i + 1);
    for (int k = 0; k < 4; ++k) {   // dec4 .. dec1
        const int l = 3 - k;        // decoder level
        const int cin = f << (l + 1), cout = f << l;
        const std::string pre = "dec" + std::to_string(l + 1) + ".";
        add_param(h, pre + "up.weight", {cin, cout, 2, 2}, P_CONVT_W);
        add_param(h, pre + "up.bias", {cout}, P_CONVT_B);
        h->up[l] = Up{(int)h->params.size() - 2, (int)h->params.size() - 1, cin, cout, nullptr};
        add_double_conv(h, h->dec[l], pre + "conv.", cin, cin, cout, l);
        h->dec[l].first_param = h->up[l].widx;
    }
    add_param(h, "out_conv.weight", {1, f, 1, 1}, P_HEAD_W);
    add_param(h, "out_conv.bias", {1}, P_HEAD_B);
    h->head_w = (int)h->params.size() - 2;
    h->head_b = (int)h->params.size() - 1;
    h->n_flat = (h->n_flat + 63) & ~int64_t(63);
}

void bn_alloc(Arena& a, BN& b) {
    b.rm = a.f(b.C); b.rv = a.f(b.C);
    b.mean = a.f(b.C); b.invstd = a.f(b.C); b.scale = a.f(b.C); b.shift = a.f(b.C); b.coef = a.f(3 * b.C);
}

void film_alloc(Arena& a, DoubleConv& dc, int B) {
    if (!dc.has_film()) return;
    Film& F = dc.film;
    const int H1 = cad::kFilmH1, H2 = cad::kFilmH2, C = dc.c1.cout;
    F.rm1 = a.f(H1); F.rv1 = a.f(H1); F.rm2 = a.f(H2); F.rv2 = a.f(H2);
    F.xh1 = a.f((int64_t)B * H1); F.h1 = a.f((int64_t)B * H1); F.dh1 = a.f((int64_t)B * H1);
    F.xh2 = a.f((int64_t)B * H2); F.h2 = a.f((int64_t)B * H2); F.dh2 = a.f((int64_t)B * H2);
    F.is1 = a.f(H1); F.is2 = a.f(H2);
    F.gam = a.f((int64_t)B * C); F.bet = a.f((int64_t)B * C);
    F.dgam = a.f((int64_t)B * C); F.dbet = a.f((int64_t)B * C);
}

void layout(cad_unet* h, Arena& a) {
    const int B = h->Bmax;
    const bool film = h->model != CAD_MODEL_BASELINE;
    // pre-split (bf16) twin of `elems` fp32 values
    auto sp = [&](int64_t elems) -> void* { return a.take((size_t)elems * 2 * cad::kMaxPlanes); };
    auto conv_split_alloc = [&](Conv& c, bool dgrad) {
        if (c.cin % 8) return;   // (every conv of this family has cin % 8 == 0)
        const int64_t n = (int64_t)c.cout * 9 * c.cin;
        c.ws = sp(n);
        if (dgrad) c.wds = sp(n);
    };
    h->flat_p = a.f(h->n_flat);
    h->flat_g = a.f(h->n_flat);
    h->norm_coef = a.f(4);
    h->camn = a.f((int64_t)B * 4);
    for (int l = 0; l < 5; ++l) {
        DoubleConv& e = h->enc[l];
        bn_alloc(a, e.b1); bn_alloc(a, e.b2);
        const int64_t MC = h->Ml(l, B) * h->Cl(l);
        e.y1 = a.f(MC); e.y2 = a.f(MC);
        e.a1 = a.f(MC);   // relu(bn1(y1)) (FiLM'd) feeding conv2
        e.a1s = sp(MC);
        film_alloc(a, e, B);
        if (l > 0) e.c1.wd = a.f((int64_t)e.c1.cout * 9 * e.c1.cin);
        e.c2.wd = a.f((int64_t)e.c2.cout * 9 * e.c2.cin);
        conv_split_alloc(e.c1, l > 0);
        conv_split_alloc(e.c2, true);
        if (l < 4) { h->cat[l] = a.f(2 * MC); h->cats[l] = sp(2 * MC); }
        if (l > 0) {
            h->pool[l] = a.f(h->Ml(l, B) * h->Cl(l - 1));
            h->pools[l] = sp(h->Ml(l, B) * h->Cl(l - 1));
            h->pidx[l] = a.u8(h->Ml(l, B) * h->Cl(l - 1));
        }
    }
    h->a2_bott = a.f(h->Ml(4, B) * h->Cl(4));
    h->botts = sp(h->Ml(4, B) * h->Cl(4));
    for (int l = 0; l < 4; ++l) {
        DoubleConv& d = h->dec[l];
        bn_alloc(a, d.b1); bn_alloc(a, d.b2);
        const int64_t MC = h->Ml(l, B) * h->Cl(l);
        d.y1 = a.f(MC); d.y2 = a.f(MC);
        d.a1 = a.f(MC);
        d.a1s = sp(MC);
        film_alloc(a, d, B);
        h->dout[l] = a.f(MC);
        if (l > 0) h->douts[l] = sp(MC);
        d.c1.wd = a.f((int64_t)d.c1.cout * 9 * d.c1.cin);
        d.c2.wd = a.f((int64_t)d.c2.cout * 9 * d.c2.cin);
        conv_split_alloc(d.c1, true);
        conv_split_alloc(d.c2, true);
        h->up[l].wf = a.f((int64_t)4 * h->up[l].cout * h->up[l].cin);
        h->up[l].wfs = sp((int64_t)4 * h->up[l].cout * h->up[l].cin);
        h->up[l].wms = sp((int64_t)4 * h->up[l].cout * h->up[l].cin);
        h->dcat[l] = a.f(2 * MC);
        h->dcats[l] = sp(MC);
        h->dskips[l] = sp(MC);
    }
    h->x0 = a.f(h->Ml(0, B) * h->x0_ld);
    if (h->x0_ld % 8 == 0) h->x0s = sp(h->Ml(0, B) * h->x0_ld);
    h->dYs = sp(h->Ml(0, B) * h->Cl(0));
    h->sig = a.f(h->Ml(0, B));
    const int64_t M0C0 = h->Ml(0, B) * h->Cl(0);
    h->Sa = a.f(M0C0);
    h->Sb = a.f(M0C0);
    h->Sb2 = a.f(M0C0);
    h->dYs2 = sp(h->Ml(0, B) * h->Cl(0));
    h->Sc = a.f(h->Ml(1, B) * h->Cl(0));
    // BN tile partials: rows x (2C + 1) (S, M2 per channel + the row's count), max over layers
    int64_t st = 0, colmax = 0;
    for (int l = 0; l < 5; ++l) {
        const int64_t r = (h->Ml(l, B) + 63) / 64;   // any tile height: the engine may change at run time
        st = std::max<int64_t>(st, r * (2 * h->Cl(l) + 1));
        colmax = std::max<int64_t>(colmax, h->Cl(l));
    }
    h->stats = a.f(st);
    int64_t dscr = (int64_t)(cad::colsum_slices(h->Ml(0, B)) + 2) * 4 * colmax + 4 * colmax + 8192;
    for (int l = 0; l < 5 && film; ++l)
        dscr = std::max(dscr, cad::film_reduce_doubles(B, (int64_t)h->Hl(l) * h->Wl(l), h->Cl(l)) + 8192);
    h->dscr = a.d(dscr);
    h->dscr2 = a.d(dscr);
    // wgrad split-K slab: enough for the largest-benefit layers, capped at 64M floats (256 MB)
    int64_t sl = 0;
    for (int l = 0; l < 5; ++l) {
        const int64_t Kp = h->Ml(l, B);
        sl = std::max(sl, cad::wgrad_slab_floats(h->Cl(l), 9 * h->Cl(l) * 2, (int)std::min<int64_t>(Kp, INT32_MAX)));
    }
    h->slab_cap = std::min<int64_t>(sl, (int64_t)64 << 20);
    h->slab = a.f(h->slab_cap);
    // bn1's per-tile backward sums: tiles of at least 64 rows
    h->part_cap = (h->Ml(0, B) + 63) / 64 * 2 * h->Cl(0);
    h->rc_part = a.d(h->part_cap);
    // buffers table (running stats), named_buffers() order (parameter order of the BNs)
    h->bufs.clear();
    auto add_bn_bufs = [&](const std::string& pre, BN& b) {
        h->bufs.push_back({pre + ".running_mean", b.C, b.rm});
        h->bufs.push_back({pre + ".running_var", b.C, b.rv});
    };
    auto add_block = [&](const std::string& pre, DoubleConv& dc) {
        add_bn_bufs(pre + "bn1", dc.b1);
        add_bn_bufs(pre + "bn2", dc.b2);
        if (!dc.has_film()) return;
        h->bufs.push_back({pre + "film.bn1.running_mean", cad::kFilmH1, dc.film.rm1});
        h->bufs.push_back({pre + "film.bn1.running_var", cad::kFilmH1, dc.film.rv1});
        h->bufs.push_back({pre + "film.bn2.running_mean", cad::kFilmH2, dc.film.rm2});
        h->bufs.push_back({pre + "film.bn2.running_var", cad::kFilmH2, dc.film.rv2});
    };
    const char* en[5] = {"enc1.", "enc2.conv.", "enc3.conv.", "enc4.conv.", "bottleneck.conv."};
    for (int l = 0; l < 5; ++l) add_block(en[l], h->enc[l]);
    for (int k = 0; k < 4; ++k) {
        const int l = 3 - k;
        add_block("dec" + std::to_string(l + 1) + ".conv.", h->dec[l]);
    }
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// the FilmLayer view of a block (pointers into the current slabs: rebuilt per use because the slabs
// can move, cad_unet_use_external_slabs)
cad::FilmLayer film_view(const cad_unet* h, const DoubleConv& dc) {
    const Film& F = dc.film;
    const int i = F.p0;
    cad::FilmLayer L;
    L.C = dc.c1.cout;
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

// pre-split operands (gemm_ps.hpp) are used when the engine splits (S3 / B1) and the operand's
// channel count is a multiple of 8; the fp32 tensors are still written (BN, pooling, the head and
// the loss read them), the split twin is written right after by split_rows
cad::Split sv(const void* p, int64_t ld, int coff = 0) {
    cad::Split v;
    v.p = p; v.ld = ld; v.coff = coff;
    return v;
}
void split_into(const float* x, int64_t ldx, int xcoff, int C, int64_t M, void* out, int64_t ldo, int ocoff,
                hipStream_t st) {
    if (out) cad::split_rows(x, ldx, xcoff, C, M, out, ldo, ocoff, st);
}
void wprep_add(cad::WPrepList& L, int kind, const float* src, float* d32, void* d16, int cout, int cin, int64_t n) {
    if (!d32 && !d16) return;
    if (L.njobs == cad::kWPrepMaxJobs) throw std::runtime_error("weight_prep: job list full");
    cad::WPrepJob& j = L.job[L.njobs++];
    j.src = src; j.d32 = d32; j.d16 = d16; j.kind = kind; j.cout = cout; j.cin = cin; j.n = n;
}
// forward weights, every forward (they change per step), in one launch: the ConvT forward repack
// [q][co][ci] (rows 4*cout, K = cin) and, with pre-split operands, the bf16 twins of the conv weights
// and of that repack
void prep_fwd_weights(const cad_unet* h, bool ps, hipStream_t st) {
    cad::WPrepList L{};
    for (int l = 0; l < 4; ++l) {
        const Up& u = h->up[l];
        wprep_add(L, cad::WPREP_CONVT, h->P(u.widx), u.wf, ps ? u.wfs : nullptr, u.cout, u.cin, (int64_t)4 * u.cout * u.cin);
    }
    if (ps) {
        auto sw = [&](const Conv& c) {
            if (c.ws) wprep_add(L, cad::WPREP_SPLIT, h->P(c.pidx), nullptr, c.ws, c.cout, c.cin, (int64_t)c.cout * 9 * c.cin);
        };
        for (int l = 0; l < 5; ++l) { sw(h->enc[l].c1); sw(h->enc[l].c2); }
        for (int l = 0; l < 4; ++l) { sw(h->dec[l].c1); sw(h->dec[l].c2); }
    }
    cad::weight_prep(L, st);
}

// in_s / out_s: split twins of the block input / output (p == nullptr: none)
// out_f32 = false: with pre-split GEMMs downstream only the output's twin is read (decoder outputs
// above level 0, the bottleneck), so the fp32 output is not written
// A/B switches read once per process: CAD_ENC1PS=0 runs enc1.conv1 on the in-loader kernel (fp32
// input, fp32 dY), CAD_ENC1BF16=1 stores its output as bf16 like the other convolutions
int env_flag(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e && e[0] ? std::atoi(e) : dflt;
}
// conv1 of a block runs on the pre-split twins (its input twin and weight twin exist)
bool conv1_presplit(cad_unet* h, const DoubleConv& dc, bool ps, const cad::Split& in_s) {
    static const bool enc1_ps = env_flag("CAD_ENC1PS", 1) != 0;
    return ps && in_s.p && dc.c1.ws && (enc1_ps || &dc != &h->enc[0]);
}
// the next level's max-pool written by an encoder block's bn2 pass (bn_relu_pool_fwd)
struct PoolOut {
    float* pool;      // fp32 pooled output (nullptr: only its twin is read)
    uint8_t* idx;     // argmax codes
    void* pool_s;     // pooled twin (bf16 engine)
};
// CAD_BNPOOL=0: the encoder bn2 apply and the max-pool as separate passes (A/B measurements;
// bit-identical, tests/test_gpu_headfuse.py)
bool bn_pool_on() {
    static const bool on = env_flag("CAD_BNPOOL", 1) != 0;
    return on;
}

// head_pred != nullptr: the block's bn2 + ReLU feeds the depth head directly (level-0 fusion): sig
// and head_pred are written, out is not.  pool != nullptr: the block's bn2 pass also writes the next
// level's max-pool
void double_conv_fwd(cad_unet* h, DoubleConv& dc, const float* in, int64_t ldin, cad::Split in_s, int B, float* out,
                     int64_t ldo, int ocoff, cad::Split out_s, hipStream_t st, bool out_f32 = true,
                     float* head_pred = nullptr, const PoolOut* pool = nullptr) {
    const int l = dc.level, Hh = h->Hl(l), Ww = h->Wl(l), C = dc.c1.cout;
    const int64_t M = h->Ml(l, B);
    const bool tr = h->train;
    const bool ps = h->fwd_np > 0;
    auto bn = [&](BN& b, int cin, bool ps_conv) {
        const int rows = cad::conv3x3_stats_rows(cin, B, Hh, Ww, C, ps_conv);
        if (tr)
            cad::bn_fwd_finalize(h->stats, rows, C, M, h->P(b.widx), h->P(b.bidx), b.rm, b.rv, 0.1f, 1e-5f, h->dscr,
                                 b.mean, b.invstd, b.scale, b.shift, st);
        else
            cad::bn_eval_coeffs(h->P(b.widx), h->P(b.bidx), b.rm, b.rv, C, 1e-5f, b.mean, b.invstd, b.scale, b.shift, st);
    };
    float* stats = tr ? h->stats : nullptr;
    const bool ps1 = conv1_presplit(h, dc, ps, in_s);
    // the pre-split (bf16 engine) convolutions store their pre-BN outputs as bf16 (BN statistics are
    // those of the stored values); BN apply / backward and FiLM read them as such
    static const bool enc1_bf16 = env_flag("CAD_ENC1BF16", 0) != 0;
    dc.y1b = ps1 && (!dc.y1_f32 || enc1_bf16);
    dc.y2b = ps;
    if (ps1) {
        cad::conv3x3_fwd_ps(in_s, dc.c1.cin, sv(dc.c1.ws, 9 * dc.c1.cin), C, dc.y1, C, 0, B, Hh, Ww, stats, st, dc.y1b);
    } else {
        cad::conv3x3_fwd(in, ldin, 0, dc.c1.cin, h->P(dc.c1.pidx), C, dc.y1, C, 0, B, Hh, Ww, stats, st);
    }
    bn(dc.b1, dc.c1.cin, ps1);
    if (dc.has_film()) {   // FiLMDoubleConvImpl::forward (intrinsics_unet.h:38-52)
        // pre-split GEMMs read only a1's twin (written by the same pass): the fp32 a1 is not written
        cad::film_apply(dc.y1, C, dc.b1.scale, dc.b1.shift, dc.film.gam, dc.film.bet, B, (int64_t)Hh * Ww,
                        ps ? nullptr : dc.a1, st, dc.y1b, ps ? dc.a1s : nullptr);
    } else {
        // pre-split GEMMs read only a1's twin (conv2 and its weight gradient): the fp32 a1 is not written
        cad::bn_relu_fwd(dc.y1, C, dc.b1.scale, dc.b1.shift, ps ? nullptr : dc.a1, C, 0, M, st, ps ? dc.a1s : nullptr,
                         C, 0, dc.y1b);
    }
    if (ps)
        cad::conv3x3_fwd_ps(sv(dc.a1s, C), C, sv(dc.c2.ws, 9 * C), C, dc.y2, C, 0, B, Hh, Ww, stats, st, true);
    else
        cad::conv3x3_fwd(dc.a1, C, 0, C, h->P(dc.c2.pidx), C, dc.y2, C, 0, B, Hh, Ww, stats, st);
    bn(dc.b2, C, ps);
    if (head_pred) {
        cad::bn_relu_head_fwd(dc.y2, C, dc.b2.scale, dc.b2.shift, h->P(h->head_w), h->P(h->head_b), h->max_depth, h->sig,
                              head_pred, M, st, dc.y2b);
        return;
    }
    const bool twin = ps && out_s.p;
    if (pool) {
        if (ocoff != 0 || (twin && out_s.coff != 0)) throw std::runtime_error("bn_relu_pool_fwd: offset outputs");
        cad::bn_relu_pool_fwd(dc.y2, C, dc.b2.scale, dc.b2.shift, (out_f32 || !twin) ? out : nullptr, ldo,
                              twin ? const_cast<void*>(out_s.p) : nullptr, out_s.ld, B, Hh, Ww, dc.y2b, pool->pool,
                              pool->idx, pool->pool_s, st);
        return;
    }
    cad::bn_relu_fwd(dc.y2, C, dc.b2.scale, dc.b2.shift, (out_f32 || !twin) ? out : nullptr, ldo, ocoff, M, st,
                     twin ? const_cast<void*>(out_s.p) : nullptr, out_s.ld, out_s.coff, dc.y2b);
}

// CAD_DCATSPLIT=0: the decoder conv1 dgrad writes all of dcat in fp32 and the up half's twin is split
// from it (A/B measurements; bit-identical)
bool dcat_split_on() {
    static const bool on = env_flag("CAD_DCATSPLIT", 1) != 0;
    return on;
}

// CAD_POOLFOLD=0 keeps the max-pool backward scatter (A/B measurements; bit-identical)
bool pool_fold_on() {
    static const bool on = env_flag("CAD_POOLFOLD", 1) != 0;
    return on;
}

// CAD_HEADFUSE=0 keeps the unfused level-0 passes (A/B measurements)
bool head_fusion_on() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_HEADFUSE");
        return !(e && e[0] == '0');
    }();
    return on;
}

void unet_forward(cad_unet* h, const float* rgb, const float* cam4, float* depth, int B, hipStream_t st) {
    const int f = h->f;
    // Pre-split operands on the bf16 engine (measured on MI355X at bs32 480x640: B1 198 -> 277
    // img/s); every block's channel count (f * 2^l) must be a multiple of 8.  The S3 engine splits in
    // its loaders (pre-split S3 operands are 6 bytes per element: measured 112 -> 101 img/s).
    h->fwd_np = h->f % 8 ? 0 : cad::split_planes();
    const bool ps = h->fwd_np > 0;
    prep_fwd_weights(h, ps, st);
    if (h->model != CAD_MODEL_BASELINE) {
        // a14 normalisation, then every block's FiLM MLP (gamma/beta depend on the camera only)
        cad::camera_normalize(cam4, B, h->H, h->W, h->camn, st);
        cad::FilmList fl;   // (one launch per MLP step for all nine layers)
        for (int l = 0; l < 5; ++l) fl.l[fl.n++] = film_view(h, h->enc[l]);
        for (int l = 3; l >= 0; --l) fl.l[fl.n++] = film_view(h, h->dec[l]);
        cad::film_mlp_fwd_all(fl, h->camn, B, h->train, st);
    }
    if (h->model == CAD_MODEL_RAY_FILM)
        cad::rgb_rays_to_nhwc8(rgb, cam4, B, h->H, h->W, h->x0, st);
    else
        cad::rgb_to_nhwc8(rgb, h->x0, B, h->H, h->W, st);
    const cad::Split none{};
    cad::Split x0s = none;
    if (ps && h->x0s) {
        cad::split_rows(h->x0, h->x0_ld, 0, h->x0_ld, h->Ml(0, B), h->x0s, h->x0_ld, 0, st);
        x0s = sv(h->x0s, h->x0_ld);
    }
    // on the bf16 engine the encoder outputs are written only as the concat twin: the max-pool reads
    // it (the decoder conv1 and its gradients read it anyway).  By default each encoder block's bn2 pass
    // writes the next level's max-pool as well (bn_relu_pool_fwd)
    auto pool_of = [&](int l) {   // the max-pool into level l; pre-split GEMMs read only the pooled twin
        const bool ptwin = ps && h->pools[l];
        return PoolOut{ptwin ? nullptr : h->pool[l], h->pidx[l], ptwin ? h->pools[l] : nullptr};
    };
    const bool fuse_pool = bn_pool_on();
    PoolOut po = pool_of(1);
    double_conv_fwd(h, h->enc[0], h->x0, h->x0_ld, x0s, B, h->cat[0], 2 * f, 0, sv(h->cats[0], 2 * f), st, !ps, nullptr,
                    fuse_pool ? &po : nullptr);
    for (int l = 1; l <= 4; ++l) {
        const int Cp = h->Cl(l - 1);
        if (!fuse_pool) {
            const PoolOut p = pool_of(l);
            cad::maxpool_fwd(ps ? static_cast<const float*>(h->cats[l - 1]) : h->cat[l - 1], 2 * Cp, Cp, B, h->Hl(l - 1),
                             h->Wl(l - 1), p.pool, p.idx, st, p.pool_s, ps);
        }
        const cad::Split pin = sv(h->pools[l], Cp);
        if (l < 4) {
            po = pool_of(l + 1);
            double_conv_fwd(h, h->enc[l], h->pool[l], Cp, pin, B, h->cat[l], 2 * h->Cl(l), 0,
                            sv(h->cats[l], 2 * h->Cl(l)), st, !ps, nullptr, fuse_pool ? &po : nullptr);
        } else {
            double_conv_fwd(h, h->enc[4], h->pool[4], Cp, pin, B, h->a2_bott, h->Cl(4), 0, sv(h->botts, h->Cl(4)), st,
                            false);
        }
    }
    h->head_fused = head_fusion_on() && cad::head_fusable(f);
    for (int l = 3; l >= 0; --l) {
        const float* upin = l == 3 ? h->a2_bott : h->dout[l + 1];
        const void* upins = l == 3 ? h->botts : h->douts[l + 1];
        const Up& u = h->up[l];
        const int C = h->Cl(l);
        if (ps) {   // the up half goes straight into the concat twin (its fp32 copy has no reader)
            cad::convT_fwd_ps(sv(upins, u.cin), u.cin, sv(u.wfs, u.cin), h->P(u.bidx), u.cout,
                              static_cast<float*>(h->cats[l]), 2 * C, C, B, h->Hl(l + 1), h->Wl(l + 1), st, true);
        } else {
            cad::convT_fwd(upin, u.cin, u.cin, u.wf, h->P(u.bidx), u.cout, h->cat[l], 2 * C, C, B, h->Hl(l + 1),
                           h->Wl(l + 1), st);
        }
        double_conv_fwd(h, h->dec[l], h->cat[l], 2 * C, sv(h->cats[l], 2 * C), B, h->dout[l], C, 0,
                        l > 0 ? sv(h->douts[l], C) : none, st, l == 0, l == 0 && h->head_fused ? depth : nullptr);
    }
    if (!h->head_fused)
        cad::head_fwd(h->dout[0], f, h->P(h->head_w), h->P(h->head_b), h->max_depth, h->sig, depth, h->Ml(0, B), st);
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// g: grad wrt the DoubleConv output (ld ldg, channel offset gcoff); in: the block input (ld ldin,
// cin channels; in_s its split twin); din: where conv1's dgrad goes (nullptr = not needed), ld lddin.
// head != nullptr (level-0 fusion): g is null and bn2's upstream gradient is the head's, rebuilt per row.
// fork: the side stream continues after everything issued on st so far
void side_fork(cad_unet* h, hipStream_t st) {
    HIPCHK(hipEventRecord(h->ev_fork, st));
    HIPCHK(hipStreamWaitEvent(h->side, h->ev_fork, 0));
}
// join: st continues after everything issued on the side stream so far
void side_join(cad_unet* h, hipStream_t st) {
    HIPCHK(hipEventRecord(h->ev_tail, h->side));
    HIPCHK(hipStreamWaitEvent(st, h->ev_tail, 0));
}
// the stream the weight gradients run on: the side stream on the S3 engine (configs[1] -1.9 %); on the
// bf16 engine they stay on the step's stream — there the GEMMs beside each other measured neutral to
// +0.7 % (profiles/r06_lab/README.md).  CAD_SIDE_WGRAD=1 / 0 forces either; read per call, so bench.py's
// untimed census step can time every GEMM alone (a kernel beside another one takes longer per launch)
hipStream_t wgrad_stream(cad_unet* h, bool ps, hipStream_t st) {
    const int f = env_flag("CAD_SIDE_WGRAD", -1);
    const bool side = f < 0 ? !ps : f != 0;
    if (!side) return st;
    side_fork(h, st);
    return h->side;
}

void double_conv_bwd(cad_unet* h, DoubleConv& dc, const float* g, int64_t ldg, int gcoff, const float* in,
                     int64_t ldin, cad::Split in_s, int B, float* din, int64_t lddin, hipStream_t st,
                     const cad::HeadGrad* head = nullptr, const cad::PoolAdd* pool = nullptr, void* din_hi = nullptr,
                     bool* din_hi_done = nullptr, bool g_bf16 = false, bool din_bf16 = false) {
    const int l = dc.level, Hh = h->Hl(l), Ww = h->Wl(l), C = dc.c1.cout;
    const int64_t M = h->Ml(l, B);
    const bool ps = h->fwd_np > 0 && h->fwd_np == cad::split_planes();
    hipStream_t sd = h->side;
    // bn2's dL/dz in (Sb, dYs), bn1's in (Sb2, dYs2): the weight gradients on the side stream read them
    // while this stream goes on
    float* dY = h->Sb;
    void* dYs = h->dYs;
    float* dY1 = h->Sb2;
    void* dYs1 = h->dYs2;
    // conv2's input gradient; the bf16 engine stores it as bf16 (read by FiLM's and bn1's backward)
    float* dA1 = h->Sa;
    // bn2 + relu
    // with pre-split GEMMs both consumers of dY2 read its twin: the fp32 dY2 is not written
    HIPCHK(hipStreamWaitEvent(st, h->evA, 0));   // the previous block's conv2 weight gradient has read them
    cad::bn_relu_bwd(g, ldg, gcoff, dc.y2, C, dc.b2.mean, dc.b2.invstd, dc.b2.scale, dc.b2.shift, h->P(dc.b2.widx), M,
                     h->dscr, dc.b2.coef, h->G(dc.b2.widx), h->G(dc.b2.bidx), ps ? nullptr : dY, st, nullptr, 1,
                     ps ? dYs : nullptr, true, dc.y2b, head, g_bf16, pool);
    // conv2: wgrad, dgrad.  On the S3 engine (plain blocks) the dgrad's window epilogue also forms
    // bn1's backward sums over the dL/da1 it stores (conv3x3_dgrad_bnsums), so bn1's backward skips its
    // column-reduction pass over (dL/da1, y1); CAD_BNSUMS=0 keeps that pass (A/B; the same fp64 sums in
    // another order, tests/test_gpu_headfuse.py).  (Measured slower on the bf16 engine: conv_kernels.hip)
    static const bool bnsums = env_flag("CAD_BNSUMS", 1) != 0;
    int bn1_tiles = 0;
    cad::BnSums bs;
    if (bnsums && !ps && !dc.has_film() && h->rc_part) {
        bs.y = dc.y1; bs.ldy = C; bs.y_bf16 = dc.y1b;
        bs.mean = dc.b1.mean; bs.invstd = dc.b1.invstd; bs.scale = dc.b1.scale; bs.shift = dc.b1.shift;
        bs.part = h->rc_part; bs.part_cap = h->part_cap;
    }
    hipStream_t wg = wgrad_stream(h, ps, st);
    if (ps) {
        cad::conv3x3_wgrad_ps(sv(dYs, C), C, sv(dc.a1s, C), C, h->G(dc.c2.pidx), B, Hh, Ww, h->slab, h->slab_cap, wg);
        HIPCHK(hipEventRecord(h->evA, wg));
        cad::conv3x3_dgrad_ps(sv(dYs, C), C, sv(dc.c2.wds, 9 * C), C, dA1, C, B, Hh, Ww, st, true);
    } else {
        cad::conv3x3_wgrad(dY, C, dc.a1, C, 0, C, h->G(dc.c2.pidx), B, Hh, Ww, h->slab, h->slab_cap, wg);
        HIPCHK(hipEventRecord(h->evA, wg));
        if (bs.part) bn1_tiles = cad::conv3x3_dgrad_bnsums(dY, C, dc.c2.wd, C, dA1, C, B, Hh, Ww, bs, st);
        if (!bn1_tiles) cad::conv3x3_dgrad(dY, C, dc.c2.wd, C, dA1, C, B, Hh, Ww, st);
    }
    // FiLM: dgamma/dbeta per (sample, channel); the ReLU sees dA1 * gamma (folded into bn_relu_bwd).  By
    // default the FiLM sums come from bn1's backward reduction pass over the same (dA1, y1) (round 4;
    // CAD_FILMFUSE=0: the separate film_affine_bwd pass)
    const int64_t HW = (int64_t)Hh * Ww;
    static const bool film_fuse = env_flag("CAD_FILMFUSE", 1) != 0;
    const bool film_sep = dc.has_film() && !film_fuse;
    if (film_sep)
        cad::film_affine_bwd(dA1, dc.y1, C, dc.b1.scale, dc.b1.shift, B, HW, h->dscr, dc.film.dgam, dc.film.dbet, st,
                             dc.y1b, ps);
    // bn1 + relu; the fp32 dY1 only when a conv1 GEMM below reads it (enc1's 4-channel input keeps the
    // in-loader weight gradient)
    const bool ps1 = conv1_presplit(h, dc, ps, in_s);
    const bool dy1_f32 = !ps1 || (din && !(ps && dc.c1.wds));
    HIPCHK(hipStreamWaitEvent(st, h->evB, 0));   // the previous block's conv1 weight gradient has read them
    {
        const bool ff = dc.has_film() && !film_sep;
        cad::bn_relu_bwd(dA1, C, 0, dc.y1, C, dc.b1.mean, dc.b1.invstd, dc.b1.scale, dc.b1.shift, h->P(dc.b1.widx), M,
                         h->dscr, dc.b1.coef, h->G(dc.b1.widx), h->G(dc.b1.bidx), dy1_f32 ? dY1 : nullptr, st,
                         dc.has_film() ? dc.film.gam : nullptr, HW, ps ? dYs1 : nullptr, true, dc.y1b, nullptr, ps,
                         nullptr, ff ? dc.film.dgam : nullptr, ff ? dc.film.dbet : nullptr,
                         bn1_tiles ? h->rc_part : nullptr, bn1_tiles);
    }
    // side: the FiLM MLP backward (needs this bn1's dgamma / dbeta: ~1.2 ms/step of small latency-bound
    // kernels beside the block's GEMMs), then conv1's weight gradient on wgrad_stream's choice
    if (dc.has_film()) {
        side_fork(h, st);
        cad::film_mlp_bwd(film_view(h, dc), h->camn, B, sd);
    }
    hipStream_t wg1 = wgrad_stream(h, ps, st);
    if (ps1)
        cad::conv3x3_wgrad_ps(sv(dYs1, C), C, in_s, dc.c1.cin, h->G(dc.c1.pidx), B, Hh, Ww, h->slab, h->slab_cap, wg1);
    else
        cad::conv3x3_wgrad(dY1, C, in, ldin, 0, dc.c1.cin, h->G(dc.c1.pidx), B, Hh, Ww, h->slab, h->slab_cap, wg1);
    HIPCHK(hipEventRecord(h->evB, wg1));
    // conv1 dgrad
    if (din) {
        // din_hi: the upper half of din's columns goes straight into that bf16 twin (decoder concat)
        if (ps && dc.c1.wds) {
            const bool done = cad::conv3x3_dgrad_ps(sv(dYs1, C), C, sv(dc.c1.wds, 9 * C), dc.c1.cin, din, lddin, B, Hh,
                                                    Ww, st, din_bf16, din_hi, dc.c1.cin / 2, dc.c1.cin / 2);
            if (din_hi_done) *din_hi_done = done && din_hi;
        } else
            cad::conv3x3_dgrad(dY1, C, dc.c1.wd, dc.c1.cin, din, lddin, B, Hh, Ww, st);
    }
}

void repack_dgrad_weights(cad_unet* h, hipStream_t st) {   // one launch (prep_fwd_weights)
    const bool ps = h->fwd_np > 0 && h->fwd_np == cad::split_planes();
    cad::WPrepList L{};
    auto rp = [&](Conv& c) {   // dgrad repack [ci][tap][co]: rows cin, K = 9*cout
        wprep_add(L, cad::WPREP_DGRAD, h->P(c.pidx), c.wd, ps ? c.wds : nullptr, c.cout, c.cin, (int64_t)c.cout * 9 * c.cin);
    };
    for (int l = 0; l < 5; ++l) {
        if (l > 0) rp(h->enc[l].c1);
        rp(h->enc[l].c2);
    }
    for (int l = 0; l < 4; ++l) {
        rp(h->dec[l].c1);
        rp(h->dec[l].c2);
        const Up& u = h->up[l];   // ConvT weights [ci][q][co]: rows cin, K = 4*cout
        if (ps) wprep_add(L, cad::WPREP_SPLIT, h->P(u.widx), nullptr, u.wms, u.cout, u.cin, (int64_t)4 * u.cout * u.cin);
    }
    cad::weight_prep(L, st);
}

// stages: 0 head, 1..4 dec1..dec4, 5 bottleneck, 6..9 enc4..enc1
constexpr int kStages = 10;

void backward_stage_body(cad_unet* h, int stage, const float* dpred, hipStream_t st);
void backward_stage(cad_unet* h, int stage, const float* dpred, hipStream_t st) {
    backward_stage_body(h, stage, dpred, st);
    if (!h->defer_join) side_join(h, st);   // the stage's gradients complete on st
}
void backward_stage_body(cad_unet* h, int stage, const float* dpred, hipStream_t st) {
    const int B = h->fwd_B;
    const int f = h->f;
    const bool ps = h->fwd_np > 0 && h->fwd_np == cad::split_planes();
    if (stage == 0) {
        // the buffer-pair events start on this stream (so a captured step never waits on a prior step)
        HIPCHK(hipEventRecord(h->evA, st));
        HIPCHK(hipEventRecord(h->evB, st));
        repack_dgrad_weights(h, st);
        if (h->head_fused) {   // head weight / bias gradient from dec1's bn2 input; its input gradient: stage 1
            const DoubleConv& d = h->dec[0];
            cad::head_bwd_y(d.y2, f, d.b2.scale, d.b2.shift, dpred, h->sig, h->max_depth, h->Ml(0, B), h->dscr,
                            h->G(h->head_w), h->G(h->head_b), st, d.y2b);
        } else {
            cad::head_bwd(h->dout[0], f, h->P(h->head_w), dpred, h->sig, h->max_depth, h->Sa, h->Ml(0, B), h->dscr,
                          h->G(h->head_w), h->G(h->head_b), st);
        }
        return;
    }
    if (stage <= 4) {   // decoder level l = stage-1; grad of its output is in Sa
        const int l = stage - 1;
        const int C = h->Cl(l);
        const cad::HeadGrad hg{dpred, h->sig, h->P(h->head_w), h->max_depth};
        const bool hf = l == 0 && h->head_fused;
        // the bf16 engine keeps dcat as two bf16 halves: the skip half (dskips, the encoder bn2 gradient)
        // and the up half (dcats, the ConvT GEMMs' operand).  The conv1 dgrad writes both straight from
        // its window kernel when the shape allows (split store); otherwise it writes dcat in fp32 and the
        // halves are split from it (same rounding)
        const bool split = ps && dcat_split_on() &&
                           cad::conv3x3_dgrad_split_ok(sv(h->dYs, C), C, sv(h->dec[l].c1.wds, 9 * C), 2 * C, h->Wl(l), C);
        bool up_twin = false;
        // above level 0 the block-output gradient in Sa comes from the ConvT dgrad: bf16 on the bf16 engine
        double_conv_bwd(h, h->dec[l], hf ? nullptr : h->Sa, C, 0, h->cat[l], 2 * C, sv(h->cats[l], 2 * C), B,
                        split ? static_cast<float*>(h->dskips[l]) : h->dcat[l], split ? C : 2 * C, st,
                        hf ? &hg : nullptr, nullptr, split ? h->dcats[l] : nullptr, &up_twin, ps && l > 0, split);
        if (split != up_twin) throw std::runtime_error("decoder dgrad split store not taken");
        const Up& u = h->up[l];
        const float* upin = l == 3 ? h->a2_bott : h->dout[l + 1];
        const void* upins = l == 3 ? h->botts : h->douts[l + 1];
        // up (ConvTranspose2d) backward: grad of its output = dcat[:, C:2C]
        if (ps && !split) {
            cad::split_rows(h->dcat[l], 2 * C, C, C, h->Ml(l, B), h->dcats[l], C, 0, st);
            cad::split_rows(h->dcat[l], 2 * C, 0, C, h->Ml(l, B), h->dskips[l], C, 0, st);
        }
        // the ConvT's weight and bias gradients on the side stream (its own column-sum scratch)
        hipStream_t sd = wgrad_stream(h, ps, st);
        if (ps) {
            cad::convT_wgrad_ps(sv(upins, u.cin), u.cin, sv(h->dcats[l], C), u.cout, h->G(u.widx), B, h->Hl(l + 1),
                                h->Wl(l + 1), h->slab, h->slab_cap, sd);
        } else {
            cad::convT_wgrad(upin, u.cin, h->dcat[l], 2 * C, C, u.cout, h->G(u.widx), B, h->Hl(l + 1), h->Wl(l + 1),
                             h->slab, h->slab_cap, sd);
        }
        // ConvT bias gradient: on the bf16 engine the sum of the (bf16) gradient the ConvT GEMMs read
        if (ps) cad::colsum_bf16(h->dcats[l], C, 0, h->Ml(l, B), C, h->dscr2, sd);
        else cad::colsum(h->dcat[l], 2 * C, C, h->Ml(l, B), C, h->dscr2, sd);
        cad::colsum_finalize(h->dscr2, cad::colsum_slices(h->Ml(l, B)), C, h->G(u.bidx), 1.f, sd);
        if (ps)
            cad::convT_dgrad_ps(sv(h->dcats[l], C), u.cout, sv(u.wms, 4 * u.cout), u.cin, h->Sa, B, h->Hl(l + 1),
                                h->Wl(l + 1), st, true);
        else
            cad::convT_dgrad(h->dcat[l], 2 * C, C, u.cout, h->P(u.widx), u.cin, h->Sa, B, h->Hl(l + 1), h->Wl(l + 1), st);
        return;
    }
    // encoder side: stage 5 = bottleneck (level 4), 6..9 = enc4..enc1 (levels 3..0)
    const int l = 4 - (stage - 5);
    DoubleConv& e = h->enc[l];
    const int C = h->Cl(l);
    // bn2's gradient: the bottleneck's from dec4's ConvT dgrad (Sa), the others the skip half of dcat
    // (bf16 in dskips on the bf16 engine)
    const float* g = l == 4 ? h->Sa : ps ? static_cast<const float*>(h->dskips[l]) : h->dcat[l];
    const int64_t ldg = l == 4 || ps ? C : 2 * C;
    // the max-pool backward of the level below (its pooled gradient in Sc, written by the previous
    // stage) is folded into this block's bn2 backward instead of scattered into dcat beforehand
    // (always on the bf16 engine, whose skip gradient is bf16)
    const bool fold = pool_fold_on() || ps;
    const cad::PoolAdd pa{h->Sc, h->pidx[l + 1], h->Hl(l), h->Wl(l)};
    const cad::PoolAdd* pool = l < 4 && fold ? &pa : nullptr;
    if (l == 0) {
        double_conv_bwd(h, e, g, ldg, 0, h->x0, h->x0_ld, sv(h->x0s, h->x0_ld), B, nullptr, 0, st, nullptr, pool, nullptr,
                        nullptr, ps);
        return;
    }
    const int Cp = h->Cl(l - 1);
    // the bottleneck's output gradient (Sa) comes from dec4's ConvT dgrad: bf16 on the bf16 engine
    double_conv_bwd(h, e, g, ldg, 0, h->pool[l], Cp, sv(h->pools[l], Cp), B, h->Sc, Cp, st, nullptr, pool, nullptr,
                    nullptr, ps);
    // max-pool backward: the pooled gradient is added at the recorded argmax of dcat's skip half
    // (folded into the next stage's bn2 backward unless CAD_POOLFOLD=0)
    if (!fold)
        cad::maxpool_bwd(h->Sc, h->pidx[l], Cp, B, h->Hl(l - 1), h->Wl(l - 1), h->dcat[l - 1], 2 * Cp, st);
}

void compute_stage_ranges(cad_unet* h) {
    auto rng = [&](int first, int last) {
        const int64_t a = h->params[first].off;
        const int64_t b = h->params[last].off + h->params[last].n_int;
        return std::make_pair(a, b - a);
    };
    h->stage_range.clear();
    h->stage_range.push_back(rng(h->head_w, h->head_b));
    for (int l = 0; l < 4; ++l) h->stage_range.push_back(rng(h->dec[l].first_param, h->dec[l].last_param));
    for (int l = 4; l >= 0; --l) h->stage_range.push_back(rng(h->enc[l].first_param, h->enc[l].last_param));
}

// reference layout <-> internal layout
void ref_to_int(const PInfo& p, const float* src, std::vector<float>& dst) {
    dst.assign(p.n_int, 0.f);
    if (p.kind == P_CONV3) {   // (co, ci, ky, kx) -> [co][ky*3+kx][ci_pad]
        for (int co = 0; co < p.cout; ++co)
            for (int ci = 0; ci < p.cin_ref; ++ci)
                for (int t = 0; t < 9; ++t)
                    dst[((int64_t)co * 9 + t) * p.cin_int + ci] = src[((int64_t)co * p.cin_ref + ci) * 9 + t];
    } else if (p.kind == P_CONVT_W) {   // (ci, co, dy, dx) -> [ci][q][co]
        const int64_t ci_n = p.shape[0], co_n = p.shape[1];
        for (int64_t ci = 0; ci < ci_n; ++ci)
            for (int64_t co = 0; co < co_n; ++co)
                for (int q = 0; q < 4; ++q) dst[(ci * 4 + q) * co_n + co] = src[(ci * co_n + co) * 4 + q];
    } else {
        std::memcpy(dst.data(), src, sizeof(float) * p.n_ref);
    }
}
void int_to_ref(const PInfo& p, const float* src, float* dst) {
    if (p.kind == P_CONV3) {
        for (int co = 0; co < p.cout; ++co)
            for (int ci = 0; ci < p.cin_ref; ++ci)
                for (int t = 0; t < 9; ++t)
                    dst[((int64_t)co * p.cin_ref + ci) * 9 + t] = src[((int64_t)co * 9 + t) * p.cin_int + ci];
    } else if (p.kind == P_CONVT_W) {
        const int64_t ci_n = p.shape[0], co_n = p.shape[1];
        for (int64_t ci = 0; ci < ci_n; ++ci)
            for (int64_t co = 0; co < co_n; ++co)
                for (int q = 0; q < 4; ++q) dst[(ci * co_n + co) * 4 + q] = src[(ci * 4 + q) * co_n + co];
    } else {
        std::memcpy(dst, src, sizeof(float) * p.n_ref);
    }
}

// default init: reference module defaults (kaiming_uniform(a=sqrt5) => U(+-1/sqrt(fan_in)) weights and
// biases, BN weight 1 bias 0, running mean 0 var 1); deterministic host LCG stream (seed 42)
void default_init(cad_unet* h) {
    uint64_t s = 0x2545F4914F6CDD1Dull ^ 42;
    auto rnd = [&]() {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        return (float)((s >> 40) * (1.0 / 16777216.0));
    };
    auto normal = [&]() {   // Box-Muller
        const float u1 = std::max(rnd(), 1e-7f), u2 = rnd();
        return std::sqrt(-2.f * std::log(u1)) * std::cos(6.2831853f * u2);
    };
    std::vector<float> ref, inter;
    for (const PInfo& p : h->params) {
        ref.assign(p.n_ref, 0.f);
        if (p.kind == P_BNW || p.kind == P_FILM_GAMMA_B) std::fill(ref.begin(), ref.end(), 1.f);
        else if (p.kind == P_BNB || p.kind == P_FILM_BETA_B) { /* zeros */ }
        else if (p.kind == P_FILM_HEAD_W) { for (auto& x : ref) x = 0.01f * normal(); }   // N(0, 0.01)
        else if (p.kind == P_FC_W || p.kind == P_FC_B) {
            const PInfo& w = p.kind == P_FC_W ? p : h->params[&p - &h->params[0] - 1];
            const float bound = 1.f / std::sqrt((float)w.shape[1]);
            for (auto& x : ref) x = (rnd() * 2.f - 1.f) * bound;
        } else {
            int64_t fan_in;
            if (p.kind == P_CONV3) fan_in = (int64_t)p.cin_ref * 9;
            else if (p.kind == P_CONVT_W || p.kind == P_CONVT_B) {
                const PInfo& w = p.kind == P_CONVT_W ? p : h->params[&p - &h->params[0] - 1];
                fan_in = w.shape[1] * 4;
            } else fan_in = h->f;
            const float bound = 1.f / std::sqrt((float)fan_in);
            for (auto& x : ref) x = (rnd() * 2.f - 1.f) * bound;
        }
        ref_to_int(p, ref.data(), inter);
        HIPCHK(hipMemcpy(h->flat_p + p.off, inter.data(), sizeof(float) * p.n_int, hipMemcpyHostToDevice));
    }
    for (const BufInfo& b : h->bufs) {
        std::vector<float> v(b.C, b.name.find("running_var") != std::string::npos ? 1.f : 0.f);
        HIPCHK(hipMemcpy(b.ptr, v.data(), sizeof(float) * b.C, hipMemcpyHostToDevice));
    }
}

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

int cad_abi_version(void) { return CAD_ABI_VERSION; }
cad_status cad_set_gemm_engine(int engine) {
    return guard([&] {
        require(engine == CAD_GEMM_F32 || engine == CAD_GEMM_S3 || engine == CAD_GEMM_BF16, "unknown GEMM engine");
        cad::set_gemm_engine(engine);
    });
}
int cad_get_gemm_engine(void) { return cad::gemm_engine(); }
const char* cad_last_error(void) { return g_err.c_str(); }

cad_status cad_device_count(int* n) {
    return guard([&] { HIPCHK(hipGetDeviceCount(n)); });
}
cad_status cad_set_device(int device) {
    return guard([&] { HIPCHK(hipSetDevice(device)); });
}
cad_status cad_stream_synchronize(void* stream) {
    return guard([&] { HIPCHK(hipStreamSynchronize(S(stream))); });
}

cad_status cad_malloc(int device, int64_t bytes, void** out) {
    return guard([&] {
        require(out && bytes >= 0, "bad arguments");
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipMalloc(out, (size_t)std::max<int64_t>(bytes, 1)));
    });
}
void cad_free(void* p) {
    if (p) (void)hipFree(p);
}
cad_status cad_memcpy(void* dst, const void* src, int64_t bytes, int kind, void* stream) {
    return guard([&] {
        require(kind >= 0 && kind <= 2 && bytes >= 0, "bad memcpy arguments");
        const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                              : hipMemcpyDeviceToDevice;
        if (stream) HIPCHK(hipMemcpyAsync(dst, src, (size_t)bytes, k, S(stream)));
        else HIPCHK(hipMemcpy(dst, src, (size_t)bytes, k));
    });
}

cad_status cad_unet_create(const cad_unet_desc* d, int device, cad_unet** out) {
    return cad_unet_create_model(d, CAD_MODEL_BASELINE, device, out);
}

cad_status cad_unet_create_model(const cad_unet_desc* d, int model, int device, cad_unet** out) {
    return guard([&] {
        require(d && out, "null argument");
        require(model == CAD_MODEL_BASELINE || model == CAD_MODEL_INTRINSICS_FILM || model == CAD_MODEL_RAY_FILM,
                "unknown model kind");
        require(d->in_channels == 3, "in_channels must be 3 (rgb)");
        require(d->init_features >= 4 && d->init_features % 4 == 0, "init_features must be a multiple of 4");
        require(d->height > 0 && d->width > 0 && d->height % 16 == 0 && d->width % 16 == 0,
                "height/width must be positive multiples of 16");
        require(d->max_batch >= 1, "max_batch must be >= 1");
        HIPCHK(hipSetDevice(device));
        auto h = std::make_unique<cad_unet>();
        h->device = device;
        h->model = model;
        h->x0_ld = 8;
        h->in_ch = d->in_channels;
        h->f = d->init_features;
        h->max_depth = d->max_depth;
        h->Bmax = d->max_batch;
        h->H = d->height;
        h->W = d->width;
        build_tables(h.get());
        Arena sz;
        layout(h.get(), sz);
        void* base = nullptr;
        HIPCHK(hipMalloc(&base, sz.off + 4096));
        HIPCHK(hipMemset(base, 0, sz.off + 4096));
        h->arena_base = base;
        Arena real;
        real.base = static_cast<char*>(base);
        layout(h.get(), real);
        require(real.off == sz.off, "internal: arena layout differs between the sizing and the real pass", CAD_ERR_STATE);
        compute_stage_ranges(h.get());
        default_init(h.get());
        HIPCHK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
        for (hipEvent_t* e : {&h->ev_fork, &h->evA, &h->evB, &h->ev_tail})
            HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        HIPCHK(hipDeviceSynchronize());
        *out = h.release();
    });
}

void cad_unet_destroy(cad_unet* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->side) (void)hipStreamSynchronize(h->side);
    for (hipEvent_t e : {h->ev_fork, h->evA, h->evB, h->ev_tail})
        if (e) (void)hipEventDestroy(e);
    if (h->side) (void)hipStreamDestroy(h->side);
    (void)hipFree(h->arena_base);
    delete h;
}

int64_t cad_unet_count_parameters(const cad_unet* h) {
    int64_t n = 0;
    for (const auto& p : h->params) n += p.n_ref;
    return n;
}
int cad_unet_num_params(const cad_unet* h) { return (int)h->params.size(); }
int cad_unet_model(const cad_unet* h) { return h->model; }
int cad_unet_num_buffers(const cad_unet* h) { return (int)h->bufs.size(); }

cad_status cad_unet_tensor_info(const cad_unet* h, int kind, int idx, const char** name, int* ndim, int64_t shape[4]) {
    return guard([&] {
        if (kind == 0) {
            require(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
            const PInfo& p = h->params[idx];
            if (name) *name = p.name.c_str();
            if (ndim) *ndim = p.ndim;
            if (shape) for (int i = 0; i < 4; ++i) shape[i] = p.shape[i];
        } else {
            require(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            const BufInfo& b = h->bufs[idx];
            if (name) *name = b.name.c_str();
            if (ndim) *ndim = 1;
            if (shape) { shape[0] = b.C; shape[1] = shape[2] = shape[3] = 1; }
        }
    });
}

cad_status cad_unet_set_tensor(cad_unet* h, int kind, int idx, const float* host, int64_t numel) {
    return guard([&] {
        HIPCHK(hipSetDevice(h->device));
        if (kind == 0) {
            require(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
            const PInfo& p = h->params[idx];
            require(numel == p.n_ref, "numel mismatch for " + p.name);
            std::vector<float> inter;
            ref_to_int(p, host, inter);
            HIPCHK(hipMemcpy(h->flat_p + p.off, inter.data(), sizeof(float) * p.n_int, hipMemcpyHostToDevice));
        } else {
            require(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            require(numel == h->bufs[idx].C, "numel mismatch for " + h->bufs[idx].name);
            HIPCHK(hipMemcpy(h->bufs[idx].ptr, host, sizeof(float) * numel, hipMemcpyHostToDevice));
        }
    });
}

static void get_slab_tensor(const cad_unet* h, const float* slab, int idx, float* host, int64_t numel) {
    require(idx >= 0 && idx < (int)h->params.size(), "param index out of range");
    const PInfo& p = h->params[idx];
    require(numel == p.n_ref, "numel mismatch for " + p.name);
    std::vector<float> inter(p.n_int);
    HIPCHK(hipMemcpy(inter.data(), slab + p.off, sizeof(float) * p.n_int, hipMemcpyDeviceToHost));
    int_to_ref(p, inter.data(), host);
}

cad_status cad_unet_get_tensor(const cad_unet* h, int kind, int idx, float* host, int64_t numel) {
    return guard([&] {
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        if (kind == 0) {
            get_slab_tensor(h, h->flat_p, idx, host, numel);
        } else {
            require(idx >= 0 && idx < (int)h->bufs.size(), "buffer index out of range");
            require(numel == h->bufs[idx].C, "numel mismatch");
            HIPCHK(hipMemcpy(host, h->bufs[idx].ptr, sizeof(float) * numel, hipMemcpyDeviceToHost));
        }
    });
}

cad_status cad_unet_get_grad(const cad_unet* h, int idx, float* host, int64_t numel) {
    return guard([&] {
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        get_slab_tensor(h, h->flat_g, idx, host, numel);
    });
}

cad_status cad_unet_train(cad_unet* h, int train) {
    return guard([&] { h->train = train != 0; });
}

cad_status cad_unet_flat(cad_unet* h, float** params, float** grads, int64_t* n) {
    return guard([&] {
        if (params) *params = h->flat_p;
        if (grads) *grads = h->flat_g;
        if (n) *n = h->n_flat;
    });
}

int64_t cad_unet_debug_buffer(cad_unet* h, const char* name, float* host, int64_t numel) {
    const int B = h->fwd_B > 0 ? h->fwd_B : h->Bmax;
    std::string n(name ? name : "");
    const float* p = nullptr;
    int64_t cnt = -1;
    auto lvl = [&](const std::string& pre) -> int {
        if (n.compare(0, pre.size(), pre) != 0 || n.size() < pre.size() + 1) return -1;
        return n[pre.size()] - '0';
    };
    int l;
    bool bf16 = false;   // the buffer holds bf16 values (widened to fp32 on the copy)
    if (n == "x0") { p = h->x0; cnt = h->Ml(0, B) * h->x0_ld; }
    else if (n == "Sa" || n == "Sb") { p = n == "Sa" ? h->Sa : h->Sb; cnt = h->Ml(0, B) * h->Cl(0); }
    else if (n == "Sc") { p = h->Sc; cnt = h->Ml(1, B) * h->Cl(0); }
    else if (n == "bott") { p = h->a2_bott; cnt = h->Ml(4, B) * h->Cl(4); }
    else if ((l = lvl("dcat")) >= 0 && l < 4) { p = h->dcat[l]; cnt = h->Ml(l, B) * 2 * h->Cl(l); }
    else if ((l = lvl("cat")) >= 0 && l < 4) { p = h->cat[l]; cnt = h->Ml(l, B) * 2 * h->Cl(l); }
    else if ((l = lvl("pool")) >= 1 && l <= 4) { p = h->pool[l]; cnt = h->Ml(l, B) * h->Cl(l - 1); }
    else if ((l = lvl("dout")) >= 0 && l < 4) { p = h->dout[l]; cnt = h->Ml(l, B) * h->Cl(l); }
    else if (((l = lvl("enc")) >= 0 && l < 5) || ((l = lvl("dec")) >= 0 && l < 4)) {
        DoubleConv& dc = n[0] == 'e' ? h->enc[l] : h->dec[l];
        const std::string t = n.size() > 5 ? n.substr(5) : "";
        p = t == "y1" ? dc.y1 : t == "a1" ? dc.a1 : t == "y2" ? dc.y2 : nullptr;
        cnt = p ? h->Ml(l, B) * h->Cl(l) : -1;
        bf16 = (t == "y1" && dc.y1b) || (t == "y2" && dc.y2b);
        if (dc.has_film() && (t == "gamma" || t == "beta")) {
            p = t == "gamma" ? dc.film.gam : dc.film.bet;
            cnt = (int64_t)B * h->Cl(l);
        }
    }
    else if (n == "camn") { p = h->camn; cnt = (int64_t)B * 4; }
    if (!p || cnt < 0) {
        g_err = "unknown debug buffer '" + n + "'";
        return -1;
    }
    if (n == "dout0" && h->head_fused) {
        g_err = "debug buffer 'dout0' is not written when decoder level 0 is fused with the head (CAD_HEADFUSE=0 keeps it)";
        return -1;
    }
    // With pre-split operands (bf16 engine) the last forward/backward wrote only the bf16 twins of
    // these buffers: their fp32 copies are stale, so refuse them rather than return old data
    if (h->fwd_np > 0) {
        const bool twin_only = n == "Sb" || n == "bott" || (n.compare(0, 4, "pool") == 0) ||
                               (n.compare(0, 3, "cat") == 0) ||   // up half: twin only
                               (n.compare(0, 4, "dout") == 0 && n != "dout0") ||
                               (n.size() > 5 && n.substr(5) == "a1");
        if (twin_only) {
            g_err = "debug buffer '" + n + "' holds no fp32 copy on the pre-split (bf16) engine";
            return -1;
        }
    }
    if (host) {
        if (numel < cnt) return -1;
        if (hipDeviceSynchronize() != hipSuccess) return -1;
        if (bf16) {   // pre-BN conv outputs of the bf16 engine: the stored bf16 values, widened
            std::vector<uint16_t> tmp((size_t)cnt);
            if (hipMemcpy(tmp.data(), p, sizeof(uint16_t) * cnt, hipMemcpyDeviceToHost) != hipSuccess) return -1;
            for (int64_t i = 0; i < cnt; ++i) {
                const uint32_t u = (uint32_t)tmp[(size_t)i] << 16;
                std::memcpy(host + i, &u, 4);
            }
        } else if (hipMemcpy(host, p, sizeof(float) * cnt, hipMemcpyDeviceToHost) != hipSuccess) {
            return -1;
        }
    }
    return cnt;
}

cad_status cad_unet_use_external_slabs(cad_unet* h, float* params, float* grads) {
    return guard([&] {
        require(params && grads, "null slab");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy(params, h->flat_p, sizeof(float) * h->n_flat, hipMemcpyDeviceToDevice));
        HIPCHK(hipMemcpy(grads, h->flat_g, sizeof(float) * h->n_flat, hipMemcpyDeviceToDevice));
        h->flat_p = params;
        h->flat_g = grads;
    });
}

// ---- torch::save / torch::load checkpoints (torch_archive.cpp holds the format) ----
int64_t cad_unet_num_batches_tracked(const cad_unet* h) { return h ? h->nbt : -1; }

cad_status cad_unet_save_torch(cad_unet* h, const char* path) {
    return guard([&] {
        require(h && path, "null argument");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        std::deque<std::vector<float>> data;
        std::deque<std::string> names;
        std::vector<cad_archive_entry> E;
        auto entry = [&](const std::string& name, int kind, int dtype, int ndim, const int64_t* shape, const void* d) {
            names.push_back(name);
            cad_archive_entry e{};
            e.name = names.back().c_str();
            e.kind = kind; e.dtype = dtype; e.ndim = ndim; e.data = d;
            for (int k = 0; k < ndim; ++k) e.shape[k] = shape[k];
            E.push_back(e);
        };
        // parameters in named_parameters() order; the encoder blocks' MaxPool2d ("pool", registered
        // before "conv", baseline_unet.h:56 / intrinsics_unet.h:65) has no tensors but is a submodule
        const char* pooled[4] = {"enc2.", "enc3.", "enc4.", "bottleneck."};
        bool placed[4] = {};
        for (size_t i = 0; i < h->params.size(); ++i) {
            const PInfo& p = h->params[i];
            for (int k = 0; k < 4; ++k)
                if (!placed[k] && p.name.rfind(std::string(pooled[k]) + "conv.", 0) == 0) {
                    entry(std::string(pooled[k]) + "pool", 2, CAD_DTYPE_F32, 0, nullptr, nullptr);
                    placed[k] = true;
                }
            data.emplace_back((size_t)p.n_ref);
            get_slab_tensor(h, h->flat_p, (int)i, data.back().data(), p.n_ref);
            entry(p.name, 0, CAD_DTYPE_F32, p.ndim, p.shape, data.back().data());
        }
        // buffers: running_mean, running_var, num_batches_tracked per BatchNorm
        for (const BufInfo& b : h->bufs) {
            data.emplace_back((size_t)b.C);
            HIPCHK(hipMemcpy(data.back().data(), b.ptr, sizeof(float) * b.C, hipMemcpyDeviceToHost));
            const int64_t C = b.C;
            entry(b.name, 1, CAD_DTYPE_F32, 1, &C, data.back().data());
            const std::string tail = ".running_var";
            if (b.name.size() > tail.size() && b.name.compare(b.name.size() - tail.size(), tail.size(), tail) == 0) {
                const bool film = b.name.find(".film.") != std::string::npos;
                entry(b.name.substr(0, b.name.size() - tail.size()) + ".num_batches_tracked", 1, CAD_DTYPE_I64, 0,
                      nullptr, film ? &h->nbt_film : &h->nbt);
            }
        }
        if (cad_archive_write(path, E.data(), (int)E.size()) != CAD_OK) throw std::runtime_error(cad_last_error());
    });
}

}  // extern "C"

namespace {
float half_to_float(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000) << 16, exp = (h >> 10) & 0x1F, man = h & 0x3FF;
    float v;
    if (exp == 0) v = std::ldexp((float)man, -24);                    // zero / subnormal
    else if (exp == 31) v = man ? NAN : INFINITY;
    else v = std::ldexp((float)(man | 0x400), (int)exp - 25);
    uint32_t w;
    std::memcpy(&w, &v, 4);
    w |= sign;
    std::memcpy(&v, &w, 4);
    return v;
}

// one archive tensor as fp32 host values (float dtypes converted; integer dtypes refused)
std::vector<float> archive_f32(const cad_archive* a, int i, const std::string& name) {
    int dt = 0, nd = 0;
    int64_t shp[8];
    if (cad_archive_info(a, i, nullptr, &dt, &nd, shp) != CAD_OK) throw std::runtime_error(cad_last_error());
    int64_t n = 1;
    for (int k = 0; k < nd; ++k) n *= shp[k];
    std::vector<float> out((size_t)n);
    auto read = [&](void* dst, int64_t bytes) {
        if (cad_archive_read(a, i, dst, bytes) != CAD_OK) throw std::runtime_error(cad_last_error());
    };
    if (dt == CAD_DTYPE_F32) {
        read(out.data(), n * 4);
    } else if (dt == CAD_DTYPE_F64) {
        std::vector<double> t((size_t)n);
        read(t.data(), n * 8);
        for (int64_t k = 0; k < n; ++k) out[(size_t)k] = (float)t[(size_t)k];
    } else if (dt == CAD_DTYPE_F16 || dt == CAD_DTYPE_BF16) {
        std::vector<uint16_t> t((size_t)n);
        read(t.data(), n * 2);
        for (int64_t k = 0; k < n; ++k) {
            const uint16_t u = t[(size_t)k];
            if (dt == CAD_DTYPE_BF16) {
                const uint32_t w = (uint32_t)u << 16;
                std::memcpy(&out[(size_t)k], &w, 4);
            } else {
                out[(size_t)k] = half_to_float(u);
            }
        }
    } else {
        throw std::runtime_error("'" + name + "' is not a floating-point tensor in the archive");
    }
    return out;
}
}  // namespace

extern "C" {

cad_status cad_unet_load_torch(cad_unet* h, const char* path) {
    return guard([&] {
        require(h && path, "null argument");
        cad_archive* raw = nullptr;
        if (cad_archive_open(path, &raw) != CAD_OK) throw std::runtime_error(cad_last_error());
        std::unique_ptr<cad_archive, void (*)(cad_archive*)> a(raw, cad_archive_close);
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        auto find = [&](const std::string& name, int ndim, const int64_t* shape) {
            const int i = cad_archive_find(a.get(), name.c_str());
            require(i >= 0, "checkpoint has no '" + name + "'");
            int nd = 0;
            int64_t shp[8];
            cad_archive_info(a.get(), i, nullptr, nullptr, &nd, shp);
            bool same = nd == ndim;
            for (int k = 0; same && k < nd; ++k) same = shp[k] == shape[k];
            require(same, "shape mismatch for '" + name + "' between the checkpoint and the model");
            return i;
        };
        // read everything first: a failing checkpoint leaves the model untouched
        std::vector<std::vector<float>> pv, bv;
        for (const PInfo& p : h->params) pv.push_back(archive_f32(a.get(), find(p.name, p.ndim, p.shape), p.name));
        for (const BufInfo& b : h->bufs) {
            const int64_t C = b.C;
            bv.push_back(archive_f32(a.get(), find(b.name, 1, &C), b.name));
        }
        auto counter = [&](bool film) -> int64_t {
            int64_t v = -1;
            for (const BufInfo& b : h->bufs) {
                const std::string tail = ".running_var";
                if (b.name.size() <= tail.size() || b.name.compare(b.name.size() - tail.size(), tail.size(), tail) != 0) continue;
                if ((b.name.find(".film.") != std::string::npos) != film) continue;
                const std::string n = b.name.substr(0, b.name.size() - tail.size()) + ".num_batches_tracked";
                const int i = find(n, 0, nullptr);
                int dt = 0;
                cad_archive_info(a.get(), i, nullptr, &dt, nullptr, nullptr);
                int64_t x = 0;
                if (dt == CAD_DTYPE_I64) {
                    if (cad_archive_read(a.get(), i, &x, 8) != CAD_OK) throw std::runtime_error(cad_last_error());
                } else if (dt == CAD_DTYPE_I32) {
                    int32_t y = 0;
                    if (cad_archive_read(a.get(), i, &y, 4) != CAD_OK) throw std::runtime_error(cad_last_error());
                    x = y;
                } else {
                    throw std::runtime_error("'" + n + "' is not an integer tensor");
                }
                v = std::max(v, x);
            }
            return v;
        };
        const int64_t n2 = counter(false), n1 = counter(true);
        for (size_t i = 0; i < h->params.size(); ++i) {
            std::vector<float> inter;
            ref_to_int(h->params[i], pv[i].data(), inter);
            HIPCHK(hipMemcpy(h->flat_p + h->params[i].off, inter.data(), sizeof(float) * h->params[i].n_int,
                             hipMemcpyHostToDevice));
        }
        for (size_t i = 0; i < h->bufs.size(); ++i)
            HIPCHK(hipMemcpy(h->bufs[i].ptr, bv[i].data(), sizeof(float) * h->bufs[i].C, hipMemcpyHostToDevice));
        if (n2 >= 0) h->nbt = n2;
        if (n1 >= 0) h->nbt_film = n1;
    });
}

cad_status cad_unet_forward(cad_unet* h, const float* rgb, float* depth, int B, void* stream) {
    return cad_unet_forward_cam(h, rgb, nullptr, depth, B, stream);
}

cad_status cad_unet_forward_cam(cad_unet* h, const float* rgb, const float* cam4, float* depth, int B, void* stream) {
    return guard([&] {
        require(rgb && depth, "null tensor");
        require(B >= 1 && B <= h->Bmax, "batch exceeds max_batch");
        require(h->model == CAD_MODEL_BASELINE || cam4, "this model is conditioned on camera intrinsics: pass cam4");
        HIPCHK(hipSetDevice(h->device));
        unet_forward(h, rgb, cam4, depth, B, S(stream));
        HIPCHK(hipGetLastError());
        if (h->train) {
            ++h->nbt;
            if (B > 1) ++h->nbt_film;
        }
        h->have_fwd = h->train;
        h->fwd_B = B;
    });
}

int cad_unet_num_stages(const cad_unet*) { return kStages; }

cad_status cad_model_grad_layout(int model, int in_channels, int init_features, int* nstages, int64_t stage_off[16],
                                 int64_t stage_cnt[16], int64_t* n_flat) {
    return guard([&] {
        require(model == CAD_MODEL_BASELINE || model == CAD_MODEL_INTRINSICS_FILM || model == CAD_MODEL_RAY_FILM,
                "unknown model kind");
        require(in_channels == 3 && init_features >= 4 && init_features % 4 == 0, "bad model description");
        cad_unet t;   // tables only: no device memory is touched
        t.model = model;
        t.in_ch = in_channels;
        t.f = init_features;
        build_tables(&t);
        compute_stage_ranges(&t);
        if (nstages) *nstages = kStages;
        for (int s = 0; s < kStages; ++s) {
            if (stage_off) stage_off[s] = t.stage_range[s].first;
            if (stage_cnt) stage_cnt[s] = t.stage_range[s].second;
        }
        if (n_flat) *n_flat = t.n_flat;
    });
}

cad_status cad_unet_backward_stage(cad_unet* h, int stage, const float* ddepth, void* stream) {
    return guard([&] {
        require(h->have_fwd, "backward needs a preceding train-mode forward", CAD_ERR_STATE);
        // the forward kept only the split twins of some operands (a1) for the pre-split backward
        require(h->fwd_np == 0 || h->fwd_np == cad::split_planes(),
                "GEMM engine changed between forward and backward", CAD_ERR_STATE);
        require(stage >= 0 && stage < kStages, "stage out of range");
        require(stage != 0 || ddepth, "null ddepth");
        HIPCHK(hipSetDevice(h->device));
        backward_stage(h, stage, ddepth, S(stream));
        HIPCHK(hipGetLastError());
    });
}

cad_status cad_unet_backward(cad_unet* h, const float* ddepth, void* stream) {
    return guard([&] {
        require(h->have_fwd, "backward needs a preceding train-mode forward", CAD_ERR_STATE);
        // the forward kept only the split twins of some operands (a1) for the pre-split backward
        require(h->fwd_np == 0 || h->fwd_np == cad::split_planes(),
                "GEMM engine changed between forward and backward", CAD_ERR_STATE);
        require(ddepth, "null ddepth");
        HIPCHK(hipSetDevice(h->device));
        // one join at the end: the side stream's weight gradients overlap across stages too
        h->defer_join = true;
        try {
            for (int s = 0; s < kStages; ++s) backward_stage(h, s, ddepth, S(stream));
        } catch (...) {
            h->defer_join = false;
            throw;
        }
        h->defer_join = false;
        side_join(h, S(stream));
        HIPCHK(hipGetLastError());
    });
}

cad_status cad_unet_stage_grad_range(const cad_unet* h, int stage, int64_t* offset, int64_t* count) {
    return guard([&] {
        require(stage >= 0 && stage < kStages, "stage out of range");
        if (offset) *offset = h->stage_range[stage].first;
        if (count) *count = h->stage_range[stage].second;
    });
}

cad_status cad_clip_grad_norm(cad_unet* h, float max_norm, float prescale, void* stream) {
    return guard([&] {
        HIPCHK(hipSetDevice(h->device));
        cad::grad_norm_clip(h->flat_g, h->n_flat, max_norm, prescale, h->dscr, h->norm_coef, S(stream));
        HIPCHK(hipGetLastError());
    });
}

cad_status cad_unet_last_grad_norm(cad_unet* h, float* total_norm, void* stream) {
    return guard([&] {
        float v[2];
        HIPCHK(hipMemcpyAsync(v, h->norm_coef, sizeof(v), hipMemcpyDeviceToHost, S(stream)));
        HIPCHK(hipStreamSynchronize(S(stream)));
        *total_norm = v[0];
    });
}

cad_status cad_adam_create(cad_unet* model, const cad_adam_opts* o, cad_adam** out) {
    return guard([&] {
        require(model && o && out, "null argument");
        HIPCHK(hipSetDevice(model->device));
        auto a = std::make_unique<cad_adam>();
        a->model = model;
        a->o = *o;
        HIPCHK(hipMalloc(&a->m, sizeof(float) * model->n_flat));
        HIPCHK(hipMalloc(&a->v, sizeof(float) * model->n_flat));
        HIPCHK(hipMemset(a->m, 0, sizeof(float) * model->n_flat));
        HIPCHK(hipMemset(a->v, 0, sizeof(float) * model->n_flat));
        *out = a.release();
    });
}
void cad_adam_destroy(cad_adam* a) {
    if (!a) return;
    (void)hipFree(a->m);
    (void)hipFree(a->v);
    delete a;
}
cad_status cad_adam_step(cad_adam* a, void* stream) {
    return guard([&] {
        cad_unet* h = a->model;
        HIPCHK(hipSetDevice(h->device));
        a->step += 1;
        cad::adam_step(h->flat_p, h->flat_g, a->m, a->v, h->n_flat, h->norm_coef, a->o.lr, a->o.beta1, a->o.beta2,
                       a->o.eps, a->o.weight_decay, (int)a->step, S(stream));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_adam_set_lr(cad_adam* a, float lr) {
    return guard([&] { a->o.lr = lr; });
}
int64_t cad_adam_step_count(const cad_adam* a) { return a->step; }
cad_status cad_adam_state(cad_adam* a, float** m, float** v) {
    return guard([&] {
        if (m) *m = a->m;
        if (v) *v = a->v;
    });
}
cad_status cad_adam_set_step_count(cad_adam* a, int64_t step) {
    return guard([&] {
        require(step >= 0, "negative step");
        a->step = step;
    });
}

cad_status cad_loss_create(float si, float gr, float sm, float rp, int max_batch, int height, int width, int device,
                           cad_loss** out) {
    return guard([&] {
        require(out && max_batch >= 1 && height >= 2 && width >= 2, "bad loss arguments");
        HIPCHK(hipSetDevice(device));
        auto l = std::make_unique<cad_loss>();
        l->device = device; l->Bmax = max_batch; l->H = height; l->W = width;
        l->w[0] = si; l->w[1] = gr; l->w[2] = sm; l->w[3] = rp;
        const int64_t nf = cad::loss_workspace_floats(max_batch, height, width);
        const int64_t nd = cad::loss_part_doubles(max_batch, height, width);
        size_t bytes = ((sizeof(double) * nd + 255) & ~size_t(255)) + sizeof(float) * (nf + 64);
        HIPCHK(hipMalloc(&l->base, bytes));
        HIPCHK(hipMemset(l->base, 0, bytes));
        l->ws.part = static_cast<double*>(l->base);
        l->ws.part_cap = nd;
        l->ws.pyr = reinterpret_cast<float*>(static_cast<char*>(l->base) + ((sizeof(double) * nd + 255) & ~size_t(255)));
        l->out5 = l->ws.pyr + nf;
        *out = l.release();
    });
}
void cad_loss_destroy(cad_loss* l) {
    if (!l) return;
    (void)hipFree(l->base);
    delete l;
}
cad_status cad_loss_forward_backward(cad_loss* l, const float* pred, const float* gt, const float* rgb, const float* K,
                                     int B, float* loss5, float* dpred, void* stream) {
    return cad_loss_forward_backward_masked(l, pred, gt, rgb, K, nullptr, B, loss5, dpred, stream);
}
cad_status cad_loss_forward_backward_masked(cad_loss* l, const float* pred, const float* gt, const float* rgb,
                                            const float* K, const uint8_t* mask, int B, float* loss5, float* dpred,
                                            void* stream) {
    return guard([&] {
        require(pred && gt && rgb && K && dpred, "null tensor");
        require(B >= 1 && B <= l->Bmax, "batch exceeds max_batch");
        HIPCHK(hipSetDevice(l->device));
        cad::loss_fwd_bwd(pred, gt, rgb, K, mask, B, l->H, l->W, l->w, loss5 ? loss5 : l->out5, dpred, l->ws, S(stream));
        if (loss5) HIPCHK(hipMemcpyAsync(l->out5, loss5, 5 * sizeof(float), hipMemcpyDeviceToDevice, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_loss_get_components(cad_loss* l, float out5[5], void* stream) {
    return guard([&] {
        HIPCHK(hipMemcpyAsync(out5, l->out5, 5 * sizeof(float), hipMemcpyDeviceToHost, S(stream)));
        HIPCHK(hipStreamSynchronize(S(stream)));
    });
}

cad_status cad_depth_metrics(const float* pred, const float* gt, int B, int H, int W, float out7[7], void* stream) {
    return guard([&] {
        require(pred && gt && out7 && B > 0, "bad arguments");
        double* part = nullptr;
        const int nb = cad::metrics_blocks((int64_t)H * W);
        HIPCHK(hipMalloc((void**)&part, sizeof(double) * (size_t)B * nb * 8));
        cad::depth_metrics_partials(pred, gt, B, (int64_t)H * W, part, nb, S(stream));
        std::vector<double> hp((size_t)B * nb * 8);
        HIPCHK(hipMemcpyAsync(hp.data(), part, sizeof(double) * hp.size(), hipMemcpyDeviceToHost, S(stream)));
        HIPCHK(hipStreamSynchronize(S(stream)));
        HIPCHK(hipFree(part));
        // computeDepthMetrics per sample (enhanced.h:400-439), averaged over samples (:383-391)
        double acc[7] = {0, 0, 0, 0, 0, 0, 0};
        for (int b = 0; b < B; ++b) {
            double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int i = 0; i < nb; ++i)
                for (int q = 0; q < 8; ++q) t[q] += hp[((size_t)b * nb + i) * 8 + q];
            if (t[0] <= 0) continue;   // no valid pixel: the reference returns zeros for the sample
            acc[0] += t[1] / t[0];
            acc[1] += t[2] / t[0];
            acc[2] += std::sqrt(t[3] / t[0]);
            acc[3] += std::sqrt(t[4] / t[0]);
            acc[4] += t[5] / t[0];
            acc[5] += t[6] / t[0];
            acc[6] += t[7] / t[0];
        }
        for (int q = 0; q < 7; ++q) out7[q] = (float)(acc[q] / B);
    });
}

cad_status cad_camera_from_K(const float* K, int B, float* cam4, void* stream) {
    return guard([&] {
        require(K && cam4 && B > 0, "bad arguments");
        cad::camera_from_K(K, B, cam4, S(stream));
        HIPCHK(hipGetLastError());
    });
}

cad_status cad_ray_directions(const float* K, int B, int H, int W, float* rays, void* stream) {
    return guard([&] {
        require(K && rays && B > 0 && H > 0 && W > 0, "bad arguments");
        cad::ray_directions(K, B, H, W, rays, S(stream));
        HIPCHK(hipGetLastError());
    });
}

// ---------------- batch assembly (SunRGBDLoader::getSample resize + augmentation, on device) -------
struct cad_batcher {
    int device = 0, Bmax = 0, H = 0, W = 0;
    cad::BatchSample* dev = nullptr;    // [Bmax] launch parameters
    float* tmp = nullptr;               // stage-1 planes of augmented samples: [Bmax][3][H][W] + [Bmax][H][W]
    cad::BatchSample* host = nullptr;   // pinned staging: Bmax samples, then Bmax x 9 floats of K
    hipEvent_t staged = nullptr;        // the last upload from the staging buffer
};

cad_status cad_batcher_create(int max_batch, int height, int width, int device, cad_batcher** out) {
    return guard([&] {
        require(out && max_batch >= 1 && height >= 1 && width >= 1, "bad batcher arguments");
        HIPCHK(hipSetDevice(device));
        auto b = std::make_unique<cad_batcher>();
        b->device = device; b->Bmax = max_batch; b->H = height; b->W = width;
        HIPCHK(hipMalloc((void**)&b->dev, sizeof(cad::BatchSample) * max_batch));
        HIPCHK(hipMalloc((void**)&b->tmp, sizeof(float) * 4 * (size_t)max_batch * height * width));
        HIPCHK(hipHostMalloc((void**)&b->host, (sizeof(cad::BatchSample) + 9 * sizeof(float)) * max_batch));
        HIPCHK(hipEventCreateWithFlags(&b->staged, hipEventDisableTiming));
        *out = b.release();
    });
}
void cad_batcher_destroy(cad_batcher* b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    (void)hipEventSynchronize(b->staged);
    (void)hipEventDestroy(b->staged);
    (void)hipFree(b->dev);
    (void)hipFree(b->tmp);
    (void)hipHostFree(b->host);
    delete b;
}

cad_status cad_batcher_assemble(cad_batcher* b, const cad_sample* samples, int B, float* rgb, float* depth, float* K,
                                void* stream) {
    return guard([&] {
        require(b && samples && rgb && depth && K, "null argument");
        require(B >= 1 && B <= b->Bmax, "batch exceeds max_batch");
        HIPCHK(hipSetDevice(b->device));
        HIPCHK(hipEventSynchronize(b->staged));   // the staging buffer is free again
        const int H = b->H, W = b->W;
        float* Kh = reinterpret_cast<float*>(b->host + b->Bmax);
        bool any_aug = false;
        for (int i = 0; i < B; ++i) {
            const cad_sample& s = samples[i];
            require(s.rgb && s.depth && s.h0 >= 1 && s.w0 >= 1, "sample " + std::to_string(i) + ": no image");
            cad::BatchSample& d = b->host[i];
            d = cad::BatchSample{};
            d.rgb = s.rgb; d.depth = s.depth; d.h0 = s.h0; d.w0 = s.w0; d.bgr = s.bgr;
            require((s.dh0 == 0) == (s.dw0 == 0) && s.dh0 >= 0 && s.dw0 >= 0, "sample " + std::to_string(i) + ": bad depth size");
            d.dh0 = s.dh0 ? s.dh0 : s.h0;
            d.dw0 = s.dw0 ? s.dw0 : s.w0;
            d.depth_scale = s.depth_scale;
            // intrinsics with the reference's float operations
            float* k = Kh + 9 * i;
            for (int e = 0; e < 9; ++e) k[e] = s.K[e];
            if (s.h0 != H || s.w0 != W) {   // resizeSample :480-488
                const float sx = static_cast<float>(W) / s.w0, sy = static_cast<float>(H) / s.h0;
                k[0] = k[0] * sx; k[4] = k[4] * sy; k[2] = k[2] * sx; k[5] = k[5] * sy;
            }
            if (!s.aug) continue;
            any_aug = true;
            d.aug = 1;
            d.cy = 0; d.cx = 0; d.ch = H; d.cw = W;
            if (s.crop) {   // applyCrop :389-414 (torch Slice clamps the window to the image)
                const int chn = static_cast<int>(H * s.crop_scale), cwn = static_cast<int>(W * s.crop_scale);
                require(s.crop_x >= 0 && s.crop_y >= 0 && s.crop_x < W && s.crop_y < H && chn >= 1 && cwn >= 1,
                        "sample " + std::to_string(i) + ": crop window outside the image");
                d.cy = s.crop_y; d.cx = s.crop_x;
                d.ch = std::min(s.crop_y + chn, H) - s.crop_y;
                d.cw = std::min(s.crop_x + cwn, W) - s.crop_x;
                k[2] = k[2] - s.crop_x;
                k[5] = k[5] - s.crop_y;
            }
            if (s.flip) {   // applyHorizontalFlip :416-430
                d.flip = 1;
                k[2] = d.cw - k[2] - 1;
            }
            if (s.jitter) {   // applyColorJitter :432-443
                d.jitter = 1; d.contrast = s.contrast; d.brightness = s.brightness;
            }
            if (d.ch != H || d.cw != W) {   // the second resizeSample (getSample :165)
                const float sx = static_cast<float>(W) / d.cw, sy = static_cast<float>(H) / d.ch;
                k[0] = k[0] * sx; k[4] = k[4] * sy; k[2] = k[2] * sx; k[5] = k[5] * sy;
            }
        }
        HIPCHK(hipMemcpyAsync(b->dev, b->host, sizeof(cad::BatchSample) * B, hipMemcpyHostToDevice, S(stream)));
        HIPCHK(hipMemcpyAsync(K, Kh, sizeof(float) * 9 * B, hipMemcpyHostToDevice, S(stream)));
        HIPCHK(hipEventRecord(b->staged, S(stream)));
        float* rgb_tmp = b->tmp;
        float* depth_tmp = b->tmp + 3 * (size_t)b->Bmax * H * W;
        cad::batch_assemble(b->dev, B, H, W, any_aug, rgb, depth, rgb_tmp, depth_tmp, S(stream));
        HIPCHK(hipGetLastError());
    });
}

// augmentSample's draws (sunrgbd_loader.cpp:352-443): std::mt19937, same distributions, same order
struct cad_aug_sampler {
    cad_aug_config cfg;
    std::mt19937 rng;
};
cad_status cad_aug_sampler_create(const cad_aug_config* cfg, uint32_t seed, cad_aug_sampler** out) {
    return guard([&] {
        require(cfg && out, "null argument");
        require(cfg->crop_scale_min > 0.f && cfg->crop_scale_min <= cfg->crop_scale_max && cfg->crop_scale_max <= 1.f,
                "crop scale range must satisfy 0 < min <= max <= 1");
        auto s = std::make_unique<cad_aug_sampler>();
        s->cfg = *cfg;
        s->rng.seed(seed);
        *out = s.release();
    });
}
void cad_aug_sampler_destroy(cad_aug_sampler* s) { delete s; }
cad_status cad_aug_sampler_draw(cad_aug_sampler* s, int height, int width, cad_sample* smp) {
    return guard([&] {
        require(s && smp && height >= 1 && width >= 1, "bad arguments");
        const cad_aug_config& c = s->cfg;
        smp->aug = 1;
        smp->crop = c.enable_random_crop;
        if (c.enable_random_crop) {
            std::uniform_real_distribution<float> scale_dist(c.crop_scale_min, c.crop_scale_max);
            const float scale = scale_dist(s->rng);
            const int crop_h = static_cast<int>(height * scale), crop_w = static_cast<int>(width * scale);
            std::uniform_int_distribution<int> x_dist(0, std::max(1, width - crop_w));
            std::uniform_int_distribution<int> y_dist(0, std::max(1, height - crop_h));
            smp->crop_scale = scale;
            smp->crop_x = x_dist(s->rng);
            smp->crop_y = y_dist(s->rng);
        }
        smp->flip = 0;
        if (c.enable_horizontal_flip) {
            std::uniform_real_distribution<float> flip_dist(0.0f, 1.0f);
            smp->flip = flip_dist(s->rng) < c.horizontal_flip_prob;
        }
        smp->jitter = c.enable_color_jitter;
        if (c.enable_color_jitter) {
            std::uniform_real_distribution<float> bd(1.0f - c.brightness_delta, 1.0f + c.brightness_delta);
            std::uniform_real_distribution<float> cd(1.0f - c.contrast_delta, 1.0f + c.contrast_delta);
            smp->brightness = bd(s->rng);
            smp->contrast = cd(s->rng);
        }
    });
}

// ---------------- operator-level entry points ----------------
cad_status cad_op_conv3x3_fwd(const float* x, int64_t ldx, int xcoff, int cin, const float* w, int cout, float* y,
                              int64_t ldy, int ycoff, int B, int H, int W, void* stream) {
    return guard([&] {
        require(cin % 4 == 0 && cout % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && xcoff % 4 == 0 && ycoff % 4 == 0,
                "channels / strides must be multiples of 4");
        cad::conv3x3_fwd(x, ldx, xcoff, cin, w, cout, y, ldy, ycoff, B, H, W, nullptr, S(stream));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_conv3x3_dgrad(const float* dz, int cout, const float* w, int cin, float* dx, int64_t lddx, int B,
                                int H, int W, void* stream) {
    return guard([&] {
        require(cin % 4 == 0 && cout % 4 == 0, "channels must be multiples of 4");
        float* wd = nullptr;
        HIPCHK(hipMallocAsync((void**)&wd, sizeof(float) * (size_t)cout * 9 * cin, S(stream)));
        cad::repack_conv_dgrad(w, wd, cout, cin, S(stream));
        cad::conv3x3_dgrad(dz, cout, wd, cin, dx, lddx, B, H, W, S(stream));
        HIPCHK(hipFreeAsync(wd, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_conv3x3_wgrad(const float* dz, int cout, const float* x, int64_t ldx, int xcoff, int cin, float* dw,
                                int B, int H, int W, void* stream) {
    return guard([&] {
        require(cin % 4 == 0 && cout % 4 == 0, "channels must be multiples of 4");
        const int64_t cap = cad::wgrad_slab_floats(cout, 9 * cin, B * H * W);
        float* slab = nullptr;
        HIPCHK(hipMallocAsync((void**)&slab, sizeof(float) * (size_t)std::max<int64_t>(cap, 4), S(stream)));
        cad::conv3x3_wgrad(dz, cout, x, ldx, xcoff, cin, dw, B, H, W, slab, cap, S(stream));
        HIPCHK(hipFreeAsync(slab, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_conv3x3_wgrad_bf16(const void* dz, int64_t lddz, int cout, const void* x, int64_t ldx, int xcoff,
                                     int cin, float* dw, int B, int H, int W, void* stream) {
    return guard([&] {
        require(cad::gemm_engine() == 2, "the pre-split weight gradient runs on the bf16 engine (CAD_GEMM_BF16)");
        const int64_t cap = cad::wgrad_slab_floats(cout, 9 * cin, B * H * W);
        float* slab = nullptr;
        HIPCHK(hipMallocAsync((void**)&slab, sizeof(float) * (size_t)std::max<int64_t>(cap, 4), S(stream)));
        cad::conv3x3_wgrad_ps(cad::Split{dz, lddz, 0}, cout, cad::Split{x, ldx, xcoff}, cin, dw, B, H, W, slab, cap,
                              S(stream));
        HIPCHK(hipFreeAsync(slab, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_conv3x3_fwd_bf16(const void* x, int64_t ldx, int xcoff, int cin, const float* w, int cout, void* y,
                                  int64_t ldy, int ycoff, int y_bf16, int with_stats, int B, int H, int W, void* stream) {
    return guard([&] {
        require(cad::gemm_engine() == 2, "the pre-split convolution runs on the bf16 engine (CAD_GEMM_BF16)");
        require(x && w && y && cin % 8 == 0 && xcoff % 8 == 0 && ldx % 8 == 0 && B > 0 && H > 0 && W > 0,
                "bad arguments (bf16 rows: ldx, xcoff, cin multiples of 8)");
        void* ws = nullptr;
        float* stats = nullptr;
        HIPCHK(hipMallocAsync(&ws, sizeof(uint16_t) * (size_t)cout * 9 * cin, S(stream)));
        cad::split_rows(w, 9 * cin, 0, 9 * cin, cout, ws, 9 * cin, 0, S(stream));
        if (with_stats) {
            const int rows = cad::conv3x3_stats_rows(cin, B, H, W, cout, true);
            HIPCHK(hipMallocAsync((void**)&stats, sizeof(float) * ((size_t)rows * (2 * cout + 1) + 4), S(stream)));
        }
        cad::conv3x3_fwd_ps(cad::Split{x, ldx, xcoff}, cin, cad::Split{ws, 9 * cin, 0}, cout, static_cast<float*>(y), ldy,
                            ycoff, B, H, W, stats, S(stream), y_bf16 != 0);
        if (stats) HIPCHK(hipFreeAsync(stats, S(stream)));
        HIPCHK(hipFreeAsync(ws, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_conv3x3_dgrad_bf16(const void* dz, int64_t lddz, int cout, const float* w, int cin, void* dx,
                                    int64_t lddx, int dx_bf16, int B, int H, int W, void* stream) {
    return guard([&] {
        require(cad::gemm_engine() == 2, "the pre-split convolution runs on the bf16 engine (CAD_GEMM_BF16)");
        require(dz && w && dx && cout % 8 == 0 && cin % 8 == 0 && lddz % 8 == 0 && B > 0 && H > 0 && W > 0,
                "bad arguments (bf16 rows: lddz, cout, cin multiples of 8)");
        float* wd = nullptr;
        void* wds = nullptr;
        HIPCHK(hipMallocAsync((void**)&wd, sizeof(float) * (size_t)cout * 9 * cin, S(stream)));
        HIPCHK(hipMallocAsync(&wds, sizeof(uint16_t) * (size_t)cout * 9 * cin, S(stream)));
        cad::repack_conv_dgrad(w, wd, cout, cin, S(stream));
        cad::split_rows(wd, 9 * cout, 0, 9 * cout, cin, wds, 9 * cout, 0, S(stream));
        cad::conv3x3_dgrad_ps(cad::Split{dz, lddz, 0}, cout, cad::Split{wds, 9 * cout, 0}, cin, static_cast<float*>(dx),
                              lddx, B, H, W, S(stream), dx_bf16 != 0);
        HIPCHK(hipFreeAsync(wds, S(stream)));
        HIPCHK(hipFreeAsync(wd, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_mx8_quantize(const void* src, int src_bf16, int64_t lds, int scoff, int C, int64_t M, void* q,
                               void* s, int64_t ldq, int qcoff, void* stream) {
    return guard([&] {
        require(src && q && s && M >= 0, "null argument");
        cad::Mx8 d;
        d.q = q; d.s = s; d.ld = ldq; d.coff = qcoff;
        cad::mx8_quantize(src, src_bf16 != 0, lds, scoff, C, M, d, S(stream));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_dense_x8(const void* xq, const void* xs, int64_t ldx, int K, const void* wq, const void* ws,
                           int64_t ldw, int N, float* y, int64_t M, void* stream) {
    return guard([&] {
        require(cad::dense_x8_ok(K, N), "dense MX-fp8 GEMM: K % 128 == 0 and N % 64 == 0 required");
        cad::Mx8 x, w;
        x.q = xq; x.s = xs; x.ld = ldx;
        w.q = wq; w.s = ws; w.ld = ldw;
        cad::dense_fwd_x8(x, K, w, N, y, N, 0, M, nullptr, S(stream));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_conv3x3_x8(const void* xq, const void* xs, int64_t ldx, int cin, const void* wq, const void* ws,
                             int64_t ldw, int cout, float* y, int B, int H, int W, void* stream) {
    return guard([&] {
        require(cad::conv3x3_x8_ok(cin, W, cout), "MX-fp8 window conv: cin % 64, cout % 64, a block width dividing W");
        cad::Mx8 x, w;
        x.q = xq; x.s = xs; x.ld = ldx;
        w.q = wq; w.s = ws; w.ld = ldw;
        cad::conv3x3_fwd_x8(x, cin, w, cout, y, cout, 0, B, H, W, nullptr, S(stream));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_convT_fwd(const float* x, int cin, const float* w, const float* bias, int cout, float* y,
                            int64_t ldy, int ycoff, int B, int H, int W, void* stream) {
    return guard([&] {
        require(cin % 4 == 0 && cout % 4 == 0, "channels must be multiples of 4");
        float* wf = nullptr;
        HIPCHK(hipMallocAsync((void**)&wf, sizeof(float) * (size_t)cout * 4 * cin, S(stream)));
        cad::repack_convT_fwd(w, wf, cin, cout, S(stream));
        cad::convT_fwd(x, cin, cin, wf, bias, cout, y, ldy, ycoff, B, H, W, S(stream));
        HIPCHK(hipFreeAsync(wf, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_convT_fwd_bf16(const void* x, int64_t ldx, int xcoff, int cin, const float* w, const float* bias,
                                 int cout, void* y, int64_t ldy, int ycoff, int B, int H, int W, void* stream) {
    return guard([&] {
        require(cad::gemm_engine() == 2, "the pre-split ConvTranspose runs on the bf16 engine (CAD_GEMM_BF16)");
        require(x && w && bias && y && cin % 8 == 0 && cout % 8 == 0 && xcoff % 8 == 0 && ldx % 8 == 0 &&
                    ldy % 8 == 0 && ycoff % 8 == 0 && B > 0 && H > 0 && W > 0,
                "bad arguments (bf16 rows: ldx, xcoff, ldy, ycoff, cin, cout multiples of 8)");
        float* wf = nullptr;
        void* wfs = nullptr;
        HIPCHK(hipMallocAsync((void**)&wf, sizeof(float) * (size_t)cout * 4 * cin, S(stream)));
        HIPCHK(hipMallocAsync(&wfs, sizeof(uint16_t) * (size_t)cout * 4 * cin, S(stream)));
        cad::repack_convT_fwd(w, wf, cin, cout, S(stream));
        cad::split_rows(wf, cin, 0, cin, 4 * cout, wfs, cin, 0, S(stream));
        cad::convT_fwd_ps(cad::Split{x, ldx, xcoff}, cin, cad::Split{wfs, cin, 0}, bias, cout, static_cast<float*>(y),
                          ldy, ycoff, B, H, W, S(stream), true);
        HIPCHK(hipFreeAsync(wfs, S(stream)));
        HIPCHK(hipFreeAsync(wf, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_convT_dgrad(const float* g, int64_t ldg, int gcoff, int cout, const float* w, int cin, float* dx,
                              int B, int H, int W, void* stream) {
    return guard([&] {
        require(cin % 4 == 0 && cout % 4 == 0, "channels must be multiples of 4");
        cad::convT_dgrad(g, ldg, gcoff, cout, w, cin, dx, B, H, W, S(stream));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_convT_wgrad(const float* x, int cin, const float* g, int64_t ldg, int gcoff, int cout, float* dw,
                              int B, int H, int W, void* stream) {
    return guard([&] {
        require(cin % 4 == 0 && cout % 4 == 0, "channels must be multiples of 4");
        const int64_t cap = cad::wgrad_slab_floats(cin, 4 * cout, B * H * W);
        float* slab = nullptr;
        HIPCHK(hipMallocAsync((void**)&slab, sizeof(float) * (size_t)std::max<int64_t>(cap, 4), S(stream)));
        cad::convT_wgrad(x, cin, g, ldg, gcoff, cout, dw, B, H, W, slab, cap, S(stream));
        HIPCHK(hipFreeAsync(slab, S(stream)));
        HIPCHK(hipGetLastError());
    });
}
cad_status cad_op_maxpool_fwd(const float* x, int64_t ldx, int C, int B, int H, int W, float* out, uint8_t* idx,
                              void* stream) {
    return guard([&] {
        require(C % 4 == 0, "channels must be multiples of 4");
        cad::maxpool_fwd(x, ldx, C, B, H, W, out, idx, S(stream));
        HIPCHK(hipGetLastError());
    });
}

}  // extern "C"
