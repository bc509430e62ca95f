// Internal (C++) launch API of the HIP kernels.  All activations are NHWC fp32; "ld" is the row
// stride in floats between consecutive pixels, "coff" the channel offset inside a row (so the
// decoder concat buffer [pix][skip | up] is read and written in place).  Every launcher is
// asynchronous on the given stream and allocates nothing (graph-capture safe).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <initializer_list>

namespace cad {

// ---------------- launch profiler (host/profiler.cpp) ----------------
bool prof_enabled();
void prof_push(const char* name, double flops, hipStream_t st);
void prof_pop(hipStream_t st);

// ---------------- launch-level aliasing guard (host/alias.cpp) ----------------
// CAD_ALIAS_CHECK=1 (tests/conftest.py sets it): an instrumented launcher refuses a launch whose output
// byte range overlaps one of its inputs (std::invalid_argument naming both -> CAD_ERR_INVALID) unless
// the launcher declares that operand pair in place (it then leaves the pair out);
// CAD_ALIAS_CHECK=log:<path> only records the finding.  Off by default: CAD_NO_ALIAS tests one cached
// int and evaluates none of its arguments.
struct AliasView {
    const void* p = nullptr;
    int64_t rows = 0, ld = 0, coff = 0, cols = 0;   // rows of ld elements, columns [coff, coff + cols)
    int es = 4;                                     // element bytes
    const char* what = "";
};
inline AliasView aview(const void* p, int64_t rows, int64_t ld, int64_t coff, int64_t cols, int es, const char* what) {
    AliasView v;
    v.p = p; v.rows = rows; v.ld = ld; v.coff = coff; v.cols = cols; v.es = es; v.what = what;
    return v;
}
int alias_mode();
bool views_overlap(const AliasView& a, const AliasView& b);
void alias_check_impl(const char* op, std::initializer_list<AliasView> outs, std::initializer_list<AliasView> ins,
                      bool same_view_ok = false);
// CAD_NO_ALIAS("op", {outputs...}, {inputs...} [, same_view_ok])  (variadic: the braced lists hold commas;
// same_view_ok: an elementwise pass whose output may be exactly one of its inputs)
#define CAD_NO_ALIAS(...)                                                     \
    do {                                                                      \
        if (::cad::alias_mode()) ::cad::alias_check_impl(__VA_ARGS__);        \
    } while (0)

// ---------------- convolutions (conv_kernels.hip) ----------------
// GEMM engine of the conv / ConvT contractions: 0 = exact fp32 MFMA (v_mfma_f32_32x32x2_f32),
// 1 = S3: fp32 operands split exactly into three bf16 terms on the bf16 matrix cores (gemm_s3.hpp),
// 2 = B1: bf16-rounded operands, fp32 accumulation
void set_gemm_engine(int e);
int gemm_engine();
// y = conv3x3(x) (+ per-tile BN partials [rows][2][cout] when stats != nullptr)
void conv3x3_fwd(const float* x, int64_t ldx, int xcoff, int cin, const float* w, int cout, float* y,
                 int64_t ldy, int ycoff, int B, int H, int W, float* stats, hipStream_t st);
// BN partial rows of conv3x3_fwd (ps = true: of conv3x3_fwd_ps on the pre-split twins)
int conv3x3_stats_rows(int cin, int B, int H, int W, int cout, bool ps = false);
// dx[pix][ci] = conv3x3(dz, wd) with wd = repacked [ci][tap'][co]
void conv3x3_dgrad(const float* dz, int cout, const float* wd, int cin, float* dx, int64_t lddx,
                   int B, int H, int W, hipStream_t st);
// dw[co][tap][ci] = sum_pix dz[pix][co] * im2col(x)[pix][tap,ci]
void conv3x3_wgrad(const float* dz, int cout, const float* x, int64_t ldx, int xcoff, int cin, float* dw,
                   int B, int H, int W, float* slab, int64_t slab_cap, hipStream_t st);
// ConvTranspose2d(k2,s2): (B,H,W,cin) -> (B,2H,2W,cout) written at channel offset ycoff of rows ldy
void convT_fwd(const float* x, int64_t ldx, int cin, const float* wf, const float* bias, int cout,
               float* y, int64_t ldy, int ycoff, int B, int H, int W, hipStream_t st);
void convT_dgrad(const float* g, int64_t ldg, int gcoff, int cout, const float* wm, int cin, float* dx,
                 int B, int H, int W, hipStream_t st);
void convT_wgrad(const float* x, int cin, const float* g, int64_t ldg, int gcoff, int cout, float* dw,
                 int B, int H, int W, float* slab, int64_t slab_cap, hipStream_t st);
int64_t wgrad_slab_floats(int M, int N, int Kpix);

// ---- pre-split operands (gemm_ps.hpp): on the B1 engine, tensors written once as bf16 twins by
// their producer (or a split pass after it) and read by the B1 GEMMs without per-fetch conversion.
// A view: p = bf16 rows of `ld` channels (ld, coff, channel counts multiples of 8).
struct Split {
    const void* p = nullptr;
    int64_t ld = 0;
    int coff = 0;
};
int split_planes();                    // planes of the pre-split twins: 1 on B1, 0 otherwise (no twins)
constexpr int kMaxPlanes = 1;          // twin bytes = elems * 2 * kMaxPlanes
// out[row][ocoff + c] (split, ld ldo) = split(x[row][xcoff + c]), c < C, rows < M
void split_rows(const float* x, int64_t ldx, int xcoff, int C, int64_t M, void* out, int64_t ldo, int ocoff,
                hipStream_t st);
// y_bf16: y is written as bf16 rows of ldy elements (the bf16 engine's pre-BN outputs)
void conv3x3_fwd_ps(Split x, int cin, Split w, int cout, float* y, int64_t ldy, int ycoff, int B, int H, int W,
                    float* stats, hipStream_t st, bool y_bf16 = false);
// dx_bf16: dx is written as bf16 rows of lddx elements (the bf16 engine's conv2 input gradient).
// hi != nullptr: columns [split_n, cin) go to the bf16 rows hi (ldhi elements) instead of dx when the
// window kernel runs and split_n % 32 == 0 (returns true); otherwise all of dx is written as fp32
// (returns false)
// (with dx_bf16 as well: both halves bf16, dx rows of lddx elements; requires conv3x3_dgrad_split_ok)
bool conv3x3_dgrad_ps(Split dz, int cout, Split wd, int cin, float* dx, int64_t lddx, int B, int H, int W,
                      hipStream_t st, bool dx_bf16 = false, void* hi = nullptr, int64_t ldhi = 0, int split_n = 0);
bool conv3x3_dgrad_split_ok(Split dz, int cout, Split wd, int cin, int W, int split_n);
void conv3x3_wgrad_ps(Split dz, int cout, Split x, int cin, float* dw, int B, int H, int W, float* slab,
                      int64_t slab_cap, hipStream_t st);
// y_bf16: y is a bf16 twin (rows of ldy elements) — the up half of the decoder concat twin
void convT_fwd_ps(Split x, int cin, Split wf, const float* bias, int cout, float* y, int64_t ldy, int ycoff, int B,
                  int H, int W, hipStream_t st, bool y_bf16 = false);
// dx_bf16: dx written as bf16 rows of cin elements (the bf16 engine's decoder-input gradient)
void convT_dgrad_ps(Split g, int cout, Split wm, int cin, float* dx, int B, int H, int W, hipStream_t st,
                    bool dx_bf16 = false);
void convT_wgrad_ps(Split x, int cin, Split g, int cout, float* dw, int B, int H, int W, float* slab,
                    int64_t slab_cap, hipStream_t st);

// ---- dense GEMMs on the pre-split twins (the 1x1 / im2col convolutions of the config-5 network) ----
// y[m][ycoff + n] = sum_k x[m][k] w[n][k]  (+ BN partials [rows][2][N] when stats != nullptr)
// add != nullptr: y = x w^T + add (add rows with y's stride and offset; fp32 output, no stats)
// add: y = x w^T + add (fp32 y, rows as y's); mask (with add): then y = 0 where mask (fp32, rows as y's)
// is not > 0 — relu_mask of the sum, fused; ldadd: the added matrix's row stride (0: ldy; another stride
// takes no mask and no ycoff)
void dense_fwd_ps(Split x, int K, Split w, int N, float* y, int64_t ldy, int ycoff, int64_t M, float* stats,
                  hipStream_t st, bool y_bf16 = false, const float* add = nullptr, const float* mask = nullptr,
                  int64_t ldadd = 0);
// y[r][ycoff + c] = 0 where mask[r][ycoff + c] is not > 0 (rows of ldy; in place)
void mask_inplace(float* y, int64_t ldy, int ycoff, const float* mask, int C, int64_t M, hipStream_t st);
int dense_stats_rows(int64_t M, int N);
// dw[n][k] = sum_m dz[m][n] x[m][k]  (reduction over the M pixels; split-K slabs)
void dense_wgrad_ps(Split dz, int N, Split x, int K, float* dw, int64_t ldw, int64_t M, float* slab, int64_t slab_cap,
                    hipStream_t st);

// ---- MX-fp8 operands (gemm_mx8.hpp, mx8_kernels.hip): OCP MXFP8 E4M3 with one E8M0 scale per 32
// consecutive k elements, for the block-scaled MFMA.  q = element bytes [rows][ld], s = scale bytes
// [rows][ld / 32]; ld % 128 == 0, coff % 64 == 0 (the config-5 network's forward contractions).
struct Mx8 {
    const void* q = nullptr;
    const void* s = nullptr;
    int64_t ld = 0;
    int coff = 0;
};
// dst rows [coff, coff + C) = MX(src rows [scoff, scoff + C)), src fp32 (src_bf16 = false) or bf16
// rows of lds elements; C % 32 == 0
void mx8_quantize(const void* src, bool src_bf16, int64_t lds, int scoff, int C, int64_t M, Mx8 dst, hipStream_t st);
// fp32 weights [rows][C] -> MX (q rows of ldq bytes, coff 0; one e8m0 byte per 32), several tensors
// in one launch (the bits mx8_quantize writes for each)
struct Mx8WJob {
    const float* src;
    uint8_t* q;
    uint8_t* s;
    int64_t ldq;
    int rows, C;
    int blk0;   // first block of this job (filled by mx8_quantize_weights)
};
constexpr int kMx8WMaxJobs = 56;
struct Mx8WList {
    Mx8WJob job[kMx8WMaxJobs];
    int njobs = 0;
};
void mx8_quantize_weights(Mx8WList& list, hipStream_t st);
// y[m][ycoff + n] = sum_k x[m][k] w[n][k] on MX operands (+ BN partials when stats); K % 128 == 0
bool dense_x8_ok(int K, int N);
void dense_fwd_x8(Mx8 x, int K, Mx8 w, int N, float* y, int64_t ldy, int ycoff, int64_t M, float* stats, hipStream_t st,
                  bool y_bf16 = false);
int dense_x8_stats_rows(int64_t M, int N);
// window-tiled conv3x3 forward on MX operands; w rows [cout][9 cin] in (tap, ci) order
bool conv3x3_x8_ok(int cin, int W, int N);
void conv3x3_fwd_x8(Mx8 x, int cin, Mx8 w, int cout, float* y, int64_t ldy, int ycoff, int B, int H, int W,
                    float* stats, hipStream_t st, bool y_bf16 = false);
int conv3x3_x8_stats_rows(int cin, int B, int H, int W, int cout);

// ---------------- config-5 network kernels (res_kernels.hip) ----------------
// col[pix_out][k] bf16, k = (ky*KW + kx)*C + c, rows padded with zeros to Kp (% 8)
void im2col_f32(const float* x, int64_t ldx, int xcoff, int C, int B, int H, int W, int KH, int KW, int S, int P,
                void* col, int Kp, hipStream_t st);
void im2col_ps(Split x, int C, int B, int H, int W, int KH, int KW, int S, int P, void* col, int Kp, hipStream_t st);
// dx[pix_in][c] (overwritten, ld lddx) = sum of dcol[pix_out][tap*C + c] over the taps reading pix_in
void col2im(const float* dcol, int Kc, int C, int B, int H, int W, int KH, int KW, int S, int P, float* dx,
            int64_t lddx, hipStream_t st);
void maxpool3s2_fwd(const float* x, int C, int B, int H, int W, float* out, uint8_t* idx, void* out_split,
                    hipStream_t st);
// add (rows of ldadd, first C columns): a matrix added to the gathered gradient (config 5: the dec1 skip
// gradient of the stem output), else dx is overwritten
void maxpool3s2_bwd(const float* dout, const uint8_t* idx, int C, int B, int H, int W, float* dx, hipStream_t st,
                    const float* add = nullptr, int64_t ldadd = 0);
// out = relu(y*scale + shift + (yd ? yd*dscale + dshift : x)), fp32 [M][C] + twin
void bn_add_relu(const float* y, const float* scale, const float* shift, const float* yd, const float* dscale,
                 const float* dshift, const float* x, int64_t ldx, int C, int64_t M, float* out, void* out_split,
                 hipStream_t st, bool y_bf16 = false, const Mx8* qx = nullptr);
void relu_mask(const float* g, int64_t ldg, int gcoff, const float* out, int C, int64_t M, float* gs, hipStream_t st);
// dst[(b, S*oy, S*ox)][c] += src[(b, oy, ox)][scoff + c] over the strided grid of a B x H x W image
void add_strided(float* dst, int64_t lddst, const float* src, int64_t ldsrc, int scoff, int C, int B, int H, int W,
                 int S, hipStream_t st);
// twin rows dst[(b,oy,ox)][dcoff + c] = src[(b, S*oy, S*ox)][c]
void copy_twin(Split src, int C, int B, int H, int W, int S, void* dst, int64_t ldd, int dcoff, hipStream_t st);
// wt[k][n] = bf16(w[n][k])
void transpose_split(const float* w, int64_t ldw, int N, int K, void* wt, hipStream_t st);

// ---------------- NN elementwise / reductions (nn_kernels.hip) ----------------
// column partial sums: part[s][c] (double) over row slices; returns number of slices
int colsum_slices(int64_t R);
void colsum(const float* x, int64_t ld, int coff, int64_t R, int C, double* part, hipStream_t st);
// colsum of bf16 rows (x: bf16 elements, ld / coff in elements)
void colsum_bf16(const void* x, int64_t ld, int coff, int64_t R, int C, double* part, hipStream_t st);
void colsum_finalize(const double* part, int S, int C, float* dst, float scale, hipStream_t st);
// BatchNorm2d (train mode) from conv-epilogue partials [rows][2][C]
void bn_fwd_finalize(const float* tile_part, int rows, int C, int64_t count, const float* gamma,
                     const float* beta, float* run_mean, float* run_var, float momentum, float eps,
                     double* scratch, float* mean, float* invstd, float* scale, float* shift,
                     hipStream_t st);
// eval-mode BN coefficients from running statistics
void bn_eval_coeffs(const float* gamma, const float* beta, const float* run_mean, const float* run_var,
                    int C, float eps, float* mean, float* invstd, float* scale, float* shift, hipStream_t st);
// os != nullptr: also writes the output's pre-split twin (split rows of ldos channels at channel
// offset oscoff, split_planes() planes; see Split below)
// y_bf16: y holds bf16 values (conv outputs of the bf16 engine; also in bn_relu_bwd, film_*, bn_add_relu)
// qx != nullptr: also the MX-fp8 copy of the twin (C % 32 == 0, qx->ld % 128 == 0, coff 0; the
// bytes mx8_quantize would write from the twin)
void bn_relu_fwd(const float* y, int C, const float* scale, const float* shift, float* out, int64_t ldo,
                 int ocoff, int64_t M, hipStream_t st, void* os = nullptr, int64_t ldos = 0, int oscoff = 0,
                 bool y_bf16 = false, const Mx8* qx = nullptr);
// BN+ReLU backward: dy = k1*dz - k2 - k3*xhat, dz = g*[y*scale+shift > 0];
// writes dgamma/dbeta (grad buffer) and dy (dense [M][C]).  gmul != nullptr: g is first multiplied
// by gmul[sample][c] (sample = row / HW) — the FiLM gamma sitting between this ReLU and the consumer.
// dy_split != nullptr: also the pre-split twin of dy (dense, ld C).  relu = false: plain BN backward
// (dz = g; the bottleneck's last BN, whose ReLU sits after the residual add)
// head != nullptr: g is the depth head's input gradient dp[r] * w[c] rebuilt per row (g, gmul null)
struct HeadGrad {
    const float* dpred = nullptr;
    const float* sig = nullptr;
    const float* w = nullptr;
    float md = 0.f;
};
// pool != nullptr: the max-pool backward folded in — g[r][c] += d[pooled r][c] where r is the
// recorded argmax of its 2x2 window (idx, scan order 0..3), instead of a scatter into g beforehand;
// H, W: g's image size (r < 2^32)
// unsigned 32-bit division by an invariant d >= 2 (Granlund-Montgomery: q = (t + ((n - t) >> 1)) >> s,
// t = mulhi(m, n); exact for every 32-bit n)
struct FastDiv {
    uint32_t m = 0;
    int s1 = 0, s2 = 0;
};
// n / d = (t + ((n - t) >> s1)) >> s2 with t = mulhi(m, n), l = ceil(log2 d): s1 = 1, s2 = l - 1 for
// d >= 2; d = 1 gives m = 1, t = 0 and s1 = s2 = 0 (a 1x1 image: sample = row)
inline FastDiv make_fastdiv(uint32_t d) {
    int l = 0;
    while ((1ull << l) < d) ++l;   // ceil(log2 d)
    FastDiv f;
    f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    f.s1 = l > 0 ? 1 : 0;
    f.s2 = l > 0 ? l - 1 : 0;
    return f;
}
__device__ __forceinline__ uint32_t fdiv(const FastDiv& f, uint32_t n) {
    const uint32_t t = __umulhi(f.m, n);
    return (t + ((n - t) >> f.s1)) >> f.s2;
}
struct PoolAdd {
    const float* d = nullptr;
    const uint8_t* idx = nullptr;
    int H = 0, W = 0;
    FastDiv divW, divH;   // set by bn_relu_bwd
};
void bn_relu_bwd(const float* g, int64_t ldg, int gcoff, const float* y, int C, const float* mean,
                 const float* invstd, const float* scale, const float* shift, const float* gamma,
                 int64_t M, double* scratch, float* coef, float* dgamma, float* dbeta, float* dy,
                 hipStream_t st, const float* gmul = nullptr, int64_t HW = 1, void* dy_split = nullptr,
                 bool relu = true, bool y_bf16 = false, const HeadGrad* head = nullptr, bool g_bf16 = false,
                 const PoolAdd* pool = nullptr, float* film_dgam = nullptr, float* film_dbet = nullptr,
                 const double* tile_part = nullptr, int tiles = 0);
// (tile_part: the column sums were already formed per tile by the producing GEMM's epilogue —
// conv3x3_dgrad_*_bnsums, [tiles][2][C] — and are only reduced over tiles here)
// out_split != nullptr: also the pooled output's split twin (dense, ld C); out may then be nullptr
// x_bf16: x is a bf16 twin (rows of ldx elements; requires out_split)
void maxpool_fwd(const float* x, int64_t ldx, int C, int B, int H, int W, float* out, uint8_t* idx,
                 hipStream_t st, void* out_split = nullptr, bool x_bf16 = false);
// BatchNorm-backward column sums taken in a conv input-gradient epilogue (EpiStoreBnSums): the BN
// input y (rows of ldy, bf16 or fp32) and its coefficients; per-tile fp64 partials [tiles][2][N] into
// part (capacity part_cap doubles)
struct BnSums {
    const void* y = nullptr; int64_t ldy = 0; bool y_bf16 = false;
    const float *mean = nullptr, *invstd = nullptr, *scale = nullptr, *shift = nullptr;
    double* part = nullptr; int64_t part_cap = 0;
};
// conv3x3 input gradient (S3 engine, fp32 dx) whose window epilogue also forms bn's backward sums over
// dx: returns the tile count (0 = not available for this shape: nothing launched)
int conv3x3_dgrad_bnsums(const float* dz, int cout, const float* wd, int cin, float* dx, int64_t lddx, int B, int H,
                         int W, const BnSums& bn, hipStream_t st);
// an encoder block's bn2 + ReLU fused with the next level's MaxPool2d(2): writes the block output
// (fp32 rows `out` (ldo) and/or its 1-plane twin `os` (ldos), channel offset 0) and the pooled output
// (fp32 `pool` and/or its twin `pool_split`, dense ld C) with the argmax codes, exactly what
// bn_relu_fwd followed by maxpool_fwd writes (the bf16 engine pools the twin's values)
void bn_relu_pool_fwd(const float* y, int C, const float* scale, const float* shift, float* out, int64_t ldo,
                      void* os, int64_t ldos, int B, int H, int W, bool y_bf16, float* pool, uint8_t* idx,
                      void* pool_split, hipStream_t st);
void maxpool_bwd(const float* dout, const uint8_t* idx, int C, int B, int H, int W, float* dx,
                 int64_t lddx, hipStream_t st);
void rgb_to_nhwc4(const float* rgb, float* out, int B, int H, int W, hipStream_t st);
void rgb_to_nhwc8(const float* rgb, float* out, int B, int H, int W, hipStream_t st);
void head_fwd(const float* a, int C, const float* w, const float* b, float max_depth, float* sig,
              float* pred, int64_t M, hipStream_t st);
void head_bwd(const float* a, int C, const float* w, const float* dpred, const float* sig,
              float max_depth, float* da, int64_t M, double* scratch, float* dw, float* db,
              hipStream_t st);
// level-0 fusion: BN apply + ReLU + head in one pass (relu(y*scale+shift) is never stored; sig / pred
// bit-identical to bn_relu_fwd + head_fwd) and the head weight/bias gradient from y (no stored
// activation); head_fusable: C / 4 a power of two <= 32
bool head_fusable(int C);
void bn_relu_head_fwd(const float* y, int C, const float* scale, const float* shift, const float* w, const float* b,
                      float max_depth, float* sig, float* pred, int64_t M, hipStream_t st, bool y_bf16);
void head_bwd_y(const float* y, int C, const float* scale, const float* shift, const float* dpred, const float* sig,
                float max_depth, int64_t M, double* scratch, float* dw, float* db, hipStream_t st, bool y_bf16);
// computeDepthMetrics partial sums per (sample, block): {n, |d|/g, d^2/g, d^2, dlog^2, a1, a2, a3}
int metrics_blocks(int64_t HW);
void depth_metrics_partials(const float* pred, const float* gt, int B, int64_t HW, double* part, int nb,
                            hipStream_t st);
void repack_conv_dgrad(const float* w, float* wd, int cout, int cin, hipStream_t st);
void repack_convT_fwd(const float* wm, float* wf, int cin, int cout, hipStream_t st);
// Per-step weight preparation in one launch (the weights change every step): a list of jobs, each
// one weight tensor ->  fp32 repack (d32, optional) and/or its bf16 twin (d16, optional; the
// k_split_rows<1> rounding).  Kinds: WPREP_SPLIT  [rows][K] -> bf16 same layout;
// WPREP_DGRAD  OHWI [co][tap][ci] -> [ci][8 - tap][co] (repack_conv_dgrad);
// WPREP_CONVT  [ci][q][co] -> [q][co][ci] (repack_convT_fwd);
// WPREP_TRANSPOSE [cout][cin] -> [cin][cout] (transpose_split: N = cout rows of K = cin).
// n = elements, a multiple of 8.
enum { WPREP_SPLIT = 0, WPREP_DGRAD = 1, WPREP_CONVT = 2, WPREP_TRANSPOSE = 3 };
struct WPrepJob {
    const float* src;
    float* d32;
    void* d16;
    int kind, cout, cin;
    int blk0;   // first block of this job (filled by weight_prep)
    int64_t n;
};
constexpr int kWPrepMaxJobs = 24;
struct WPrepList {
    WPrepJob job[kWPrepMaxJobs];
    int njobs;
};
void weight_prep(WPrepList& list, hipStream_t st);

// ---------------- losses (loss_kernels.hip) ----------------
struct LossWorkspace {
    double* part;        // partial sums
    float* scal;         // scalars: see loss_kernels.hip
    float* pyr;          // log-pooled pyramid (pred, gt) for scales 1..3
    int64_t part_cap;
};
int64_t loss_workspace_floats(int B, int H, int W);
int64_t loss_part_doubles(int B, int H, int W);
// total/components -> out[5] = {total, si, grad, smooth, reproj}; dpred = dL/dpred.  mask (nullable,
// B*H*W bytes, nonzero = valid) replaces gt > eps in the SI and reprojection terms (valid_mask)
void loss_fwd_bwd(const float* pred, const float* gt, const float* rgb, const float* K, const uint8_t* mask, int B,
                  int H, int W, const float w[4], float* out5, float* dpred, LossWorkspace ws, hipStream_t st);

// ---------------- optimizer (optim_kernels.hip) ----------------
int sumsq_blocks(int64_t n);
void grad_norm_clip(const float* g, int64_t n, float max_norm, float prescale, double* scratch,
                    float* norm_coef, hipStream_t st);
void adam_step(float* p, float* g, float* m, float* v, int64_t n, const float* norm_coef, float lr,
               float b1, float b2, float eps, float wd, int step, hipStream_t st);

// ---------------- batch assembly (batch_kernels.hip) ----------------
// One decoded sample and what the loader does to it (sunrgbd_loader.cpp resizeSample / augmentSample);
// an array of these lives in device memory for the launch.
struct BatchSample {
    const uint8_t* rgb;      // HWC u8, h0 x w0 x 3 (bgr = 1: OpenCV channel order)
    const uint16_t* depth;   // HW u16, dh0 x dw0
    int h0, w0, bgr;
    int dh0, dw0;
    float depth_scale;       // metres per depth unit (1/1000)
    int aug;                 // 0: output = stage 1 (resize); 1: crop / flip / jitter / resize of stage 1
    int cy, cx, ch, cw;      // crop window of the H x W stage-1 image (already clamped to it)
    int flip, jitter;
    float contrast, brightness;
};
void batch_assemble(const BatchSample* samples_dev, int B, int H, int W, bool any_aug, float* rgb, float* depth,
                    float* rgb_tmp, float* depth_tmp, hipStream_t st);

// ---------------- conditioning (cond_kernels.hip, film_kernels.hip) ----------------
void ray_directions(const float* K, int B, int H, int W, float* rays_nchw, hipStream_t st);
void camera_from_K(const float* K, int B, float* cam4, hipStream_t st);            // a15
void camera_normalize(const float* cam4, int B, int H, int W, float* camn, hipStream_t st);   // a14
// a19 input: NHWC8 [r, g, b, ray_x, ray_y, ray_z, 0, 0] with rays from cam4 (a18)
void rgb_rays_to_nhwc8(const float* rgb, const float* cam4, int B, int H, int W, float* out, hipStream_t st);

// One FiLMLayerImpl (film_layer.h:26-108): parameters, running stats, saved activations, grads.
constexpr int kFilmH1 = 128, kFilmH2 = 256;
struct FilmLayer {
    int C = 0;
    const float *w1, *b1, *w2, *b2, *wg, *bg, *wb, *bb, *g1, *be1, *g2, *be2;   // parameters
    float *rm1, *rv1, *rm2, *rv2;                                              // BatchNorm1d buffers
    float *xh1, *h1, *xh2, *h2, *is1, *is2;   // [B][128] / [B][256] xhat + relu outputs, invstd
    float *gam, *bet;                         // [B][C]
    float *dgam, *dbet, *dh2, *dh1;           // backward scratch
    float *gw1, *gb1, *gw2, *gb2, *gwg, *gbg, *gwb, *gbb, *gg1, *gbe1, *gg2, *gbe2;   // gradients
};
void film_mlp_fwd(const FilmLayer& L, const float* camn, int B, bool train, hipStream_t st);
// every layer's MLP forward in four launches (they depend on the camera only): the same per-layer
// arithmetic as film_mlp_fwd
constexpr int kFilmMaxLayers = 10;
struct FilmList {
    FilmLayer l[kFilmMaxLayers];
    int n = 0;
};
void film_mlp_fwd_all(const FilmList& list, const float* camn, int B, bool train, hipStream_t st);
void film_mlp_bwd(const FilmLayer& L, const float* camn, int B, hipStream_t st);
// a1 = gam[b,c] * relu(y*scale[c] + shift[c]) + bet[b,c]   (NHWC [B*HW][C]); out (fp32, may be null)
// and / or os (its bf16 twin, rows of C; the B1 engine's operand)
void film_apply(const float* y, int C, const float* scale, const float* shift, const float* gam, const float* bet,
                int B, int64_t HW, float* out, hipStream_t st, bool y_bf16 = false, void* os = nullptr);
// dgam[b,c] = sum_hw dA * relu(y*scale+shift), dbet[b,c] = sum_hw dA
void film_affine_bwd(const float* dA, const float* y, int C, const float* scale, const float* shift, int B, int64_t HW,
                     double* scratch, float* dgam, float* dbet, hipStream_t st, bool y_bf16 = false,
                     bool dA_bf16 = false);
int64_t film_reduce_doubles(int B, int64_t HW, int C);

// ---------------- geometry-aware family (attn_kernels.hip) ----------------
// GeometryAwareNetwork input: NHWC8 [r g b rx ry rz 0 0] from NCHW rgb and NCHW rays
void pack_rgb_rays(const float* rgb, const float* rays, int B, int H, int W, float* out, hipStream_t st);
// per-(sample, channel) mean over H*W of x[(b*HW + r)*ldx + xcoff + c] -> avg [B][C]; with mx != nullptr
// also the max and its first-occurrence pixel index (amax, within the sample)
int chan_pool_slices(int64_t HW);
void chan_pool(const float* x, int64_t ldx, int xcoff, int C, int B, int64_t HW, double* part, float* avg, float* mx,
               int* amax, hipStream_t st);
int64_t attn_scratch_doubles(int B, int64_t HW, int C);   // scratch of cbam_* / pcl_* at one level

// One CBAMImpl (spatial_attention.h:142-191): parameters, saved forward state, gradients, scratch.
struct Cbam {
    int C = 0, Cr = 0;   // Cr = max(1, C / 16)
    const float *w1, *b1, *w2, *b2, *wsp;   // channel_attention.fc1 [Cr][C], fc2 [C][Cr]; spatial conv [2][7][7]
    float *gw1, *gb1, *gw2, *gb2, *gwsp;
    float *avg, *mx;          // [B][C] pooled vectors
    int* amax;                // [B][C] argmax pixel of mx
    float *ha, *hm;           // [B][Cr] relu(fc1(.)) of the avg / max branch
    float* att;               // [B][C] channel attention
    float* s;                 // [M][2] channel mean / max of x*att
    int* sidx;                // [M] argmax channel
    float* sa;                // [M] spatial attention
    float *dlog, *ds;         // backward: [M] conv-logit grad, [M][2] grad of s
    float *dO, *dha, *dhm, *dva, *dvm;   // [B][C], [B][Cr], [B][Cr], [B][C], [B][C]
};
// out (rows of ldo, channel offset ocoff) = CBAM(x), x dense [B*H*W][C]
void cbam_fwd(const Cbam& A, const float* x, int B, int H, int W, float* out, int64_t ldo, int ocoff, double* scratch,
              hipStream_t st);
// dx (dense) = d CBAM / dx given g = grad of the output; writes the parameter gradients
void cbam_bwd(const Cbam& A, const float* x, const float* g, int64_t ldg, int gcoff, int B, int H, int W, float* dx,
              double* scratch, hipStream_t st);

// One PerspectiveCorrectionLayerImpl (pcl_layer.h:29-181, hidden 128)
constexpr int kPclHidden = 128;
struct Pcl {
    int C = 0;
    const float *w1, *b1, *w2, *b2, *w3, *b3;   // loc_fc1 [128][C+4], loc_fc2 [128][128], fc_transform [6][128]
    float *gw1, *gb1, *gw2, *gb2, *gw3, *gb3;
    float* pooled;            // [B][C]
    float *h1, *h2;           // [B][128]
    float *tp, *theta;        // [B][6] transform parameters, affine matrix (row-major 2x3)
    float* dgrid;             // [M][2]
    float *dtp, *dh1, *dh2, *dpooled;   // [B][6], [B][128], [B][128], [B][C]
};
// out (rows of ldo, channel offset ocoff) = PCL(u, camn), u dense [B*H*W][C]
void pcl_fwd(const Pcl& P, const float* u, const float* camn, int B, int H, int W, float* out, int64_t ldo, int ocoff,
             double* scratch, hipStream_t st);
// du (dense, overwritten) = d PCL / du given g = grad of the output; writes the parameter gradients
void pcl_bwd(const Pcl& P, const float* u, const float* camn, const float* g, int64_t ldg, int gcoff, int B, int H,
             int W, float* du, double* scratch, hipStream_t st);

}  // namespace cad
