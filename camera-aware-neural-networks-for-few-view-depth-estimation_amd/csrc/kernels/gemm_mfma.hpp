// fp32 MFMA implicit-GEMM engine for gfx950 (CDNA4).
//
// One engine covers every contraction on the U-Net hot path:
//   conv3x3 fwd      C[pix][co]      = sum_{tap,ci} im2col(X)[pix][tap,ci] * W[co][tap,ci]
//   conv3x3 dgrad    C[pix][ci]      = sum_{tap,co} im2col(dZ)[pix][tap,co] * Wd[ci][tap,co]
//   conv3x3 wgrad    C[co][tap,ci]   = sum_pix dZ[pix][co] * im2col(X)[pix][tap,ci]      (split-K)
//   convT2x2 fwd     C[pix][q,co]    = sum_ci X[pix][ci] * Wf[q,co][ci]   (pixel-shuffle store)
//   convT2x2 dgrad   C[pix][ci]      = sum_{q,co} up(G)[pix][q,co] * Wm[ci][q,co]
//   convT2x2 wgrad   C[ci][q,co]     = sum_pix X[pix][ci] * up(G)[pix][q,co]             (split-K)
// C[m][n] = sum_k A(m,k) * B(n,k).  Activations are NHWC fp32 (channel-contiguous rows, optional
// row stride/channel offset so the decoder concat buffer is written/read in place).
//
// Tile: 4 waves (256 threads) = WM x WN waves, each wave owns 64x64 = 2x2 blocks of
// v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chains, 64 FLOP/clk/SIMD = the fp32 peak). The K-stage
// depth KB (16 or 32) is a template parameter chosen per tile shape by the host launchers.
// Operand staging is register-staged double-buffered LDS, one barrier per K-stage.
//   "Kc"  operands (global rows are contiguous along k): LDS image [rows][KB+4] (row stride 80 B /
//         144 B: consecutive rows hit distinct 16-B bank slots -> conflict-free ds_read_b128).
//   "MNc" operands (global rows are contiguous along m/n, k = pixel is strided): LDS image
//         [KB][rows] read with one ds_read_b32 per MFMA step (32 consecutive lanes, no conflict).
// K order inside a stage is permuted so a lane's 8 k-values are contiguous: MFMA step s, lane half h
// consumes chunk-k = (KB/2)h + s (both operands use the same map, so the sum is unchanged).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace cad {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// K-stage geometry for stage depth KB (16 or 32)
template <int KB>
struct KS {
    static_assert(KB == 16 || KB == 32, "K-stage depth");
    static constexpr int BK = KB;
    static constexpr int LDK = KB + 4;        // Kc LDS row stride (floats), conflict-free b128
    static constexpr int TPR = KB / 4;        // threads per Kc row (one float4 each)
    static constexpr int RPP = 256 / TPR;     // Kc rows staged per pass of the workgroup
    static constexpr int HK = KB / 2;         // MFMA steps per stage = k values per lane half
};

struct GemmArgs {
    int M, N, K;          // GEMM extents
    // geometry of the pixel grid the gathers walk (low-res grid for convT ops)
    int B, H, W;
    // operand A
    const float* A; int64_t lda; int a_coff; int a_cin;   // a_cin: channels per tap / per quadrant
    // operand B
    const float* Bm; int64_t ldb; int b_coff; int b_cin;
    // output
    float* C; int64_t ldc; int c_coff;
    const float* bias;
    float* stats;         // BN partials [gridDim.x][2][N] (sum, M2 about the tile mean) + [gridDim.x] counts, or nullptr
    int kstages_per_split;
    int64_t slab_stride;  // elements between split-K slabs
    // conv3x3 forward/dgrad on pre-split operands: K stages in channel-major order (stage s = tap
    // s % 9 of channel block s / 9, KB channels per block) instead of tap-major, so the nine taps of
    // a channel block re-read the same input rows back to back (L2 hits) — needs cin % KB == 0
    int cimajor;
    // split store (EpiStoreSplitB16): output columns n >= split_n go to the bf16 rows C2 (ldc2 elements,
    // column n - split_n) instead of C
    void* C2; int64_t ldc2; int split_n;
    // BatchNorm epilogues of a recomputed convolution (EpiBnRelu / EpiBnBwdSums / EpiBnBwdApply,
    // epilogues.hpp): the BN's per-channel coefficients, the upstream gradient (bf16 or fp32 rows of
    // bn_ldg elements) and the per-tile fp64 partials [gridDim.x][2][N]
    const float *bn_scale, *bn_shift, *bn_mean, *bn_invstd, *bn_coef;
    const void* bn_g; int64_t bn_ldg;
    double* bn_part;
};


// --------------------------------------------------------------------------------------------
// Operand fetch: buffer loads against a per-workgroup base.  Every loader builds ONE buffer
// descriptor from wave-uniform values (kernel arguments and the tile's block-derived origin), so the
// per-lane part of an address is a 32-bit byte offset from that base.  An element that lies outside
// the operand (image border of the 3x3 gather, M/N/K tails) gets the offset kOOB: the hardware range
// check returns zeros for it, so the loaders have no branches and no selects around their loads.
// A block's window (its rows plus the 3x3 halo, or its K-slice of pixels) is far below 2 GB; the
// host launchers keep it so (conv_kernels.hip: plan_splits).
// --------------------------------------------------------------------------------------------
constexpr uint32_t kOOB = 0x80000000u;
constexpr uint32_t kRecords = 0x7FFFFFF0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, uint32_t records = kRecords) {
    // readfirstlane: make the uniformity of the descriptor provable to the compiler
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, __builtin_amdgcn_readfirstlane(records), 0x00020000);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// --------------------------------------------------------------------------------------------
// Kc loaders: operand(row r, k) with k contiguous in memory.  Thread t owns rows t/TPR + RPP*j and
// the float4 column group (t%TPR)*4 of every stage.
//
// Loader protocol: init(..., kbeg) positions the loader at K-stage kbeg; load(v) issues the next
// stage's global loads into registers; finish(v) (called right before the LDS store) completes any
// register-side transform.
// --------------------------------------------------------------------------------------------
template <int ROWS, int KB>
struct KcDense {   // op(r,k) = P[r*ld + coff + k], r < nrows, k < K
    using G = KS<KB>;
    static constexpr int NV = ROWS / G::RPP;
    __amdgpu_buffer_rsrc_t rs;
    uint32_t roff[NV];   // byte offset of the thread's row from the block base (kOOB: row out of range)
    int K, k;
    __device__ void init(const float* P, int64_t ld, int coff, int nrows, int K_, int row0, int tid, int kbeg) {
        K = K_;
        k = kbeg * KB + (tid % G::TPR) * 4;
        rs = make_rsrc(P + (int64_t)row0 * ld + coff);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int rr = tid / G::TPR + G::RPP * j;
            roff[j] = row0 + rr < nrows ? (uint32_t)(rr * ld * 4) : kOOB;
        }
    }
    __device__ void load(float4 (&v)[NV]) {
        const bool kin = k < K;
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = bload4(rs, kin ? roff[j] + (uint32_t)k * 4 : kOOB);
        k += KB;
    }
    __device__ void finish(float4 (&)[NV]) {}
};

// (tap, ci) of a thread's float4 column, carried incrementally across K-stages of KB
template <int KB>
__device__ __forceinline__ void tapci_advance(int& tap, int& ci, int cin) {
    ci += KB;
    if (cin >= KB) {   // uniform: at most one wrap per stage, branch-free
        const bool w = ci >= cin;
        ci -= w ? cin : 0;
        tap += w;
    } else {
        while (ci >= cin) { ci -= cin; ++tap; }
    }
}

// op(pix, k=(tap,ci)) = X[(b, y+ky-1, x+kx-1)*ld + coff + ci], zero outside the image.
template <int ROWS, int KB>
struct KcIm2col3x3 {
    using G = KS<KB>;
    static constexpr int NV = ROWS / G::RPP;
    __amdgpu_buffer_rsrc_t rs;
    int ld4;           // row stride in bytes
    uint32_t poff[NV]; // byte offset of the thread's pixel from the block base
    int y[NV], x[NV];
    bool ok[NV];
    int H, W, cin, tap, ci;
    __device__ void init(const float* P, int64_t ld_, int coff, int cin_, int B, int H_, int W_,
                         int row0, int tid, int kbeg) {
        H = H_; W = W_; cin = cin_; ld4 = (int)ld_ * 4;
        const int pb = max(row0 - W_ - 1, 0);   // first pixel of the block's halo window
        rs = make_rsrc(P + (int64_t)pb * ld_ + coff);
        const int k = kbeg * KB + (tid % G::TPR) * 4;
        tap = k / cin;
        ci = k - tap * cin;
        const int M = B * H * W;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int r = row0 + tid / G::TPR + G::RPP * j;
            ok[j] = r < M;
            const int rr = ok[j] ? r : 0;
            x[j] = rr % W;
            y[j] = (rr / W) % H;
            poff[j] = (uint32_t)((rr - pb) * ld4);
        }
    }
    __device__ void load(float4 (&v)[NV]) {
        const bool kin = tap < 9;
        const int t = kin ? tap : 0;
        const int dy = t / 3 - 1, dx = t - 3 * (t / 3) - 1;
        const int off = (dy * W + dx) * ld4 + ci * 4;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int yy = y[j] + dy, xx = x[j] + dx;
            const bool g = ok[j] && kin && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            v[j] = bload4(rs, g ? poff[j] + (uint32_t)off : kOOB);
        }
        tapci_advance<KB>(tap, ci, cin);
    }
    __device__ void finish(float4 (&)[NV]) {}
};

// op(lowres pix (b,y,x), k=(q=(dy,dx), co)) = G[(b, 2y+dy, 2x+dx)*ld + coff + co]
template <int ROWS, int KB>
struct KcUpGather {
    using G = KS<KB>;
    static constexpr int NV = ROWS / G::RPP;
    __amdgpu_buffer_rsrc_t rs;
    int ld4;
    uint32_t hoff[NV];   // byte offset of high-res pixel (2y, 2x) from the block base (kOOB: row out of range)
    int W2, cout, q, co;
    __device__ void init(const float* P, int64_t ld_, int coff, int cout_, int B, int H, int W,
                         int row0, int tid, int kbeg) {
        ld4 = (int)ld_ * 4; cout = cout_; W2 = 2 * W;
        const int k = kbeg * KB + (tid % G::TPR) * 4;
        q = k / cout;
        co = k - q * cout;
        const int M = B * H * W;
        auto hr = [&](int r) {
            const int xx = r % W, t = r / W, yy = t % H, b = t / H;
            return ((int64_t)b * (2 * H) + 2 * yy) * W2 + 2 * xx;
        };
        const int64_t hb = hr(min(row0, M - 1));
        rs = make_rsrc(P + hb * ld_ + coff);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int r = row0 + tid / G::TPR + G::RPP * j;
            hoff[j] = r < M ? (uint32_t)((hr(r) - hb) * ld4) : kOOB;
        }
    }
    __device__ void load(float4 (&v)[NV]) {
        const bool kin = q < 4;
        const int qq = kin ? q : 0;
        const uint32_t off = (uint32_t)(((qq >> 1) * W2 + (qq & 1)) * ld4 + co * 4);
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = bload4(rs, kin && hoff[j] != kOOB ? hoff[j] + off : kOOB);
        tapci_advance<KB>(q, co, cout);
    }
    __device__ void finish(float4 (&)[NV]) {}
};

// --------------------------------------------------------------------------------------------
// MNc loaders: operand(row r, k=pixel); memory rows are pixels, contiguous along r.
// Thread t owns row group cg = t % (ROWS/4) (4 rows) and k-rows t/(ROWS/4) + KSTEP*j.  The block's
// base is the first pixel of its K-slice (minus the 3x3 halo for the gather).
// --------------------------------------------------------------------------------------------
template <int ROWS, int KB>
struct MNcBase {
    static constexpr int TPR = ROWS / 4;          // threads per k-row
    static constexpr int KSTEP = 256 / TPR;       // k-rows per pass
    static constexpr int NV = KB / KSTEP;
};

// The MNc loaders walk pixels: each thread's k-rows advance by KB pixels per stage, so (x, y) is
// carried incrementally (one compare-subtract per stage for W >= KB) instead of dividing per stage.
template <int KB>
__device__ __forceinline__ void px_advance(int& x, int& y, int& b, int W, int H) {
    x += KB;
    while (x >= W) {
        x -= W;
        if (++y == H) { y = 0; ++b; }
    }
}

template <int ROWS, int KB>
struct MNcDense : MNcBase<ROWS, KB> {   // op(r, k) = P[k*ld + coff + r], r < nrows, k < Kp
    using Base = MNcBase<ROWS, KB>;
    static constexpr int NV = Base::NV;
    __amdgpu_buffer_rsrc_t rs;
    uint32_t koff;   // byte offset of the thread's k-row 0 (advances KB rows per stage)
    int ld4, Kp, k0;
    bool rok;
    __device__ void init(const float* P, int64_t ld_, int coff, int nrows, int Kp_, int row0, int tid, int kbeg) {
        ld4 = (int)ld_ * 4; Kp = Kp_;
        const int r = row0 + (tid % Base::TPR) * 4;
        rok = r < nrows;   // nrows % 4 == 0 is required
        const int kb0 = kbeg * KB;
        rs = make_rsrc(P + (int64_t)kb0 * ld_ + coff + row0);
        k0 = kb0 + tid / Base::TPR;
        koff = (uint32_t)((tid / Base::TPR) * ld4 + (tid % Base::TPR) * 16);
    }
    __device__ void load(float4 (&v)[NV]) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int k = k0 + Base::KSTEP * j;
            v[j] = bload4(rs, rok && k < Kp ? koff + (uint32_t)(Base::KSTEP * j * ld4) : kOOB);
        }
        k0 += KB;
        koff += (uint32_t)(KB * ld4);
    }
    __device__ void finish(float4 (&)[NV]) {}
};

// op(j=(tap,ci), k=pix) = X[(b,y+ky-1,x+kx-1)*ld + coff + ci]
template <int ROWS, int KB>
struct MNcIm2col3x3 : MNcBase<ROWS, KB> {
    using Base = MNcBase<ROWS, KB>;
    static constexpr int NV = Base::NV;
    __amdgpu_buffer_rsrc_t rs;
    int ld4, H, W, Kp, dy, dx, pb;
    int tapoff;        // byte offset of the thread's (tap, ci) relative to its pixel
    int k[NV], x[NV], y[NV];
    bool rok;
    __device__ void init(const float* P, int64_t ld_, int coff, int cin, int B, int H_, int W_,
                         int row0, int tid, int kbeg) {
        ld4 = (int)ld_ * 4; H = H_; W = W_; Kp = B * H_ * W_;
        const int j = row0 + (tid % Base::TPR) * 4;
        rok = j < 9 * cin;
        const int jj = rok ? j : 0;
        const int tap = jj / cin, ci = jj - tap * cin;
        dy = tap / 3 - 1; dx = tap % 3 - 1;
        pb = max(kbeg * KB - W_ - 1, 0);
        rs = make_rsrc(P + (int64_t)pb * ld_ + coff);
        tapoff = (dy * W + dx) * ld4 + ci * 4;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            k[i] = kbeg * KB + tid / Base::TPR + Base::KSTEP * i;
            const int kk = k[i] < Kp ? k[i] : 0;
            x[i] = kk % W;
            y[i] = (kk / W) % H;
        }
    }
    __device__ void load(float4 (&v)[NV]) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int yy = y[j] + dy, xx = x[j] + dx;
            const bool g = rok && k[j] < Kp && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            v[j] = bload4(rs, g ? (uint32_t)((k[j] - pb) * ld4 + tapoff) : kOOB);
            int b = 0;
            px_advance<KB>(x[j], y[j], b, W, H);
            k[j] += KB;
        }
    }
    __device__ void finish(float4 (&)[NV]) {}
};

// op(j=(q,co), k=lowres pix (b,y,x)) = G[(b,2y+dy,2x+dx)*ld + coff + co]
template <int ROWS, int KB>
struct MNcUpGather : MNcBase<ROWS, KB> {
    using Base = MNcBase<ROWS, KB>;
    static constexpr int NV = Base::NV;
    __amdgpu_buffer_rsrc_t rs;
    int64_t hb;          // high-res pixel of the block base
    int ld4, H, W, Kp, qy, qx, cooff;
    int k[NV], x[NV], y[NV], b[NV];
    bool rok;
    __device__ void init(const float* P, int64_t ld_, int coff, int cout, int B, int H_, int W_,
                         int row0, int tid, int kbeg) {
        ld4 = (int)ld_ * 4; H = H_; W = W_; Kp = B * H_ * W_;
        const int j = row0 + (tid % Base::TPR) * 4;
        rok = j < 4 * cout;
        const int jj = rok ? j : 0;
        const int q = jj / cout, co = jj - q * cout;
        qy = q >> 1; qx = q & 1;
        cooff = co * 4;
        {   // block base: high-res pixel (2y, 2x) of the slice's first low-res pixel
            const int kk = min(kbeg * KB, Kp - 1);
            const int xx = kk % W, t = kk / W, yy = t % H, bb = t / H;
            hb = ((int64_t)bb * (2 * H) + 2 * yy) * (2 * W) + 2 * xx;
        }
        rs = make_rsrc(P + hb * ld_ + coff);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            k[i] = kbeg * KB + tid / Base::TPR + Base::KSTEP * i;
            const int kk = k[i] < Kp ? k[i] : 0;
            x[i] = kk % W;
            const int t = kk / W;
            y[i] = t % H;
            b[i] = t / H;
        }
    }
    __device__ void load(float4 (&v)[NV]) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const bool g = rok && k[j] < Kp;
            const int64_t hp = ((int64_t)b[j] * (2 * H) + 2 * y[j] + qy) * (2 * W) + 2 * x[j] + qx;
            v[j] = bload4(rs, g ? (uint32_t)((hp - hb) * ld4 + cooff) : kOOB);
            px_advance<KB>(x[j], y[j], b[j], W, H);
            k[j] += KB;
        }
    }
    __device__ void finish(float4 (&)[NV]) {}
};

// --------------------------------------------------------------------------------------------
// LDS staging + fragment reads
// --------------------------------------------------------------------------------------------
template <int ROWS, int KB, int NV>
__device__ __forceinline__ void kc_store(float* s, const float4 (&v)[NV]) {
    using G = KS<KB>;
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NV; ++j)
        *reinterpret_cast<float4*>(s + (t / G::TPR + G::RPP * j) * G::LDK + (t % G::TPR) * 4) = v[j];
}
template <int ROWS, int KB, int NV>
__device__ __forceinline__ void mnc_store(float* s, const float4 (&v)[NV]) {   // KB: same signature as kc_store
    constexpr int TPR = ROWS / 4, KSTEP = 256 / TPR;
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NV; ++j)
        *reinterpret_cast<float4*>(s + (t / TPR + KSTEP * j) * ROWS + (t % TPR) * 4) = v[j];
}
// fragment: HK consecutive chunk-k values of row (rb + lane&31), half h = lane>>5
template <int KB>
__device__ __forceinline__ void kc_frag(const float* s, int rb, float (&f)[KS<KB>::HK]) {
    using G = KS<KB>;
    const int lane = threadIdx.x & 63;
    const float* q = s + (rb + (lane & 31)) * G::LDK + (lane >> 5) * G::HK;
#pragma unroll
    for (int i = 0; i < G::HK; i += 4) {
        float4 a = *reinterpret_cast<const float4*>(q + i);
        f[i] = a.x; f[i + 1] = a.y; f[i + 2] = a.z; f[i + 3] = a.w;
    }
}
template <int ROWS, int KB>
__device__ __forceinline__ void mnc_frag(const float* s, int rb, float (&f)[KS<KB>::HK]) {
    using G = KS<KB>;
    const int lane = threadIdx.x & 63;
    const float* q = s + (lane >> 5) * G::HK * ROWS + rb + (lane & 31);
#pragma unroll
    for (int i = 0; i < G::HK; ++i) f[i] = q[i * ROWS];
}

template <bool KC, int ROWS, int KB>
struct OpLds {
    static constexpr int FLOATS = KC ? ROWS * KS<KB>::LDK : KB * ROWS;
};

// --------------------------------------------------------------------------------------------
// The engine.  LA/LB: loader types; KCA/KCB: their LDS image kind; Epi: epilogue functor with
//   __device__ void operator()(const GemmArgs&, int m, int n, float v)
// plus static constexpr bool STATS (per-column BN partial sums written to a.stats).
// blockIdx.x -> M tile, blockIdx.y -> N tile, blockIdx.z -> split-K slice.
// --------------------------------------------------------------------------------------------
template <class E, class = void>
struct is_nostore : std::false_type {};   // a row-major epilogue that only forms BN partials
template <class E>
struct is_nostore<E, std::void_t<decltype(E::NOSTORE)>> : std::integral_constant<bool, E::NOSTORE> {};
template <class E, class = void>
struct has_finish : std::false_type {};   // a structured epilogue with per-block state and a tile finish
template <class E>
struct has_finish<E, std::void_t<decltype(E::FINISH)>> : std::integral_constant<bool, E::FINISH> {};
template <class E, class = void>
struct has_wave_store : std::false_type {};   // a structured epilogue that may store a wave's sub-tile at once
template <class E>
struct has_wave_store<E, std::void_t<decltype(E::WAVE_STORE)>> : std::integral_constant<bool, E::WAVE_STORE> {};
template <class E, class = void>
struct has_add_ld : std::false_type {};   // an ADD epilogue whose added matrix has its own row stride (a.ldc2)
template <class E>
struct has_add_ld<E, std::void_t<decltype(E::ADD_LD)>> : std::integral_constant<bool, E::ADD_LD> {};
template <class E, class = void>
struct has_mask : std::false_type {};   // an ADD epilogue that also zeroes where its mask matrix is not > 0
template <class E>
struct has_mask<E, std::void_t<decltype(E::MASK)>> : std::integral_constant<bool, E::MASK> {};
template <class E, class = void>
struct has_prefetch : std::false_type {};   // a structured epilogue that loads its operands for all blocks first
template <class E>
struct has_prefetch<E, std::void_t<decltype(E::PREFETCH)>> : std::integral_constant<bool, E::PREFETCH> {};
template <class E, class = void>
struct is_bnsums : std::false_type {};   // EpiStoreBnSums (epilogues.hpp)
template <class E>
struct is_bnsums<E, std::void_t<decltype(E::BNSUMS)>> : std::integral_constant<bool, E::BNSUMS> {};
template <class E, class = void>
struct is_structured : std::false_type {};
template <class E>
struct is_structured<E, std::void_t<decltype(E::STRUCTURED)>> : std::integral_constant<bool, E::STRUCTURED> {};

// XCD-aware tile order (cdna_hip_programming.md T1, bijective form): the dispatcher deals linear
// block ids round-robin over the 8 XCDs, so consecutive ids land on different private L2s.  Remap so
// that each XCD walks a contiguous range of logical tiles (x fastest): neighbouring M-tiles, which
// share im2col halo rows, then hit the same L2.  Speed only: any placement gives the same result.
struct TileId {
    int x, y, z;
};
__device__ __forceinline__ TileId xcd_tile() {
    const int nx = gridDim.x, ny = gridDim.y;
    const int nwg = nx * ny * gridDim.z;
    const int L = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    int logical = L;
    if (nwg > 8) {
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    TileId t;
    t.x = logical % nx;
    t.y = (logical / nx) % ny;
    t.z = logical / (nx * ny);
    return t;
}

// The same XCD-contiguous walk with y (the N tile) fastest: the N tiles of one M block run back to back
// on one XCD, so its operand A (a window conv's input rows) is fetched into that XCD's L2 once for all
// of them instead of once per XCD that holds one of them
__device__ __forceinline__ TileId xcd_tile_yfast() {
    const int nx = gridDim.x, ny = gridDim.y;
    const int nwg = nx * ny * gridDim.z;
    const int L = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    int logical = L;
    if (nwg > 8) {
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    TileId t;
    t.y = logical % ny;
    t.x = (logical / ny) % nx;
    t.z = logical / (nx * ny);
    return t;
}

// A wave whose sub-tile lies entirely past M or N (in the tail tile of a dimension that is not a
// multiple of the tile: e.g. the 576 = 2.25 x 256 columns of a 64-channel weight gradient) skips its
// MFMAs, leaving the SIMD to co-resident waves; it still stages operands and joins every barrier.
__device__ __forceinline__ bool wave_live(const GemmArgs& a, int m0, int n0, int wrows, int wcols) {
    return m0 + wrows < a.M && n0 + wcols < a.N;
}

// ---------------------------------------------------------------------------------------------
// BatchNorm partials of a GEMM tile in shifted (Chan / Welford) form.  A tile writes, per column n,
// S = sum y and M2 = sum (y - mean_tile)^2 over its valid rows, and its valid-row count once:
//   a.stats[tile][0][n] = S, a.stats[tile][1][n] = M2, a.stats[gridDim.x * 2N + tile] = count.
// bn_fwd_finalize then forms sum y^2 = sum_t (M2_t + S_t^2 / n_t) in fp64, so the variance is never
// the fp32 difference E[y^2] - E[y]^2 (which loses ~log2(1 + mu^2/sigma^2) bits; BaselineUNet's
// train-mode BN normalises with it, baseline_unet.h:32-42).  Each lane accumulates
// (y - s) and (y - s)^2 about a shift s = its first accumulator of the column (any finite value is
// exact algebra; one near the column's values keeps the fp32 sums small), then lanes, waves and
// tiles merge (n, mean, M2) with Chan's pairwise formula.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float mb, float m2b) {
    const float nn = n + nb;
    if (nn > 0.f) {
        const float d = mb - mean, f = nb / nn;
        mean = fmaf(d, f, mean);
        m2 += m2b + d * d * n * f;
    }
    n = nn;
}
template <int NJ>
struct BnTilePartials {
    float sh[NJ], d1[NJ], d2[NJ];
    float cnt;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < NJ; ++j) sh[j] = d1[j] = d2[j] = 0.f;
        cnt = 0.f;
    }
    __device__ __forceinline__ void shift(int j, float v) { sh[j] = v; }
    // valid: the row belongs to the output; count it once per row (column block 0)
    __device__ __forceinline__ void add(int j, float v, bool valid) {
        const float d = valid ? v - sh[j] : 0.f;
        d1[j] += d;
        d2[j] = fmaf(d, d, d2[j]);
        if (j == 0) cnt += valid ? 1.f : 0.f;
    }
    // lanes -> waves (LDS [WM][BN][3]) -> tile; `lds` is free scratch; every thread must call
    template <int WM, int WN>
    __device__ __forceinline__ void finish(const GemmArgs& a, float* lds, int tile_x, int n0) {
        constexpr int BN = 32 * NJ * WN;
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        const int wm = wave / WN, wn = wave % WN;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            float n = cnt, mean = 0.f, m2 = 0.f;
            if (n > 0.f) {
                const float q = d1[j] / n;
                mean = sh[j] + q;
                m2 = fmaxf(d2[j] - d1[j] * q, 0.f);
            }
            chan_merge(n, mean, m2, __shfl_xor(n, 32), __shfl_xor(mean, 32), __shfl_xor(m2, 32));
            if (lane < 32) {
                float* r = lds + (wm * BN + wn * 32 * NJ + j * 32 + lane) * 3;
                r[0] = n; r[1] = mean; r[2] = m2;
            }
        }
        __syncthreads();
        for (int c = tid; c < BN; c += 256) {
            float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) {
                const float* r = lds + (w * BN + c) * 3;
                chan_merge(n, mean, m2, r[0], r[1], r[2]);
            }
            const int nn = n0 + c;
            if (nn < a.N) {
                a.stats[(int64_t)tile_x * 2 * a.N + nn] = n * mean;
                a.stats[(int64_t)tile_x * 2 * a.N + a.N + nn] = m2;
            }
            if (n0 == 0 && c == 0) a.stats[(int64_t)gridDim.x * 2 * a.N + tile_x] = n;
        }
    }
};

// The same partials for 16 x 16 accumulator blocks (v_mfma_f32_16x16x32_bf16: column lane & 15, rows
// 4 (lane >> 4) + reg): NB16 column blocks of 16 per wave; the four lanes of a column merge by
// lane ^ 16 and lane ^ 32, then waves and the tile as above.
template <int NB16>
struct BnTilePartials16 {
    float sh[NB16], d1[NB16], d2[NB16];
    float cnt;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < NB16; ++j) sh[j] = d1[j] = d2[j] = 0.f;
        cnt = 0.f;
    }
    __device__ __forceinline__ void shift(int j, float v) { sh[j] = v; }
    __device__ __forceinline__ void add(int j, float v, bool valid) {
        const float d = valid ? v - sh[j] : 0.f;
        d1[j] += d;
        d2[j] = fmaf(d, d, d2[j]);
        if (j == 0) cnt += valid ? 1.f : 0.f;
    }
    template <int WM, int WN>
    __device__ __forceinline__ void finish(const GemmArgs& a, float* lds, int tile_x, int n0) {
        constexpr int BN = 16 * NB16 * WN;
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        const int wm = wave / WN, wn = wave % WN;
#pragma unroll
        for (int j = 0; j < NB16; ++j) {
            float n = cnt, mean = 0.f, m2 = 0.f;
            if (n > 0.f) {
                const float q = d1[j] / n;
                mean = sh[j] + q;
                m2 = fmaxf(d2[j] - d1[j] * q, 0.f);
            }
            chan_merge(n, mean, m2, __shfl_xor(n, 16), __shfl_xor(mean, 16), __shfl_xor(m2, 16));
            chan_merge(n, mean, m2, __shfl_xor(n, 32), __shfl_xor(mean, 32), __shfl_xor(m2, 32));
            if (lane < 16) {
                float* r = lds + (wm * BN + wn * 16 * NB16 + j * 16 + lane) * 3;
                r[0] = n; r[1] = mean; r[2] = m2;
            }
        }
        __syncthreads();
        for (int c = tid; c < BN; c += 256) {
            float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) {
                const float* r = lds + (w * BN + c) * 3;
                chan_merge(n, mean, m2, r[0], r[1], r[2]);
            }
            const int nn = n0 + c;
            if (nn < a.N) {
                a.stats[(int64_t)tile_x * 2 * a.N + nn] = n * mean;
                a.stats[(int64_t)tile_x * 2 * a.N + a.N + nn] = m2;
            }
            if (n0 == 0 && c == 0) a.stats[(int64_t)gridDim.x * 2 * a.N + tile_x] = n;
        }
    }
};

template <class Epi>
__device__ __forceinline__ const float* epi_row_base(const GemmArgs& a, int m0, int z) {
    if constexpr (is_structured<Epi>::value) return a.C;   // unused by structured epilogues
    else return Epi::row_base(a, m0, z);
}

// Epilogue shared by the engines.  Each wave owns MI x NJ blocks of 32x32: a (32 MI) x (32 NJ)
// sub-tile; the tile is WM x WN waves.  A block's 16 accumulator values per lane (32x32 MFMA layout)
// are visited as four "quads" of 4 consecutive rows at one column: quad g = registers 4g..4g+3, rows
// 4(lane>>5) + 8g, column lane & 31.  `lds` is free scratch (the main loop ended on a barrier).
template <int WM, int WN, int MI, int NJ, class Epi>
__device__ __forceinline__ void gemm_epilogue_t(const GemmArgs& a, const floatx16 (&acc)[MI][NJ], const TileId& tile,
                                                float* lds, Epi epi) {
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int m0 = tile.x * BM, n0 = tile.y * BN;
    // With STATS the per-column BN partials are accumulated in the same pass (each accumulator is read once: keeping them live
    // for a second pass costs 64 VGPRs and an occupancy step).  ssum[j]: the lane's column of block column j.
    BnTilePartials<NJ> bnp;
    if constexpr (Epi::STATS) {
        bnp.init();
#pragma unroll
        for (int j = 0; j < NJ; ++j) bnp.shift(j, acc[0][j][0]);
    }
    // Row-major epilogues (EpiStore, EpiSlab) store through a buffer descriptor based at the tile's
    // first output row whose range ends at row M: rows past M are dropped by the range check and
    // columns past N get an out-of-range offset, so each store is one 32-bit offset add.
    constexpr int ES = Epi::BF16 ? 2 : 4;   // output element bytes
    const int64_t ldc4 = a.ldc * ES;
    const int64_t bytes = (int64_t)(a.M - m0) * ldc4;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(epi_row_base<Epi>(a, m0, tile.z),
                                                (uint32_t)(bytes < (int64_t)kRecords ? bytes : kRecords));
    // the added matrix's row stride in bytes (fp32 rows)
    [[maybe_unused]] const int64_t lda4 = [&]() -> int64_t {
        if constexpr (has_add_ld<Epi>::value) return a.ldc2 * 4;
        else return ldc4;
    }();
    auto add_rsrc = [&]() {
        if constexpr (Epi::ADD) {
            const int64_t abytes = (int64_t)(a.M - m0) * lda4;
            return make_rsrc(Epi::add_base(a, m0), (uint32_t)(abytes < (int64_t)kRecords ? abytes : kRecords));
        } else {
            return rs;
        }
    };
    const __amdgpu_buffer_rsrc_t rsadd = add_rsrc();
    auto mask_rsrc = [&]() {
        if constexpr (has_mask<Epi>::value) return make_rsrc(Epi::mask_base(a, m0), (uint32_t)(bytes < (int64_t)kRecords ? bytes : kRecords));
        else return rs;
    };
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t rsmask = mask_rsrc();
    // the wave's MI x NJ blocks staged through its own LDS slice and stored as 16-byte pieces (when the
    // epilogue's layout allows: wave_store returns false otherwise)
    if constexpr (has_wave_store<Epi>::value) {
        if (epi.template wave_store<MI, NJ>(a, acc, m0 + wm * 32 * MI, n0 + wn * 32 * NJ,
                                            lds + wave * Epi::template lds_floats_per_wave<NJ>()))
            return;
    }
    // one memory round trip for the whole tile instead of one per block
    if constexpr (has_prefetch<Epi>::value)
        epi.template prefetch<MI, NJ>(a, m0 + wm * 32 * MI + 4 * (lane >> 5), n0 + wn * 32 * NJ + (lane & 31));
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if constexpr (is_structured<Epi>::value) {
                static_assert(!Epi::STATS, "structured epilogues carry no BN partials");
                if constexpr (has_prefetch<Epi>::value)
                    epi.block_p(a, m0 + wm * 32 * MI + i * 32 + 4 * (lane >> 5),
                                n0 + wn * 32 * NJ + j * 32 + (lane & 31), acc[i][j], i * NJ + j, j);
                else if constexpr (has_finish<Epi>::value)
                    epi.block_j(a, m0 + wm * 32 * MI + i * 32 + 4 * (lane >> 5),
                                n0 + wn * 32 * NJ + j * 32 + (lane & 31), acc[i][j], j);
                else
                    epi.block(a, m0 + wm * 32 * MI + i * 32 + 4 * (lane >> 5), n0 + wn * 32 * NJ + j * 32 + (lane & 31),
                              acc[i][j]);
                continue;
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = n0 + wn * 32 * NJ + j * 32 + (lane & 31);
                const int mr = wm * 32 * MI + i * 32 + 4 * (lane >> 5) + 8 * g;   // tile-relative row
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[i][j][4 * g + r];
                if constexpr (Epi::ADD) {
                    const uint32_t lo = n < a.N ? (uint32_t)(mr * ldc4 + (int64_t)n * ES) : kOOB;
                    const uint32_t la = n < a.N ? (uint32_t)(mr * lda4 + (int64_t)n * 4) : kOOB;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        v[r] += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                              rsadd, la + (uint32_t)(r * lda4), 0, 0));
                    if constexpr (has_mask<Epi>::value) {   // v [mask > 0] (k_relu_mask's arithmetic)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float mk = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                           rsmask, lo + (uint32_t)(r * ldc4), 0, 0));
                            v[r] = mk > 0.f ? v[r] : 0.f;
                        }
                    }
                }
                if constexpr (Epi::BF16) {   // the stored (rounded) values, which BN then normalises
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = (float)(__bf16)v[r];
                }
                if constexpr (!is_structured<Epi>::value) {
                    const uint32_t lo = n < a.N ? (uint32_t)(mr * ldc4 + (int64_t)n * ES) : kOOB;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if constexpr (!is_nostore<Epi>::value) {
                            if constexpr (Epi::BF16)
                                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (__bf16)v[r]), rs,
                                                                      lo + (uint32_t)(r * ldc4), 0, 0);
                            else
                                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[r]), rs,
                                                                      lo + (uint32_t)(r * ldc4), 0, 0);
                        }
                        if constexpr (Epi::STATS) bnp.add(j, v[r], m0 + mr + r < a.M);
                    }
                }
            }
        }

    // per-column BN partials over this block's BM rows -> a.stats (BnTilePartials); the main loop
    // ended on a barrier, so the LDS operand buffers are free for the reduction
    if constexpr (Epi::STATS) bnp.template finish<WM, WN>(a, lds, tile.x, n0);
    if constexpr (has_finish<Epi>::value) epi.template finish<WM, WN, NJ>(a, lds, tile.x, n0);
}
template <int WM, int WN, class Epi>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, floatx16 (&acc)[2][2], const TileId& tile,
                                              float* lds, Epi epi) {
    gemm_epilogue_t<WM, WN, 2, 2>(a, acc, tile, lds, epi);
}

template <int WM, int WN, int KB, class LA, bool KCA, class LB, bool KCB, class Epi, class InitA, class InitB>
__device__ __forceinline__ void gemm_body(const GemmArgs& a, InitA init_a, InitB init_b, Epi epi) {
    using G = KS<KB>;
    constexpr int BM = 64 * WM, BN = 64 * WN;
    constexpr int SA = OpLds<KCA, BM, KB>::FLOATS, SB = OpLds<KCB, BN, KB>::FLOATS;
    __shared__ __attribute__((aligned(16))) float lds[2 * (SA + SB)];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const TileId tile = xcd_tile();
    const int m0 = tile.x * BM, n0 = tile.y * BN;

    const int nk_total = (a.K + KB - 1) / KB;
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nk_total, kbeg + a.kstages_per_split);

    LA la; LB lb;
    init_a(la, m0, tid, kbeg);
    init_b(lb, n0, tid, kbeg);

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto stage_store = [&](int buf, float4 (&xa)[LA::NV], float4 (&xb)[LB::NV]) {
        la.finish(xa);
        lb.finish(xb);
        float* da = lds + buf * (SA + SB);
        if constexpr (KCA) kc_store<BM, KB>(da, xa); else mnc_store<BM, KB>(da, xa);
        if constexpr (KCB) kc_store<BN, KB>(da + SA, xb); else mnc_store<BN, KB>(da + SA, xb);
    };
    auto stage_compute = [&](int buf) {
        const float* sa = lds + buf * (SA + SB);
        const float* sb = sa + SA;
        float fa[2][G::HK], fb[2][G::HK];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if constexpr (KCA) kc_frag<KB>(sa, wm * 64 + i * 32, fa[i]); else mnc_frag<BM, KB>(sa, wm * 64 + i * 32, fa[i]);
            if constexpr (KCB) kc_frag<KB>(sb, wn * 64 + i * 32, fb[i]); else mnc_frag<BN, KB>(sb, wn * 64 + i * 32, fb[i]);
        }
#pragma unroll
        for (int s = 0; s < G::HK; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
    };

    float4 ra[LA::NV], rb[LB::NV];
    if (kbeg < kend) {
        la.load(ra);
        lb.load(rb);
        stage_store(0, ra, rb);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        if (more) { la.load(ra); lb.load(rb); }
        stage_compute(cur);
        if (more) stage_store(cur ^ 1, ra, rb);
        __syncthreads();
        cur ^= 1;
    }

    gemm_epilogue<WM, WN>(a, acc, tile, lds, epi);
}

}  // namespace cad
