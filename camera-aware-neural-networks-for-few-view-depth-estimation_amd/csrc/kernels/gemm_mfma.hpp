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
// v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chains, 64 FLOP/clk/SIMD = the fp32 peak). BK = 16.
// Operand staging is register-staged double-buffered LDS, one barrier per K-stage.
//   "Kc"  operands (global rows are contiguous along k): LDS image [rows][BK+4] (row stride 80 B:
//         16 consecutive rows hit 16 distinct 16-B bank slots -> conflict-free ds_read_b128).
//   "MNc" operands (global rows are contiguous along m/n, k = pixel is strided): LDS image
//         [BK][rows] read with one ds_read_b32 per MFMA step (32 consecutive lanes, no conflict).
// K order inside a stage is permuted so a lane's 8 k-values are contiguous: MFMA step s, lane half h
// consumes chunk-k = 8h + s (both operands use the same map, so the sum is unchanged).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cad {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 16;
constexpr int LDK = BK + 4;   // Kc LDS row stride (floats)

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
    float* stats;         // BN partials [gridDim.x][2][N]  (sum, sumsq) or nullptr
    int kstages_per_split;
    int64_t slab_stride;  // elements between split-K slabs
};

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// --------------------------------------------------------------------------------------------
// Kc loaders: operand(row r, k) with k contiguous in memory.  Thread t owns rows t/4 + 64j and
// the float4 column group (t&3)*4 of every stage.
// --------------------------------------------------------------------------------------------
template <int ROWS>
struct KcDense {   // op(r,k) = P[r*ld + coff + k], r < nrows, k < K
    static constexpr int NV = ROWS / 64;
    const float* p[NV];
    bool ok[NV];
    int K;
    __device__ void init(const float* P, int64_t ld, int coff, int nrows, int K_, int row0, int tid) {
        K = K_;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            int r = row0 + tid / 4 + 64 * j;
            ok[j] = r < nrows;
            p[j] = P + (int64_t)(ok[j] ? r : 0) * ld + coff + (tid & 3) * 4;
        }
    }
    __device__ void load(int kt, float4 (&v)[NV]) const {
        int k = kt * BK;
        bool kin = (k + ((threadIdx.x & 3) * 4)) < K;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            bool g = ok[j] && kin;
            float4 t = *reinterpret_cast<const float4*>(g ? p[j] + k : p[j]);
            v[j] = g ? t : f4zero();
        }
    }
};

// op(pix, k=(tap,ci)) = X[(b, y+ky-1, x+kx-1)*ld + coff + ci], zero outside the image.
template <int ROWS>
struct KcIm2col3x3 {
    static constexpr int NV = ROWS / 64;
    const float* base;
    int64_t ld;
    int y[NV], x[NV];
    int64_t pix[NV];
    bool ok[NV];
    int H, W, cin, K;
    __device__ void init(const float* P, int64_t ld_, int coff, int cin_, int B, int H_, int W_,
                         int row0, int tid) {
        H = H_; W = W_; cin = cin_; ld = ld_; K = 9 * cin_;
        base = P + coff;   // the float4 column (tid&3)*4 is folded into ci by load()
        int M = B * H * W;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            int r = row0 + tid / 4 + 64 * j;
            ok[j] = r < M;
            int rr = ok[j] ? r : 0;
            x[j] = rr % W;
            y[j] = (rr / W) % H;
            pix[j] = rr;
        }
    }
    __device__ void load(int kt, float4 (&v)[NV]) const {
        int k = kt * BK + (threadIdx.x & 3) * 4;
        bool kin = k < K;
        int tap = kin ? k / cin : 0;
        int ci = k - tap * cin;
        int dy = tap / 3 - 1, dx = tap % 3 - 1;
        int64_t off = (int64_t)(dy * W + dx) * ld + ci;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            int yy = y[j] + dy, xx = x[j] + dx;
            bool g = ok[j] && kin && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            const float* q = base + pix[j] * ld + (g ? off : 0);
            float4 t = *reinterpret_cast<const float4*>(q);
            v[j] = g ? t : f4zero();
        }
    }
};

// op(lowres pix (b,y,x), k=(q=(dy,dx), co)) = G[(b, 2y+dy, 2x+dx)*ld + coff + co]
template <int ROWS>
struct KcUpGather {
    static constexpr int NV = ROWS / 64;
    const float* base;
    int64_t ld;
    int64_t hrpix[NV];   // high-res pixel index of (2y, 2x)
    bool ok[NV];
    int W2, cout, K;
    __device__ void init(const float* P, int64_t ld_, int coff, int cout_, int B, int H, int W,
                         int row0, int tid) {
        ld = ld_; cout = cout_; K = 4 * cout_; W2 = 2 * W;
        base = P + coff;   // the float4 column (tid&3)*4 is folded into ci by load()
        int M = B * H * W;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            int r = row0 + tid / 4 + 64 * j;
            ok[j] = r < M;
            int rr = ok[j] ? r : 0;
            int xx = rr % W, t = rr / W, yy = t % H, b = t / H;
            hrpix[j] = ((int64_t)b * (2 * H) + 2 * yy) * W2 + 2 * xx;
        }
    }
    __device__ void load(int kt, float4 (&v)[NV]) const {
        int k = kt * BK + (threadIdx.x & 3) * 4;
        bool kin = k < K;
        int q = kin ? k / cout : 0;
        int co = k - q * cout;
        int64_t off = (int64_t)((q >> 1) * W2 + (q & 1)) * ld + co;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            bool g = ok[j] && kin;
            const float* p = base + hrpix[j] * ld + (g ? off : 0);
            float4 t = *reinterpret_cast<const float4*>(p);
            v[j] = g ? t : f4zero();
        }
    }
};

// --------------------------------------------------------------------------------------------
// MNc loaders: operand(row r, k=pixel); memory rows are pixels, contiguous along r.
// Thread t owns row group cg = t % (ROWS/4) (4 rows) and k-rows t/(ROWS/4) + KSTEP*j.
// --------------------------------------------------------------------------------------------
template <int ROWS>
struct MNcBase {
    static constexpr int TPR = ROWS / 4;          // threads per k-row
    static constexpr int KSTEP = 256 / TPR;       // k-rows per pass
    static constexpr int NV = BK / KSTEP;
};

template <int ROWS>
struct MNcDense : MNcBase<ROWS> {   // op(r, k) = P[k*ld + coff + r], r < nrows, k < Kp
    using Base = MNcBase<ROWS>;
    static constexpr int NV = Base::NV;
    const float* p;
    int64_t ld;
    int Kp;
    bool rok;
    __device__ void init(const float* P, int64_t ld_, int coff, int nrows, int Kp_, int row0, int tid) {
        ld = ld_; Kp = Kp_;
        int r = row0 + (tid % Base::TPR) * 4;
        rok = r < nrows;   // nrows % 4 == 0 is required
        p = P + coff + (rok ? r : 0);
    }
    __device__ void load(int kt, float4 (&v)[NV]) const {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            int k = kt * BK + threadIdx.x / Base::TPR + Base::KSTEP * j;
            bool g = rok && k < Kp;
            float4 t = *reinterpret_cast<const float4*>(p + (int64_t)(g ? k : 0) * ld);
            v[j] = g ? t : f4zero();
        }
    }
};

// op(j=(tap,ci), k=pix) = X[(b,y+ky-1,x+kx-1)*ld + coff + ci]
template <int ROWS>
struct MNcIm2col3x3 : MNcBase<ROWS> {
    using Base = MNcBase<ROWS>;
    static constexpr int NV = Base::NV;
    const float* p;
    int64_t ld;
    int H, W, Kp, dy, dx;
    bool rok;
    __device__ void init(const float* P, int64_t ld_, int coff, int cin, int B, int H_, int W_,
                         int row0, int tid) {
        ld = ld_; H = H_; W = W_; Kp = B * H_ * W_;
        int j = row0 + (tid % Base::TPR) * 4;
        rok = j < 9 * cin;
        int jj = rok ? j : 0;
        int tap = jj / cin, ci = jj - tap * cin;
        dy = tap / 3 - 1; dx = tap % 3 - 1;
        p = P + coff + ci;
    }
    __device__ void load(int kt, float4 (&v)[NV]) const {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            int k = kt * BK + threadIdx.x / Base::TPR + Base::KSTEP * j;
            int kk = k < Kp ? k : 0;
            int x = kk % W, y = (kk / W) % H;
            int yy = y + dy, xx = x + dx;
            bool g = rok && k < Kp && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            int64_t q = g ? (int64_t)kk + dy * W + dx : 0;
            float4 t = *reinterpret_cast<const float4*>(p + q * ld);
            v[j] = g ? t : f4zero();
        }
    }
};

// op(j=(q,co), k=lowres pix (b,y,x)) = G[(b,2y+dy,2x+dx)*ld + coff + co]
template <int ROWS>
struct MNcUpGather : MNcBase<ROWS> {
    using Base = MNcBase<ROWS>;
    static constexpr int NV = Base::NV;
    const float* p;
    int64_t ld;
    int H, W, Kp, qy, qx;
    bool rok;
    __device__ void init(const float* P, int64_t ld_, int coff, int cout, int B, int H_, int W_,
                         int row0, int tid) {
        ld = ld_; H = H_; W = W_; Kp = B * H_ * W_;
        int j = row0 + (tid % Base::TPR) * 4;
        rok = j < 4 * cout;
        int jj = rok ? j : 0;
        int q = jj / cout, co = jj - q * cout;
        qy = q >> 1; qx = q & 1;
        p = P + coff + co;
    }
    __device__ void load(int kt, float4 (&v)[NV]) const {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            int k = kt * BK + threadIdx.x / Base::TPR + Base::KSTEP * j;
            bool g = rok && k < Kp;
            int kk = g ? k : 0;
            int x = kk % W, t = kk / W, y = t % H, b = t / H;
            int64_t hp = ((int64_t)b * (2 * H) + 2 * y + qy) * (2 * W) + 2 * x + qx;
            float4 t4 = *reinterpret_cast<const float4*>(p + hp * ld);
            v[j] = g ? t4 : f4zero();
        }
    }
};

// --------------------------------------------------------------------------------------------
// LDS staging + fragment reads
// --------------------------------------------------------------------------------------------
template <int ROWS, int NV>
__device__ __forceinline__ void kc_store(float* s, const float4 (&v)[NV]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NV; ++j)
        *reinterpret_cast<float4*>(s + (t / 4 + 64 * j) * LDK + (t & 3) * 4) = v[j];
}
template <int ROWS, int NV>
__device__ __forceinline__ void mnc_store(float* s, const float4 (&v)[NV]) {
    constexpr int TPR = ROWS / 4, KSTEP = 256 / TPR;
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NV; ++j)
        *reinterpret_cast<float4*>(s + (t / TPR + KSTEP * j) * ROWS + (t % TPR) * 4) = v[j];
}
// fragment: 8 consecutive chunk-k values of row (rb + lane&31), half h = lane>>5
__device__ __forceinline__ void kc_frag(const float* s, int rb, float (&f)[8]) {
    const int lane = threadIdx.x & 63;
    const float* q = s + (rb + (lane & 31)) * LDK + (lane >> 5) * 8;
    float4 a = *reinterpret_cast<const float4*>(q);
    float4 b = *reinterpret_cast<const float4*>(q + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
template <int ROWS>
__device__ __forceinline__ void mnc_frag(const float* s, int rb, float (&f)[8]) {
    const int lane = threadIdx.x & 63;
    const float* q = s + (lane >> 5) * 8 * ROWS + rb + (lane & 31);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = q[i * ROWS];
}

template <bool KC, int ROWS>
struct OpLds {
    static constexpr int FLOATS = KC ? ROWS * LDK : BK * ROWS;
};

// --------------------------------------------------------------------------------------------
// The engine.  LA/LB: loader types; KCA/KCB: their LDS image kind; Epi: epilogue functor with
//   __device__ void operator()(const GemmArgs&, int m, int n, float v)
// plus static constexpr bool STATS (per-column BN partial sums written to a.stats).
// blockIdx.x -> M tile, blockIdx.y -> N tile, blockIdx.z -> split-K slice.
// --------------------------------------------------------------------------------------------
template <int WM, int WN, class LA, bool KCA, class LB, bool KCB, class Epi, class InitA, class InitB>
__device__ __forceinline__ void gemm_body(const GemmArgs& a, InitA init_a, InitB init_b, Epi epi) {
    constexpr int BM = 64 * WM, BN = 64 * WN;
    constexpr int SA = OpLds<KCA, BM>::FLOATS, SB = OpLds<KCB, BN>::FLOATS;
    __shared__ __attribute__((aligned(16))) float lds[2 * (SA + SB)];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

    LA la; LB lb;
    init_a(la, m0, tid);
    init_b(lb, n0, tid);

    const int nk_total = (a.K + BK - 1) / BK;
    const int kbeg = blockIdx.z * a.kstages_per_split;
    const int kend = min(nk_total, kbeg + a.kstages_per_split);

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[LA::NV], rb[LB::NV];
    if (kbeg < kend) {
        la.load(kbeg, ra);
        lb.load(kbeg, rb);
        if constexpr (KCA) kc_store<BM>(lds, ra); else mnc_store<BM>(lds, ra);
        if constexpr (KCB) kc_store<BN>(lds + SA, rb); else mnc_store<BN>(lds + SA, rb);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        if (more) { la.load(kt + 1, ra); lb.load(kt + 1, rb); }
        const float* sa = lds + cur * (SA + SB);
        const float* sb = sa + SA;
        float fa[2][8], fb[2][8];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if constexpr (KCA) kc_frag(sa, wm * 64 + i * 32, fa[i]); else mnc_frag<BM>(sa, wm * 64 + i * 32, fa[i]);
            if constexpr (KCB) kc_frag(sb, wn * 64 + i * 32, fb[i]); else mnc_frag<BN>(sb, wn * 64 + i * 32, fb[i]);
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
        if (more) {
            float* da = lds + (cur ^ 1) * (SA + SB);
            if constexpr (KCA) kc_store<BM>(da, ra); else mnc_store<BM>(da, ra);
            if constexpr (KCB) kc_store<BN>(da + SA, rb); else mnc_store<BN>(da + SA, rb);
        }
        __syncthreads();
        cur ^= 1;
    }

    // epilogue: element (m, n) of sub-block (i, j), register r
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 64 + j * 32 + col;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < a.M && n < a.N) epi(a, m, n, acc[i][j][r]);
            }
        }

    if constexpr (Epi::STATS) {
        // per-column partial sum / sum of squares over this block's BM rows -> a.stats[bx][2][N]
        float* red = lds;   // reuse: [WM][BN][2]
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float s = 0.f, q = 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const float v = m < a.M ? acc[i][j][r] : 0.f;
                    s += v;
                    q += v * v;
                }
            s += __shfl_xor(s, 32);
            q += __shfl_xor(q, 32);
            if (h == 0) {
                const int cl = wn * 64 + j * 32 + col;
                red[(wm * BN + cl) * 2 + 0] = s;
                red[(wm * BN + cl) * 2 + 1] = q;
            }
        }
        __syncthreads();
        for (int c = tid; c < BN; c += 256) {
            float s = 0.f, q = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) { s += red[(w * BN + c) * 2]; q += red[(w * BN + c) * 2 + 1]; }
            const int n = n0 + c;
            if (n < a.N) {
                a.stats[(int64_t)blockIdx.x * 2 * a.N + n] = s;
                a.stats[(int64_t)blockIdx.x * 2 * a.N + a.N + n] = q;
            }
        }
    }
}

}  // namespace cad
