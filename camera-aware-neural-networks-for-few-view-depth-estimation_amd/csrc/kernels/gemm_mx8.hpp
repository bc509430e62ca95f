// MX-fp8 contraction engine ("X8"): block-scaled fp8 operands on v_mfma_scale_f32_32x32x64_f8f6f4.
//
// Operand format (OCP Microscaling v1.0, MXFP8 with E4M3 elements): a tensor of rows (pixels, or
// output channels for weights) whose k axis (channels, or (tap, channel) for the 3x3 weights) is cut
// into blocks of 32 consecutive elements; each block stores one shared power-of-two scale (E8M0 byte,
// 2^(byte - 127)) and 32 E4M3 elements (OCP e4m3fn: bias 7, max normal 448, no infinities).
//   Mx8 view: q = element bytes [rows][ld] (element k of a row at byte k), s = scale bytes
//   [rows][ld / 32] (block k / 32); ld % 128 == 0, so a row's scales are whole 32-bit words.
// Quantisation of a block v[0..31] (MX spec §6.3, with the saturating element conversion):
//   e = floor(log2(max |v|)) from the fp32 exponent field (0 for a zero block), shared = e - 8
//   (8 = emax of E4M3) clamped to [-127, 127]; element = e4m3_rne(clamp(v * 2^-shared, +-448)).
// The block's largest element then lands in [256, 512) before saturation, i.e. in E4M3's top binade.
// tests/test_gpu_mx8.py checks the GPU quantiser bit for bit against torch's float8_e4m3fn cast of
// the same arithmetic (oracle/resunet_oracle.py mx8_quantize).
//
// The MFMA (lane map measured on MI355X with exact integer data, tools/probe_mx_fp8.hip): lane l (row
// r = l & 31, half h = l >> 5) holds 32 elements of its A row (B column) in 8 VGPRs — bytes 0..15 are
// k = 16h .. 16h + 15 (k-block 0), bytes 16..31 are k = 32 + 16h .. (k-block 1) — and one scale byte,
// which the hardware applies to k-block h of row r (lanes r and r + 32 carry the row's two scales).
// So the per-block scales of both operands are applied exactly (products of E4M3 values and powers
// of two are exact in fp32; accumulation fp32).  Rate: 64 cycles per 32x32x64 = twice the
// bf16 MFMA's 32 cycles per 32x32x16 (MI355X_MICROARCH.md § Matrix cores).
#pragma once
#include "gemm_s3.hpp"
#include "gemm_ps.hpp"
#include "gemm_win.hpp"
#include "kernels.hpp"   // Mx8
#include "mx8_quant.hpp"

namespace cad {

typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ i32x8 x8_join(uint4 lo, uint4 hi) {
    i32x8 f;
    f[0] = (int)lo.x; f[1] = (int)lo.y; f[2] = (int)lo.z; f[3] = (int)lo.w;
    f[4] = (int)hi.x; f[5] = (int)hi.y; f[6] = (int)hi.z; f[7] = (int)hi.w;
    return f;
}

// one 32-element block: v[32] -> 32 element bytes (8 words) + the scale byte
__device__ __forceinline__ uint32_t mx8_quant_block(const float (&v)[32], uint32_t (&q)[8]) {
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(v[i]));
    const int sh = mx8_shared_exp(amax);
    const float inv = mx8_inv_scale(sh < 127 ? sh : 126);
#pragma unroll
    for (int w = 0; w < 8; ++w) q[w] = mx8_pack4(v[4 * w] * inv, v[4 * w + 1] * inv, v[4 * w + 2] * inv, v[4 * w + 3] * inv);
    return (uint32_t)(sh + 127);
}

// ------------------------------------------------------------------------------------------------
// Dense k-contiguous operands: op(r, k) = Q[r][coff + k] (scales S[r][(coff + k) / 32]).
// One stage = KB = 128 k = 8 pieces of 16 B per row + one 32-bit scale word per row.  Thread t owns
// pieces t + 256 j (row = piece / 8) and, for t < ROWS, the scale word of row t.
// LDS image per operand: [ROWS][144 B] elements (128 + 16 pad: conflict-free ds_read_b128, the
// byte geometry of the bf16 KB = 64 rows) then [ROWS] scale words.
// ------------------------------------------------------------------------------------------------
constexpr int kX8KB = 128;
constexpr int kX8Row = 144;   // LDS bytes per element row

template <int ROWS>
struct X8Kc {
    static constexpr int NV = ROWS * 8 / 256;
    static constexpr int NS = (ROWS + 255) / 256;
    static constexpr int BYTES = ROWS * kX8Row + ROWS * 4;
    using Regs = uint4[NV];
    using SRegs = uint32_t[NS];
    __amdgpu_buffer_rsrc_t rq, rs;
    uint32_t qoff[NV];
    uint32_t soff[NS];
    int lofs[NV];
    int k0, K;
    __device__ void init(const Mx8& m, int nrows, int K_, int row0, int tid, int kbeg) {
        K = K_;
        k0 = kbeg * kX8KB;
        rq = make_rsrc(ps_at(reinterpret_cast<const float*>(m.q), (int64_t)row0 * m.ld + m.coff));
        rs = make_rsrc(ps_at(reinterpret_cast<const float*>(m.s), (int64_t)row0 * (m.ld >> 5) + (m.coff >> 5)));
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int p = tid + 256 * j, row = p >> 3, g = p & 7;
            qoff[j] = row0 + row < nrows ? (uint32_t)(row * m.ld + g * 16) : kOOB;
            lofs[j] = row * kX8Row + g * 16;
        }
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int row = tid + 256 * j;
            soff[j] = (row < ROWS && row0 + row < nrows) ? (uint32_t)(row * (m.ld >> 5)) : kOOB;
        }
    }
    __device__ void load(Regs& v, SRegs& sv) {
        const bool kin = k0 < K;
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = bload16(rq, kin && qoff[j] != kOOB ? qoff[j] + (uint32_t)k0 : kOOB);
#pragma unroll
        for (int j = 0; j < NS; ++j)
            sv[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, kin && soff[j] != kOOB ? soff[j] + (uint32_t)(k0 >> 5) : kOOB, 0, 0);
        k0 += kX8KB;
    }
    __device__ void store(const Regs& v, const SRegs& sv, char* s) const {
#pragma unroll
        for (int j = 0; j < NV; ++j) *reinterpret_cast<uint4*>(s + lofs[j]) = v[j];
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NS; ++j)
            if (tid + 256 * j < ROWS) *reinterpret_cast<uint32_t*>(s + ROWS * kX8Row + 4 * (tid + 256 * j)) = sv[j];
    }
};

// fragment of 32-row block rb, k-step q (64 k): the lane's 32 elements + its block scale byte
template <int ROWS>
__device__ __forceinline__ void x8_frag(const char* s, int rb, int q, i32x8& f, int& sc) {
    const int lane = threadIdx.x & 63;
    const int r = rb + (lane & 31), h = lane >> 5;
    const char* p = s + r * kX8Row + q * 64 + h * 16;   // block 2q: bytes 16h..; block 2q+1: 32 + 16h..
    const uint4 lo = *reinterpret_cast<const uint4*>(p);
    const uint4 hi = *reinterpret_cast<const uint4*>(p + 32);
    f = x8_join(lo, hi);
    const uint32_t w = *reinterpret_cast<const uint32_t*>(s + ROWS * kX8Row + 4 * r);
    sc = (int)((w >> (8 * (2 * q + h))) & 0xFF);
}

__device__ __forceinline__ floatx16 x8_mfma(const i32x8& a, int sa, const i32x8& b, int sb, const floatx16& c) {
    // cbsz = blgp = 0: both operands E4M3; opsel 0: the scale in byte 0 of the scale operands
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

// C[m][n] = sum_k A(m, k) B(n, k): 4 waves (WM x WN), MI x NJ blocks of 32x32 per wave, 128-deep
// stages, double-buffered LDS + one register set per operand (ps_pipeline of gemm_ps.hpp)
template <int WM, int WN, int MI, int NJ, class Epi>
__device__ __forceinline__ void dense_body_x8(const GemmArgs& a, const Mx8& ma, const Mx8& mb) {
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    using LA = X8Kc<BM>;
    using LB = X8Kc<BN>;
    constexpr int SA = LA::BYTES, SB = LB::BYTES;
    __shared__ __attribute__((aligned(16))) char lds[2 * (SA + SB)];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const TileId tile = xcd_tile();
    const int m0 = tile.x * BM, n0 = tile.y * BN;
    const int nk = (a.K + kX8KB - 1) / kX8KB;

    LA la; LB lb;
    la.init(ma, a.M, a.K, m0, tid, 0);
    lb.init(mb, a.N, a.K, n0, tid, 0);

    floatx16 acc[MI][NJ];
    acc_zero(acc);
    typename LA::Regs ra; typename LA::SRegs rsa;
    typename LB::Regs rb; typename LB::SRegs rsb;
    auto store = [&](int buf) {
        char* d = lds + buf * (SA + SB);
        la.store(ra, rsa, d);
        lb.store(rb, rsb, d + SA);
    };
    auto compute = [&](int buf) {
        const char* sa = lds + buf * (SA + SB);
        const char* sb = sa + SA;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            i32x8 fa[MI], fb[NJ];
            int ca[MI], cb[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) x8_frag<BN>(sb, wn * 32 * NJ + j * 32, q, fb[j], cb[j]);
#pragma unroll
            for (int i = 0; i < MI; ++i) x8_frag<BM>(sa, wm * 32 * MI + i * 32, q, fa[i], ca[i]);
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = x8_mfma(fa[i], ca[i], fb[j], cb[j], acc[i][j]);
        }
    };
    if (nk > 0) {
        la.load(ra, rsa);
        lb.load(rb, rsb);
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
        const bool more = kt + 1 < nk;
        if (more) { la.load(ra, rsa); lb.load(rb, rsb); }
        compute(cur);
        if (more) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    gemm_epilogue_t<WM, WN, MI, NJ>(a, acc, tile, reinterpret_cast<float*>(lds), Epi{});
}

// ------------------------------------------------------------------------------------------------
// Window-tiled conv3x3 forward on MX operands (the structure of conv3x3_win_ps_body, gemm_win.hpp):
// a workgroup owns an R x CW block of output pixels; stage (cb, ky) = 64 channels cb*64.. of kernel
// row ky: A = the input window R x (CW+2) pixels x 64 elements (+ 2 scale bytes per pixel), B = the
// three taps' weights [3][BN][64] (+ 2 scale bytes per row).  Tap kx reads the window at pixel
// offset kx; one 32x32x64 MFMA per tap and block pair covers the stage's 64 channels.
// LDS rows of 80 B (64 + 16 pad, conflict-free ds_read_b128); scale images as 16-bit words.
// Weights: MX rows [cout][9 cin] in (tap, ci) order.  Requirements (host): cin % 64 == 0,
// W % CW == 0, N % BN == 0, operand offsets % 64 == 0.
// ------------------------------------------------------------------------------------------------
template <int R, int CW, int BN>
struct WinX8Geo {
    static constexpr int WC = CW + 2;
    static constexpr int WPIX = R * WC;
    static constexpr int ROW = 80;                         // LDS bytes per pixel / weight row
    static constexpr int NTA = WPIX * 4;                   // 16-B pieces of A per stage
    static constexpr int NVA = (NTA + 255) / 256;
    static constexpr int NTB = BN * 4;                     // pieces of one tap of B
    static constexpr int JB = (NTB + 255) / 256;
    static constexpr int NSA = (WPIX + 255) / 256;         // scale words (u16) of A per stage
    static constexpr int NSB = (3 * BN + 255) / 256;       // ... of B (tap, row)
    static constexpr int SA = WPIX * ROW, SBT = BN * ROW;  // bytes
    static constexpr int SSA = WPIX * 2, SSB = 3 * BN * 2;
    static constexpr int BYTES = SA + 3 * SBT + SSA + SSB;
};

template <int R, int CW, int WM, int WN, class Epi, int MI = 2>
__device__ __forceinline__ void conv3x3_win_x8_body(const GemmArgs& a, const Mx8& mx, const Mx8& mw) {
    constexpr int NJ = 2;
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    static_assert(BM == R * CW, "tile");
    using G = WinX8Geo<R, CW, BN>;
    __shared__ __attribute__((aligned(16))) char lds[G::BYTES];
    char* const lA = lds;
    char* const lB = lds + G::SA;
    char* const lSA = lds + G::SA + 3 * G::SBT;
    char* const lSB = lSA + G::SSA;

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const TileId tile = xcd_tile();
    const int nbx = a.W / CW, nby = (a.H + R - 1) / R;
    const int tx = tile.x % nbx, t2 = tile.x / nbx, ty = t2 % nby, b = t2 / nby;
    const int y0 = ty * R, x0 = tx * CW, n0 = tile.y * BN;
    const int H = a.H, W = a.W, cin = a.a_cin;
    const int S = 3 * (cin / 64);

    // A: element rows of mx.ld bytes; piece (window pixel w, 16-B group g) of stage (cb, ky)
    const int rowq = (int)mx.ld, rows_ = (int)(mx.ld >> 5);
    const int64_t pbase = ((int64_t)b * H + y0 - 1) * W + x0 - 1;
    const int64_t pb = pbase > 0 ? pbase : 0;
    const __amdgpu_buffer_rsrc_t rqa = make_rsrc(ps_at(reinterpret_cast<const float*>(mx.q), pb * mx.ld + mx.coff));
    const __amdgpu_buffer_rsrc_t rsa =
        make_rsrc(ps_at(reinterpret_cast<const float*>(mx.s), pb * (mx.ld >> 5) + (mx.coff >> 5)));
    int aoff[G::NVA], awr[G::NVA];
#pragma unroll
    for (int j = 0; j < G::NVA; ++j) {
        const int f = tid + 256 * j;
        const int w = f >> 2, g = f & 3;
        const int r = w / G::WC, c = w - r * G::WC;
        const int x = x0 - 1 + c;
        const bool ok = f < G::NTA && (unsigned)x < (unsigned)W;
        awr[j] = ok ? r : -(1 << 28);
        aoff[j] = (int)((r * (int64_t)W + c + (pbase - pb)) * rowq) + g * 16;
    }
    int soff[G::NSA], swr[G::NSA];
#pragma unroll
    for (int j = 0; j < G::NSA; ++j) {
        const int w = tid + 256 * j;
        const int r = w / G::WC, c = w - r * G::WC;
        const int x = x0 - 1 + c;
        const bool ok = w < G::WPIX && (unsigned)x < (unsigned)W;
        swr[j] = ok ? r : -(1 << 28);
        soff[j] = (int)((r * (int64_t)W + c + (pbase - pb)) * rows_);
    }
    // B: weight rows of mw.ld bytes (= 9 cin), piece (tap, row, group)
    const int rowqb = (int)mw.ld, rowsb = (int)(mw.ld >> 5);
    const __amdgpu_buffer_rsrc_t rqb = make_rsrc(ps_at(reinterpret_cast<const float*>(mw.q), (int64_t)n0 * mw.ld + mw.coff));
    const __amdgpu_buffer_rsrc_t rsb =
        make_rsrc(ps_at(reinterpret_cast<const float*>(mw.s), (int64_t)n0 * (mw.ld >> 5) + (mw.coff >> 5)));
    int boff[G::JB];
#pragma unroll
    for (int jj = 0; jj < G::JB; ++jj) {
        const int task = tid + 256 * jj;
        boff[jj] = (task >> 2) * rowqb + (task & 3) * 16;
    }
    auto bact = [&](int jj) { return 256 * (jj + 1) <= G::NTB || tid + 256 * jj < G::NTB; };

    int wpix[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int p = wm * 32 * MI + i * 32 + (lane & 31);
        const int r = p / CW;
        wpix[i] = r * G::WC + (p - r * CW);
    }

    floatx16 acc[MI][NJ];
    acc_zero(acc);
    uint4 ra[G::NVA], rb[3 * G::JB];
    uint32_t rsA[G::NSA], rsB[G::NSB];
    int cb = 0, ky = 0;
    auto load = [&]() {
        const int adda = ky * W * rowq + cb * 64;
        const int adds = ky * W * rows_ + cb * 2;
#pragma unroll
        for (int j = 0; j < G::NVA; ++j) {
            const int y = y0 - 1 + ky + awr[j];
            ra[j] = bload16(rqa, (unsigned)y < (unsigned)H ? (uint32_t)(aoff[j] + adda) : kOOB);
        }
#pragma unroll
        for (int j = 0; j < G::NSA; ++j) {
            const int y = y0 - 1 + ky + swr[j];
            rsA[j] = __builtin_amdgcn_raw_buffer_load_b16(rsa, (unsigned)y < (unsigned)H ? (uint32_t)(soff[j] + adds) : kOOB,
                                                          0, 0);
        }
        const int addb = 3 * ky * cin + cb * 64;
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int jj = 0; jj < G::JB; ++jj)
                if (bact(jj)) rb[t * G::JB + jj] = bload16(rqb, (uint32_t)(boff[jj] + addb + t * cin));
        // B scales: slot e = tid + 256 j < 3 BN is (tap e / BN, row e % BN)
#pragma unroll
        for (int j = 0; j < G::NSB; ++j) {
            const int e = tid + 256 * j;
            const int t = e / BN, row = e - t * BN;
            rsB[j] = e < 3 * BN ? __builtin_amdgcn_raw_buffer_load_b16(
                                      rsb, (uint32_t)(row * rowsb + ((3 * ky + t) * cin + cb * 64) / 32), 0, 0)
                                : 0u;
        }
        if (++ky == 3) { ky = 0; ++cb; }
    };
    auto store = [&]() {
#pragma unroll
        for (int j = 0; j < G::NVA; ++j) {
            const int f = tid + 256 * j;
            if (f < G::NTA) *reinterpret_cast<uint4*>(lA + (f >> 2) * G::ROW + (f & 3) * 16) = ra[j];
        }
#pragma unroll
        for (int j = 0; j < G::NSA; ++j)
            if (tid + 256 * j < G::WPIX) *reinterpret_cast<uint16_t*>(lSA + 2 * (tid + 256 * j)) = (uint16_t)rsA[j];
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int jj = 0; jj < G::JB; ++jj)
                if (bact(jj)) {
                    const int task = tid + 256 * jj;
                    *reinterpret_cast<uint4*>(lB + t * G::SBT + (task >> 2) * G::ROW + (task & 3) * 16) = rb[t * G::JB + jj];
                }
#pragma unroll
        for (int j = 0; j < G::NSB; ++j)
            if (tid + 256 * j < 3 * BN) *reinterpret_cast<uint16_t*>(lSB + 2 * (tid + 256 * j)) = (uint16_t)rsB[j];
    };
    const int h = lane >> 5;
    auto compute = [&]() {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            i32x8 fa[MI], fb[NJ];
            int ca[MI], cbs[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = wn * 32 * NJ + j * 32 + (lane & 31);
                const char* p = lB + kx * G::SBT + row * G::ROW + h * 16;
                fb[j] = x8_join(*reinterpret_cast<const uint4*>(p), *reinterpret_cast<const uint4*>(p + 32));
                cbs[j] = (int)((*reinterpret_cast<const uint16_t*>(lSB + 2 * (kx * BN + row)) >> (8 * h)) & 0xFF);
            }
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int w = wpix[i] + kx;
                const char* p = lA + w * G::ROW + h * 16;
                fa[i] = x8_join(*reinterpret_cast<const uint4*>(p), *reinterpret_cast<const uint4*>(p + 32));
                ca[i] = (int)((*reinterpret_cast<const uint16_t*>(lSA + 2 * w) >> (8 * h)) & 0xFF);
            }
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = x8_mfma(fa[i], ca[i], fb[j], cbs[j], acc[i][j]);
        }
    };

    if (S > 0) {
        load();
        store();
    }
    __syncthreads();
    for (int s = 0; s < S; ++s) {
        const bool more = s + 1 < S;
        if (more) load();
        compute();
        __syncthreads();
        if (more) {
            store();
            __syncthreads();
        }
    }
    win_epilogue<WM, WN, MI, NJ, CW, Epi>(a, acc, tile.x, n0, b, y0, x0, reinterpret_cast<float*>(lds));
}

}  // namespace cad
