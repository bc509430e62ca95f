// Window-tiled conv3x3 forward / dgrad on the S3 (NP = 3) and B1 (NP = 1) engines.
//
// The im2col GEMM (gemm_s3.hpp + KcIm2col3x3) fetches and splits every input element once per tap
// that reads it: 9 fetches + 9 three-plane splits per element and output tile.  Here a workgroup
// owns an R x CW block of output pixels of one image (BM = R*CW) and walks K in stages of
// (16-channel block cb, kernel row ky): the stage's A operand is the input WINDOW of R rows x (CW+2)
// columns (the block's rows shifted by ky-1, one halo column each side) x 16 channels, fetched and
// split ONCE, and the three taps kx = 0, 1, 2 of the kernel row read it at column offsets kx — the
// shift is a whole LDS row (one window pixel = 32 B per plane), so the fragment reads stay aligned
// ds_read_b128.  Per three k16 steps the A traffic (global loads, split VALU, LDS stores) drops from
// 3*BM*16 to R*(CW+2)*16 elements (~2.9x).  B is the three taps' weights (Kc, 3 x BN x 16).
//
//   C[pix][n] = sum_{cb, ky, kx, ci} X[(b, y+ky-1, x+kx-1)][cb*16+ci] * Wt[n][(3ky+kx)*cin + cb*16+ci]
//
// Per stage and wave: 3 k16 steps x MI x NJ blocks x NP products (S3: 72 MFMAs).  LDS holds ONE
// stage (A window + B taps; 49.5 KB for BM = BN = 128 on S3, so 3 workgroups per CU), register-staged:
// the next stage's global loads are in flight during the MFMAs, then barrier / store / barrier.
// Requirements (host: conv_kernels.hip pick_win): cin % 16 == 0, W % CW == 0, N % BN == 0; rows past H in the
// last block row are computed on zeros and not stored.  Accumulation order differs from the im2col
// kernel (cb-major), so the two agree to rounding, not bit for bit.
#pragma once
#include "gemm_s3.hpp"
#include "gemm_ps.hpp"

namespace cad {

template <int R, int CW, int BN>
struct WinGeo {
    static constexpr int BM = R * CW;
    static constexpr int WC = CW + 2;              // window columns
    static constexpr int WPIX = R * WC;            // window pixels per stage
    static constexpr int NFA = WPIX * 4;           // A float4s per stage (16 channels = 4 float4)
    static constexpr int NVA = (NFA + 255) / 256;  // per thread
    static constexpr int NFB = 3 * BN * 4;         // B float4s per stage (3 taps x BN rows x 16 k)
    static_assert(NFB % 256 == 0, "BN");
    static constexpr int NVB = NFB / 256;
    static constexpr int PLA = WPIX * 16;          // bf16 elements per A plane
    static constexpr int PLB = BN * 16;            // bf16 elements per B plane (one tap)
};

// A: the input window of stage (cb, ky) of the block whose first output pixel is (b, y0, x0)
template <int R, int CW, int BN>
struct WinA {
    using G = WinGeo<R, CW, BN>;
    __amdgpu_buffer_rsrc_t rs;
    int poff[G::NVA];   // byte offset of the element at ky = 0, cb = 0 from the base (valid elements)
    int wr[G::NVA];     // window row of the element; a large negative value marks x / tail padding
    int H, y0, rowbytes, cb, ky;
    __device__ void init(const float* P, int64_t ld, int coff, int H_, int W, int b, int y0_, int x0, int tid,
                         int kbeg) {
        H = H_; y0 = y0_;
        const int ld4 = (int)ld * 4;
        rowbytes = W * ld4;
        const int64_t pbase = ((int64_t)b * H + y0 - 1) * W + x0 - 1;   // window pixel (0, 0) at ky = 0
        const int64_t pb = pbase > 0 ? pbase : 0;
        rs = make_rsrc(P + pb * ld + coff);
#pragma unroll
        for (int j = 0; j < G::NVA; ++j) {
            const int f = tid + 256 * j;
            const int w = f >> 2, q = f & 3;
            const int r = w / G::WC, c = w - r * G::WC;
            const int x = x0 - 1 + c;
            const bool ok = f < G::NFA && (unsigned)x < (unsigned)W;
            wr[j] = ok ? r : -(1 << 28);
            poff[j] = (int)((r * (int64_t)W + c + (pbase - pb)) * ld4) + q * 16;
        }
        cb = kbeg / 3;
        ky = kbeg - 3 * cb;
    }
    __device__ void load(float4 (&v)[G::NVA]) {
        const int add = ky * rowbytes + cb * 64;
#pragma unroll
        for (int j = 0; j < G::NVA; ++j) {
            const int y = y0 - 1 + ky + wr[j];
            v[j] = bload4(rs, (unsigned)y < (unsigned)H ? (uint32_t)(poff[j] + add) : kOOB);
        }
        if (++ky == 3) { ky = 0; ++cb; }
    }
};

// B: weights of the three taps (3ky + kx) of stage (cb, ky); Wt[n][tap*cin + ci], row stride ldb.
// Element f = tid + 256 j of a stage is (tap t, row, quarter q) with f = (t*BN + row)*4 + q; as 256
// divides BN*4, t and the row step are compile-time functions of j: one base offset per thread.
// The host guarantees N % BN == 0 (pick_win), so every row is in range.
template <int R, int CW, int BN>
struct WinB {
    using G = WinGeo<R, CW, BN>;
    static constexpr int JPT = BN * 4 / 256;   // j per tap
    __amdgpu_buffer_rsrc_t rs;
    int base, ldb4, cin4, cb, ky;
    __device__ void init(const float* Wt, int64_t ldb, int cin, int n0, int tid, int kbeg) {
        rs = make_rsrc(Wt + (int64_t)n0 * ldb);
        ldb4 = (int)ldb * 4;
        cin4 = cin * 4;
        base = (tid >> 2) * ldb4 + (tid & 3) * 16;
        cb = kbeg / 3;
        ky = kbeg - 3 * cb;
    }
    __device__ void load(float4 (&v)[G::NVB]) {
        const int add = base + 3 * ky * cin4 + cb * 64;
#pragma unroll
        for (int j = 0; j < G::NVB; ++j) {
            const int t = j / JPT, rstep = (j % JPT) * 64;   // 64 rows per 256 float4s
            v[j] = bload4(rs, (uint32_t)(add + rstep * ldb4 + t * cin4));
        }
        if (++ky == 3) { ky = 0; ++cb; }
    }
};

// Window epilogue: tile row mr -> output pixel (b, y0 + mr / CW, x0 + mr % CW), rows past H dropped.
// EpiStore / EpiStoreStats semantics of gemm_epilogue_t (stats row = the block's linear index).
// Timing experiments only (variant builds, `make VARIANT=... EXTRA=-DCAD_XP_WIN=k`; wrong outputs):
// 1 = no stores (the epilogue's store cost), 2 = no BN partials, 3 = neither.
#ifndef CAD_XP_WIN
#define CAD_XP_WIN 0
#endif
// BN-backward column sums of a window epilogue (EpiStoreBnSums): NB column blocks of CB (32 or 16)
// columns per lane; lanes whose lane % CB agree share a column.  y (the BN input) is read at the
// element the epilogue stores; the per-lane fp64 sums merge over lanes, then waves, into
// a.bn_part[tile][2][N] (EpiBnBwdSums' layout).
template <int NB, int CB, bool YB>
struct WinBnSums {
    double s0[NB], s1[NB];
    float sc[NB], sh[NB], mu[NB], is[NB];
    __amdgpu_buffer_rsrc_t ry;
    int64_t ldyb;   // bytes per y row
    __device__ void init(const GemmArgs& a, int b, int y0, int x0, int ncol0) {
        constexpr int YS = YB ? 2 : 4;
        ldyb = a.bn_ldg * YS;
        ry = make_rsrc(reinterpret_cast<const float*>(static_cast<const char*>(a.bn_g) +
                                                      (((int64_t)b * a.H + y0) * a.W + x0) * ldyb));
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int n = min(ncol0 + j * CB, a.N - 1);
            sc[j] = a.bn_scale[n]; sh[j] = a.bn_shift[n]; mu[j] = a.bn_mean[n]; is[j] = a.bn_invstd[n];
            s0[j] = 0.0; s1[j] = 0.0;
        }
    }
    // four rows of column n at pixel offset pix (r W + c) of the block, row stride one pixel row
    __device__ void load4(int64_t pix, int n, bool ok, float (&y)[4]) const {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t off = ok ? (uint32_t)((pix + q) * ldyb + (int64_t)n * (YB ? 2 : 4)) : kOOB;
            if constexpr (YB)
                y[q] = __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(ry, off, 0, 0) << 16);
            else
                y[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, off, 0, 0));
        }
    }
    __device__ void add(int j, float v, float y) {
        const float z = __fmaf_rn(y, sc[j], sh[j]);
        const float dz = z > 0.f ? v : 0.f;
        const float xh = (y - mu[j]) * is[j];
        s0[j] += dz;
        s1[j] += (double)dz * xh;
    }
    template <int WM, int WN>
    __device__ void finish(const GemmArgs& a, float* ldsf, int tile_x, int n0) {
        constexpr int BN = CB * NB * WN;
        double* lds = reinterpret_cast<double*>(ldsf);
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        const int wm = wave / WN, wn = wave % WN;
        __syncthreads();   // the LDS image may still be read by other waves' last fragments
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            double t0 = s0[j], t1 = s1[j];
#pragma unroll
            for (int x = CB; x < 64; x *= 2) {
                t0 += __shfl_xor(t0, x);
                t1 += __shfl_xor(t1, x);
            }
            if (lane < CB) {
                double* r = lds + ((int64_t)wm * BN + wn * CB * NB + j * CB + lane) * 2;
                r[0] = t0;
                r[1] = t1;
            }
        }
        __syncthreads();
        for (int c = tid; c < BN; c += 256) {
            double u0 = 0.0, u1 = 0.0;
#pragma unroll
            for (int w = 0; w < WM; ++w) {
                u0 += lds[((int64_t)w * BN + c) * 2];
                u1 += lds[((int64_t)w * BN + c) * 2 + 1];
            }
            const int n = n0 + c;
            if (n < a.N) {
                a.bn_part[((int64_t)tile_x * 2) * a.N + n] = u0;
                a.bn_part[((int64_t)tile_x * 2 + 1) * a.N + n] = u1;
            }
        }
    }
};
template <class Epi>
constexpr bool epi_y_bf16() {
    if constexpr (is_bnsums<Epi>::value) return Epi::Y_BF16;
    else return false;
}

template <int WM, int WN, int MI, int NJ, int CW, class Epi>
__device__ __forceinline__ void win_epilogue(const GemmArgs& a, const floatx16 (&acc)[MI][NJ], int tile_lin, int n0,
                                             int b, int y0, int x0, float* lds) {
    if constexpr (CAD_XP_WIN != 0) {
        if constexpr ((CAD_XP_WIN & 1) != 0 && ((CAD_XP_WIN & 2) != 0 || !Epi::STATS)) {
            // keep the accumulators live so the main loop is not removed
            float t = 0.f;
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int q = 0; q < 16; ++q) t += acc[i][j][q];
            if (t == 1234.5f) a.stats[0] = t;
            return;
        }
    }
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;   // (wave: uniform, SGPR)
    const int wm = wave / WN, wn = wave % WN;
    BnTilePartials<NJ> bnp;
    if constexpr (Epi::STATS) {
        bnp.init();
#pragma unroll
        for (int j = 0; j < NJ; ++j) bnp.shift(j, acc[0][j][0]);
    }
    constexpr bool BNS = is_bnsums<Epi>::value;
    [[maybe_unused]] WinBnSums<BNS ? NJ : 1, 32, epi_y_bf16<Epi>()> bns;
    if constexpr (BNS) bns.init(a, b, y0, x0, n0 + wn * 32 * NJ + (lane & 31));
    constexpr int ES = Epi::BF16 ? 2 : 4;   // output element bytes
    const int64_t ldc4 = a.ldc * ES;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const float*>(
        reinterpret_cast<const char*>(a.C) + ((((int64_t)b * a.H + y0) * a.W + x0) * a.ldc + a.c_coff) * ES));
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rs2;
    [[maybe_unused]] int64_t ldc2b = 0;
    if constexpr (Epi::SPLIT) {
        ldc2b = a.ldc2 * 2;
        rs2 = make_rsrc(reinterpret_cast<const float*>(static_cast<const char*>(a.C2) +
                                                       (((int64_t)b * a.H + y0) * a.W + x0) * ldc2b));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = n0 + wn * 32 * NJ + j * 32 + (lane & 31);
                const int mr = wm * 32 * MI + i * 32 + 4 * (lane >> 5) + 8 * g;   // 4 rows mr..mr+3: same r
                const int r = mr / CW, c = mr - r * CW;
                const bool ok = n < a.N && y0 + r < a.H;
                const uint32_t lo = ok ? (uint32_t)((r * (int64_t)a.W + c) * ldc4 + (int64_t)n * ES) : kOOB;
                float v[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = acc[i][j][4 * g + q];
                if constexpr (Epi::BF16) {   // the stored (rounded) values, which BN then normalises
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = (float)(__bf16)v[q];
                }
                if constexpr (BNS) {   // rows of one block row: r, c .. c + 3 (CW % 4 == 0); rows past H skipped
                    float yv[4];
                    bns.load4(r * (int64_t)a.W + c, n, ok, yv);
                    if (ok) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) bns.add(j, v[q], yv[q]);
                    }
                }
                if constexpr (Epi::SPLIT) {
                    // uniform per 32-column block (host: split_n % 32 == 0), tested on the block's first
                    // column so the compiler sees it: a per-lane test let it merge the two stores into one
                    // with a divergent descriptor (a readfirstlane loop around every store)
                    if (n0 + wn * 32 * NJ + j * 32 >= a.split_n) {
                        const uint32_t lo2 =
                            ok ? (uint32_t)((r * (int64_t)a.W + c) * ldc2b + (int64_t)(n - a.split_n) * 2) : kOOB;
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (__bf16)v[q]), rs2,
                                                                  lo2 + (uint32_t)(q * ldc2b), 0, 0);
                        continue;
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if constexpr ((CAD_XP_WIN & 1) == 0) {
                        if constexpr (Epi::BF16)
                            __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (__bf16)v[q]), rs,
                                                                  lo + (uint32_t)(q * ldc4), 0, 0);
                        else
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[q]), rs,
                                                                  lo + (uint32_t)(q * ldc4), 0, 0);
                    }
                    if constexpr (Epi::STATS && (CAD_XP_WIN & 2) == 0) bnp.add(j, v[q], y0 + r < a.H);
                }
            }
        }
    if constexpr (Epi::STATS && (CAD_XP_WIN & 2) == 0) bnp.template finish<WM, WN>(a, lds, tile_lin, n0);
    if constexpr (BNS) bns.template finish<WM, WN>(a, lds, tile_lin, n0);
}

// The same epilogue for 16 x 16 accumulator blocks (v_mfma_f32_16x16x32_bf16): a wave's MB x NB
// blocks; block (i, j) register q of a lane is output row 16 i + 4 (lane >> 4) + q, column
// 16 j + (lane & 15) of the wave's sub-tile.
template <int WM, int WN, int MB, int NB, int CW, class Epi>
__device__ __forceinline__ void win_epilogue16(const GemmArgs& a, const floatx4 (&acc)[MB][NB], int tile_lin, int n0,
                                               int b, int y0, int x0, float* lds) {
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;   // (wave: uniform, SGPR)
    const int wm = wave / WN, wn = wave % WN;
    BnTilePartials16<NB> bnp;
    if constexpr (Epi::STATS) {
        bnp.init();
#pragma unroll
        for (int j = 0; j < NB; ++j) bnp.shift(j, acc[0][j][0]);
    }
    constexpr bool BNS = is_bnsums<Epi>::value;
    [[maybe_unused]] WinBnSums<BNS ? NB : 1, 16, epi_y_bf16<Epi>()> bns;
    if constexpr (BNS) bns.init(a, b, y0, x0, n0 + wn * 16 * NB + (lane & 15));
    constexpr int ES = Epi::BF16 ? 2 : 4;
    const int64_t ldc4 = a.ldc * ES;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const float*>(
        reinterpret_cast<const char*>(a.C) + ((((int64_t)b * a.H + y0) * a.W + x0) * a.ldc + a.c_coff) * ES));
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rs2;
    [[maybe_unused]] int64_t ldc2b = 0;
    if constexpr (Epi::SPLIT) {
        ldc2b = a.ldc2 * 2;
        rs2 = make_rsrc(reinterpret_cast<const float*>(static_cast<const char*>(a.C2) +
                                                       (((int64_t)b * a.H + y0) * a.W + x0) * ldc2b));
    }
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int n = n0 + wn * 16 * NB + j * 16 + (lane & 15);
            const int mr = wm * 16 * MB + i * 16 + 4 * (lane >> 4);   // 4 rows mr..mr+3: same r
            const int r = mr / CW, c = mr - r * CW;
            const bool ok = n < a.N && y0 + r < a.H;
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = acc[i][j][q];
            if constexpr (Epi::BF16) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = (float)(__bf16)v[q];
            }
            if constexpr (Epi::SPLIT) {
                if (n0 + wn * 16 * NB + j * 16 >= a.split_n) {   // uniform per 16-column block (split_n % 32 == 0)
                    const uint32_t lo2 =
                        ok ? (uint32_t)((r * (int64_t)a.W + c) * ldc2b + (int64_t)(n - a.split_n) * 2) : kOOB;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (__bf16)v[q]), rs2,
                                                              lo2 + (uint32_t)(q * ldc2b), 0, 0);
                    continue;
                }
            }
            const uint32_t lo = ok ? (uint32_t)((r * (int64_t)a.W + c) * ldc4 + (int64_t)n * ES) : kOOB;
            if constexpr (BNS) {
                float yv[4];
                bns.load4(r * (int64_t)a.W + c, n, ok, yv);
                if (ok) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) bns.add(j, v[q], yv[q]);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if constexpr (Epi::BF16)
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (__bf16)v[q]), rs,
                                                          lo + (uint32_t)(q * ldc4), 0, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[q]), rs,
                                                          lo + (uint32_t)(q * ldc4), 0, 0);
                if constexpr (Epi::STATS) bnp.add(j, v[q], y0 + r < a.H);
            }
        }
    if constexpr (Epi::STATS) bnp.template finish<WM, WN>(a, lds, tile_lin, n0);
    if constexpr (BNS) bns.template finish<WM, WN>(a, lds, tile_lin, n0);
}

// blocks: gridDim.x = B * ceil(H / R) * (W / CW) output blocks (XCD-aware order), gridDim.y = N tiles
template <int NP, int R, int CW, int WM, int WN, class Epi>
__device__ __forceinline__ void conv3x3_win_body(const GemmArgs& a) {
    constexpr int MI = 2, NJ = 2;
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    static_assert(BM == R * CW, "tile");
    using G = WinGeo<R, CW, BN>;
    constexpr int SA = NP * G::PLA, SB = 3 * NP * G::PLB;   // bf16 elements
    __shared__ __attribute__((aligned(16))) uint16_t lds[SA + SB];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const TileId tile = xcd_tile();
    const int nbx = a.W / CW, nby = (a.H + R - 1) / R;
    const int tx = tile.x % nbx, t2 = tile.x / nbx, ty = t2 % nby, b = t2 / nby;
    const int y0 = ty * R, x0 = tx * CW, n0 = tile.y * BN;
    const int cin = a.a_cin;
    const int S = 3 * (cin / 16);   // stages

    WinA<R, CW, BN> la;
    WinB<R, CW, BN> lb;
    la.init(a.A, a.lda, a.a_coff, a.H, a.W, b, y0, x0, tid, 0);
    lb.init(a.Bm, a.ldb, cin, n0, tid, 0);

    // window pixel of the lane's A row in each of its MI blocks (tap kx adds kx)
    int wpix[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int p = wm * 32 * MI + i * 32 + (lane & 31);
        const int r = p / CW;
        wpix[i] = r * G::WC + (p - r * CW);
    }

    floatx16 acc[MI][NJ];
    acc_zero(acc);
    float4 ra[G::NVA], rb[G::NVB];

    auto store = [&]() {
#pragma unroll
        for (int j = 0; j < G::NVA; ++j) {
            const int f = tid + 256 * j;
            if (f < G::NFA) {
                const auto sp = split_np<NP>(ra[j]);
                const int off = s3_off<16>(f >> 2, (f & 3) * 4);
#pragma unroll
                for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(lds + p * G::PLA + off) = sp.p[p];
            }
        }
#pragma unroll
        for (int j = 0; j < G::NVB; ++j) {
            const int f = tid + 256 * j;
            const int t = f / (BN * 4), rem = f - t * (BN * 4);
            const auto sp = split_np<NP>(rb[j]);
            const int off = SA + t * NP * G::PLB + s3_off<16>(rem >> 2, (rem & 3) * 4);
#pragma unroll
            for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(lds + off + p * G::PLB) = sp.p[p];
        }
    };
    auto compute = [&]() {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            bf16x8 fa[MI][NP], fb[NJ][NP];
#pragma unroll
            for (int j = 0; j < NJ; ++j) s3_frag<BN, 16, NP>(lds + SA + kx * NP * G::PLB, wn * 32 * NJ + j * 32, 0, fb[j]);
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const uint16_t* base = lds + s3_off<16>(wpix[i] + kx, (lane >> 5) * 8);
#pragma unroll
                for (int p = 0; p < NP; ++p) fa[i][p] = *reinterpret_cast<const bf16x8*>(base + p * G::PLA);
            }
            s3_mfma<NP>(acc, fa, fb);
        }
    };

    if (S > 0) {
        la.load(ra);
        lb.load(rb);
        store();
    }
    __syncthreads();
    for (int s = 0; s < S; ++s) {
        const bool more = s + 1 < S;
        if (more) {
            la.load(ra);
            lb.load(rb);
        }
        compute();
        __syncthreads();
        if (more) {
            store();
            __syncthreads();
        }
    }
    win_epilogue<WM, WN, MI, NJ, CW, Epi>(a, acc, tile.x, n0, b, y0, x0, reinterpret_cast<float*>(lds));
}

// ------------------------------------------------------------------------------------------------
// B1 window kernel on pre-split operands (the bf16 twins of gemm_ps.hpp, NP = 1: plain NHWC bf16):
// the same blocks and window walk, with 32-channel stages (cb, ky) and no conversion at all — the
// loaders move 16-B pieces (8 channels) global -> registers -> LDS.  LDS images use the 80-B rows of
// S3<32> (conflict-free ds_read_b128): A window [R*(CW+2)][32] + B [3 taps][BN][32], one stage
// (41 KB for 128x128), 6 k16 steps x MI x NJ MFMAs per wave and stage.
// Requirements (host): A channels % 32 == 0, twin offsets % 8 == 0, W % CW == 0, N % BN == 0.
// ------------------------------------------------------------------------------------------------
template <int R, int CW, int BN>
struct WinPsGeo {
    static constexpr int WC = CW + 2;
    static constexpr int WPIX = R * WC;
    static constexpr int LDK = S3<32>::LDK;               // 40 bf16 per LDS row
    static constexpr int NTA = WPIX * 4;                   // A pieces per stage (4 x 8 channels per pixel)
    static constexpr int NVA = (NTA + 255) / 256;
    static constexpr int NTB = BN * 4;                     // B pieces per tap
    static constexpr int JB = (NTB + 255) / 256;
    static constexpr int SA = WPIX * LDK, SBT = BN * LDK;  // bf16 elements: A image, one tap of B
};

// MI = 4: 128 x 64 per wave (256 x 128 tiles) — two fragment reads per three MFMAs instead of one per
// MFMA: the 128 x 128 tile's LDS reads cap its MFMA rate near one half (B1 has one product per k step).
// NJ = 3 (with MI = 2, WM = 4, WN = 1): 256 x 96 tiles for the 96 / 192-channel levels of the
// reference's production width (train_config_production.yaml: init_features 96).
// M16: the same tile on v_mfma_f32_16x16x32_bf16 (2 MI x 2 NJ blocks of 16 x 16 per wave, one 32-deep
// k step per tap): the same LDS image, fragment reads and MFMA cycles per FLOP; the chip holds a
// higher clock on this shape under load (MI355X_MICROARCH.md, DVFS give-back item 7).
#ifndef CAD_WIN16
#define CAD_WIN16 0
#endif
template <int R, int CW, int WM, int WN, class Epi, int MI = 2, int NJ = 2, bool M16 = (CAD_WIN16 != 0)>
__device__ __forceinline__ void conv3x3_win_ps_body(const GemmArgs& a) {
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    static_assert(BM == R * CW, "tile");
    using G = WinPsGeo<R, CW, BN>;
    __shared__ __attribute__((aligned(16))) uint16_t lds[G::SA + 3 * G::SBT];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    // N tiles of one pixel block back to back on one XCD: its input window is fetched into that L2 once
    // (tools/winlab.py: forward 0.5 %, configs[3] step 0.55 %)
    const TileId tile = xcd_tile_yfast();
    const int nbx = a.W / CW, nby = (a.H + R - 1) / R;
    const int tx = tile.x % nbx, t2 = tile.x / nbx, ty = t2 % nby, b = t2 / nby;
    const int y0 = ty * R, x0 = tx * CW, n0 = tile.y * BN;
    const int H = a.H, W = a.W, cin = a.a_cin;
    const int S = 3 * (cin / 32);

    // A: bf16 rows of lda elements; piece (window pixel w, group g) of stage (cb, ky)
    const int rowb = (int)a.lda * 2;
    const int64_t pbase = ((int64_t)b * H + y0 - 1) * W + x0 - 1;
    const int64_t pb = pbase > 0 ? pbase : 0;
    const __amdgpu_buffer_rsrc_t rsa =
        make_rsrc(reinterpret_cast<const float*>(reinterpret_cast<const char*>(a.A) + (pb * a.lda + a.a_coff) * 2));
    // piece j = tid + 256 j is (window pixel w = j 64 + tid / 4, 16-B group tid % 4): its LDS slot is
    // a compile-time step from piece 0's; its global offset is kept per piece, and whether it lies
    // inside the image for each kernel row ky is bit 3 j + ky of amask (the per-piece registers of the
    // loop were the A operand's fragment budget: 250 VGPRs)
    static_assert(G::NVA <= 10, "amask: 3 bits per piece");
    int aoff[G::NVA];
    uint32_t amask = 0;
#pragma unroll
    for (int j = 0; j < G::NVA; ++j) {
        const int f = tid + 256 * j;
        const int w = f >> 2, g = f & 3;
        const int r = w / G::WC, c = w - r * G::WC;
        const int x = x0 - 1 + c;
        const bool okx = f < G::NTA && (unsigned)x < (unsigned)W;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
            if (okx && (unsigned)(y0 - 1 + ky + r) < (unsigned)H) amask |= 1u << (3 * j + ky);
        aoff[j] = (int)((r * (int64_t)W + c + (pbase - pb)) * rowb) + g * 16;
    }
    const int alds0 = (tid >> 2) * G::LDK + (tid & 3) * 8;   // piece j: + 64 j LDK
    // B: weight twin rows of ldb elements (ldb = 9*cin), piece (tap, row, group); piece jj = tid + 256 jj
    // is row 64 jj + tid / 4
    const int rowbb = (int)a.ldb * 2;
    const __amdgpu_buffer_rsrc_t rsb =
        make_rsrc(reinterpret_cast<const float*>(reinterpret_cast<const char*>(a.Bm) + ((int64_t)n0 * a.ldb + a.b_coff) * 2));
    const int boff0 = (tid >> 2) * rowbb + (tid & 3) * 16, blds0 = (tid >> 2) * G::LDK + (tid & 3) * 8;
    auto bact = [&](int jj) { return 256 * (jj + 1) <= G::NTB || tid + 256 * jj < G::NTB; };

    constexpr int MR = M16 ? 2 * MI : MI;   // A fragment row blocks per wave (32 or 16 rows)
    int wpix[MR];
#pragma unroll
    for (int i = 0; i < MR; ++i) {
        const int p = M16 ? wm * 32 * MI + i * 16 + (lane & 15) : wm * 32 * MI + i * 32 + (lane & 31);
        const int r = p / CW;
        wpix[i] = r * G::WC + (p - r * CW);
    }

    floatx16 acc[M16 ? 1 : MI][M16 ? 1 : NJ];
    floatx4 acc4[M16 ? 2 * MI : 1][M16 ? 2 * NJ : 1];
    if constexpr (M16) {
#pragma unroll
        for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
            for (int j = 0; j < 2 * NJ; ++j) acc4[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    } else {
        acc_zero(acc);
    }
    uint4 ra[G::NVA], rb[3 * G::JB];
    int cb = 0, ky = 0;
    auto load = [&]() {
        const int adda = ky * W * rowb + cb * 64;                   // 32 channels = 64 bytes
#pragma unroll
        for (int j = 0; j < G::NVA; ++j) {
            const bool in = (amask >> (3 * j + ky)) & 1u;
            ra[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rsa, in ? (uint32_t)(aoff[j] + adda) : kOOB, 0, 0));
        }
        const int addb = boff0 + 3 * ky * cin * 2 + cb * 64;
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int jj = 0; jj < G::JB; ++jj)
                if (bact(jj))
                    rb[t * G::JB + jj] = __builtin_bit_cast(
                        uint4, __builtin_amdgcn_raw_buffer_load_b128(rsb, (uint32_t)(addb + 64 * jj * rowbb + t * cin * 2), 0, 0));
        if (++ky == 3) { ky = 0; ++cb; }
    };
    auto store = [&]() {
#pragma unroll
        for (int j = 0; j < G::NVA; ++j)
            if (tid + 256 * j < G::NTA) *reinterpret_cast<uint4*>(lds + alds0 + 64 * j * G::LDK) = ra[j];
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int jj = 0; jj < G::JB; ++jj)
                if (bact(jj)) *reinterpret_cast<uint4*>(lds + G::SA + t * G::SBT + blds0 + 64 * jj * G::LDK) = rb[t * G::JB + jj];
    };
    auto compute = [&]() {
        if constexpr (M16) {
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                bf16x8 fb[2 * NJ];
#pragma unroll
                for (int j = 0; j < 2 * NJ; ++j)
                    fb[j] = *reinterpret_cast<const bf16x8*>(lds + G::SA + kx * G::SBT +
                                                             (wn * 32 * NJ + j * 16 + (lane & 15)) * G::LDK + (lane >> 4) * 8);
#pragma unroll
                for (int i = 0; i < 2 * MI; ++i) {
                    const bf16x8 fa = *reinterpret_cast<const bf16x8*>(lds + (wpix[i] + kx) * G::LDK + (lane >> 4) * 8);
#pragma unroll
                    for (int j = 0; j < 2 * NJ; ++j)
                        acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc4[i][j], 0, 0, 0);
                }
            }
        } else {
            // fragments of k step t + 1 read while the MFMAs of step t run (two register sets, the
            // schedule pinned by sched_barrier): hipcc's own schedule re-read each A fragment right
            // before its two MFMAs and waited on it (tools/winlab.py: 1-3 % on levels 0-2)
            bf16x8 fa[2][MI][1], fb[2][NJ][1];
            auto rd = [&](int t, int buf) {
                const int kx = t >> 1, q = t & 1;
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    s3_frag<BN, 32, 1>(lds + G::SA + kx * G::SBT, wn * 32 * NJ + j * 32, q, fb[buf][j]);
#pragma unroll
                for (int i = 0; i < MI; ++i)
                    fa[buf][i][0] = *reinterpret_cast<const bf16x8*>(lds + (wpix[i] + kx) * G::LDK + q * 16 + (lane >> 5) * 8);
            };
            rd(0, 0);
#pragma unroll
            for (int t = 0; t < 6; ++t) {
                if (t + 1 < 6) rd(t + 1, (t + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
                s3_mfma<1>(acc, fa[t & 1], fb[t & 1]);
                __builtin_amdgcn_sched_barrier(0);
            }
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
    if constexpr (M16)
        win_epilogue16<WM, WN, 2 * MI, 2 * NJ, CW, Epi>(a, acc4, tile.x, n0, b, y0, x0, reinterpret_cast<float*>(lds));
    else
        win_epilogue<WM, WN, MI, NJ, CW, Epi>(a, acc, tile.x, n0, b, y0, x0, reinterpret_cast<float*>(lds));
}

// ------------------------------------------------------------------------------------------------
// Window-tiled conv3x3 weight gradient (S3 / B1):  dW[co][tap][ci] = sum_pix dZ[pix][co] X[pix+tap][ci]
//
// The im2col weight-gradient GEMM (M = cout, N = 9*cin, K = pixels; MNcIm2col3x3) fetches and splits
// X once per tap and N tile.  Here a workgroup owns a 64 (co) x 64 (ci) channel pair over ALL nine
// taps (output 64 x 9 x 64) and a slice of K; a stage is 16 consecutive pixels of one image row:
//   A = dZ[16 px][64 co]                           MNc planes [16 k-rows][64]
//   B = X window rows y-1..y+1, columns x0-1..x0+16   MNc planes [3 x 18 k-rows][64]
// and tap (ky, kx) reads B's k-rows ky*18 + kx .. +15 (a k-row = a pixel, so the shift is a whole
// LDS row: the transposed ds_read_b64_tr_b16 fragment reads of gemm_s3.hpp apply unchanged).
// Wave w owns the 32x32 (co, ci) block (w & 1, w >> 1) for all nine taps: 9 accumulators, one A and
// nine B fragments per k16 step, 9 x NP products.  Per stage: 1024 + 3456 elements fetched and split
// for 64 x 576 x 16 MACs (the im2col kernel: 5120 per 64 x 256 x 16).  Double-buffered LDS (2 x 40 KB
// on S3: 2 workgroups per CU, the register budget's occupancy as well).  Split-K slices of whole
// stages write slabs (EpiSlab layout) reduced by the host's deterministic slab reduction.
// Requirements (host): cout % 64 == 0, cin % 64 == 0, W % 16 == 0.
// ------------------------------------------------------------------------------------------------
constexpr int kWgRows = 64;                      // channels per operand block
constexpr int kWgWinK = 3 * 18;                  // B window k-rows
using WgM = S3M<kWgRows>;                        // 64-column planes: 192 B per k-row (padded)

template <int ROWS, int NP>
__device__ __forceinline__ void mnc_frag_at(const char* s, int plane_bytes, int rb, int krow0, bf16x8 (&f)[NP]) {
    const int lane = threadIdx.x & 63;
    const int g = (lane >> 4) & 1, h = lane >> 5, i = lane & 15;
    const int krow = krow0 + 8 * h + (i >> 2);
    const int col = rb + 16 * g + 4 * (i & 3);
    const char* b0 = s + S3M<ROWS>::off(krow, col);
    const char* b1 = s + S3M<ROWS>::off(krow + 4, col);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        typedef __attribute__((address_space(3))) v4i16 lds_v4;
        const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(b0 + p * plane_bytes));
        const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(b1 + p * plane_bytes));
        const uint2 ul = __builtin_bit_cast(uint2, lo), uh = __builtin_bit_cast(uint2, hi);
        f[p] = __builtin_bit_cast(bf16x8, make_uint4(ul.x, ul.y, uh.x, uh.y));
    }
}

// pixel walk of a K-slice: stage s = 16 pixels (x0 .. x0+15) of row y of image b
struct WgPos {
    int b, y, x0;
    __device__ void init(int stage, int H, int W) {
        const int segs = W >> 4;
        const int row = stage / segs;
        x0 = (stage - row * segs) << 4;
        y = row % H;
        b = row / H;
    }
    __device__ void next(int H, int W) {
        x0 += 16;
        if (x0 == W) { x0 = 0; if (++y == H) { y = 0; ++b; } }
    }
};

template <int NP>
__device__ __forceinline__ void conv3x3_wgrad_win_body(const GemmArgs& a) {
    constexpr int PLA = 16 * WgM::STRIDE, PLB = kWgWinK * WgM::STRIDE;   // plane bytes
    constexpr int SA = NP * PLA, SB = NP * PLB;
    constexpr int NVB = (kWgWinK * 16 + 255) / 256;   // 16 float4 per k-row of 64 channels
    __shared__ __attribute__((aligned(16))) char lds[2 * (SA + SB)];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int cbk = wave & 1, cib = wave >> 1;
    const TileId tile = xcd_tile();
    const int co0 = tile.x * 64, ci0 = tile.y * 64;
    const int H = a.H, W = a.W;
    const int nst = (a.K) >> 4;                        // stages (K = B*H*W, W % 16 == 0)
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nst, kbeg + a.kstages_per_split);
    const int cin = a.b_cin;

    // operand bases: the slice's first pixel minus one row and one pixel (the window's reach back)
    const int64_t p0 = (int64_t)kbeg * 16;
    const int64_t pb = p0 - W - 1 > 0 ? p0 - W - 1 : 0;
    const int lda4 = (int)a.lda * 4, ldb4 = (int)a.ldb * 4;
    const __amdgpu_buffer_rsrc_t rsa = make_rsrc(a.A + p0 * a.lda + a.a_coff + co0);
    const __amdgpu_buffer_rsrc_t rsb = make_rsrc(a.Bm + pb * a.ldb + a.b_coff + ci0);
    // A: thread owns k-row tid/16 (pixel), columns 4(tid%16)..+3
    const uint32_t aoff = (uint32_t)((tid >> 4) * lda4 + (tid & 15) * 16);
    // B: element f = tid + 256 j -> window k-row kr = f/16 (ky = kr/18, kk = kr%18), column group f%16
    int brel[NVB], bky[NVB], bkk[NVB];
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
        const int f = tid + 256 * j;
        const int kr = f >> 4;
        const bool in = kr < kWgWinK;
        bky[j] = in ? kr / 18 : -(1 << 28);   // out-of-window slots: never in range
        bkk[j] = kr - (kr / 18) * 18;
        brel[j] = in ? ((kr / 18 - 1) * W + bkk[j] - 1) * ldb4 + (f & 15) * 16 : 0;
    }

    floatx16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    WgPos pos;
    pos.init(kbeg, H, W);
    float4 ra, rb[NVB];
    auto load = [&]() {
        const int64_t pix = ((int64_t)pos.b * H + pos.y) * W + pos.x0;   // first pixel of the stage
        ra = bload4(rsa, (uint32_t)((pix - p0) * lda4) + aoff);
        const int sb = (int)((pix - pb) * ldb4);
#pragma unroll
        for (int j = 0; j < NVB; ++j) {
            const int yy = pos.y + bky[j] - 1, xx = pos.x0 + bkk[j] - 1;
            const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            rb[j] = bload4(rsb, ok ? (uint32_t)(sb + brel[j]) : kOOB);
        }
        pos.next(H, W);
    };
    auto store = [&](int buf) {
        char* da = lds + buf * (SA + SB);
        {
            const auto sp = split_np<NP>(ra);
            const int off = WgM::off(tid >> 4, (tid & 15) * 4);
#pragma unroll
            for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(da + p * PLA + off) = sp.p[p];
        }
#pragma unroll
        for (int j = 0; j < NVB; ++j) {
            const int f = tid + 256 * j;
            if ((f >> 4) < kWgWinK) {
                const auto sp = split_np<NP>(rb[j]);
                const int off = WgM::off(f >> 4, (f & 15) * 4);
#pragma unroll
                for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(da + SA + p * PLB + off) = sp.p[p];
            }
        }
    };
    auto compute = [&](int buf) {
        const char* sa = lds + buf * (SA + SB);
        const char* sb = sa + SA;
        bf16x8 fa[1][NP];
        mnc_frag_at<kWgRows, NP>(sa, PLA, cbk * 32, 0, fa[0]);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            bf16x8 fb[NP];
            mnc_frag_at<kWgRows, NP>(sb, PLB, cib * 32, (t / 3) * 18 + (t % 3), fb);
            if constexpr (NP == 3) {   // the six products of s3_mfma, smallest first
                constexpr int P[6] = {2, 1, 0, 1, 0, 0};
                constexpr int Q[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
                for (int u = 0; u < 6; ++u)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][P[u]], fb[Q[u]], acc[t], 0, 0, 0);
            } else {
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][0], fb[0], acc[t], 0, 0, 0);
            }
        }
    };

    if (kbeg < kend) {
        load();
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        if (more) load();
        compute(cur);
        if (more) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    // slab z: C[z][co][tap*cin + ci] (row stride a.ldc = 9*cin)
    const int lane = tid & 63;
    float* dst = a.C + (int64_t)tile.z * a.slab_stride;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = t * cin + ci0 + cib * 32 + (lane & 31);
            const int co = co0 + cbk * 32 + 4 * (lane >> 5) + 8 * g;
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[(int64_t)(co + q) * a.ldc + n] = acc[t][4 * g + q];
        }
}


// ------------------------------------------------------------------------------------------------
// The same weight gradient with the stages walked down 16-pixel-wide column strips (round 4): stage s
// = pixels x0..x0+15 of row y, y fastest, so consecutive stages share two of their three window rows.
// The window rows live in a ring of four 18-pixel row slots (row yy in slot (yy + 1) & 3): a stage
// fetches and splits ONE new row (rows y'-1..y'+1 at a strip's start or a slice's first stage),
// against three in the row-major walk, whose re-fetches 40 stages apart missed a 4 MB XCD L2 shared
// by ~64 workgroups (FETCH_SIZE 7.9 GB per level-0 launch against 2.4 GB of operands).  LDS: A double-
// buffered (2 x 9 KB) + the ring (4 x 18 k-rows x NP planes = 41 KB on S3): 59 KB, two workgroups per
// CU.  Same products per (co, tap, ci) and pixel; the sums run in strip order (a different fp32 order
// than the row-major walk: both are deterministic).
// The host's window: a slice's operand span (its images, from the first image's start) below 2 GB.
// ------------------------------------------------------------------------------------------------
struct WgStrip {
    int b, seg, y;
    __device__ void init(int stage, int H, int W) {
        const int per_img = (W >> 4) * H;
        b = stage / per_img;
        const int r = stage - b * per_img;
        seg = r / H;
        y = r - seg * H;
    }
    __device__ void next(int H, int W) {
        if (++y == H) { y = 0; if (++seg == (W >> 4)) { seg = 0; ++b; } }
    }
};

template <int NP>
__device__ __forceinline__ void conv3x3_wgrad_strip_body(const GemmArgs& a) {
    constexpr int PLA = 16 * WgM::STRIDE;
    constexpr int SLOT = 18 * WgM::STRIDE;              // one window row, one plane
    constexpr int PLB = 4 * SLOT;                        // the ring, one plane
    constexpr int SA = NP * PLA, SB = NP * PLB;
    constexpr int NVR = (18 * 16 + 255) / 256;           // float4 per thread per window row (288 per row)
    __shared__ __attribute__((aligned(16))) char lds[2 * SA + SB];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int cbk = wave & 1, cib = wave >> 1;
    const TileId tile = xcd_tile();
    const int co0 = tile.x * 64, ci0 = tile.y * 64;
    const int H = a.H, W = a.W;
    const int nst = a.K >> 4;
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nst, kbeg + a.kstages_per_split);

    WgStrip pos;
    pos.init(min(kbeg, nst - 1), H, W);
    // operand bases: the slice's first image start (A), minus one row and one pixel (B)
    const int64_t p0 = (int64_t)pos.b * H * W;
    const int64_t pb = p0 - W - 1 > 0 ? p0 - W - 1 : 0;
    const int lda4 = (int)a.lda * 4, ldb4 = (int)a.ldb * 4;
    const __amdgpu_buffer_rsrc_t rsa = make_rsrc(a.A + p0 * a.lda + a.a_coff + co0);
    const __amdgpu_buffer_rsrc_t rsb = make_rsrc(a.Bm + pb * a.ldb + a.b_coff + ci0);
    const uint32_t aoff = (uint32_t)((tid >> 4) * lda4 + (tid & 15) * 16);
    // window-row element f = tid + 256 j: pixel kk = f / 16 (x0 - 1 + kk), column group f % 16
    int bkk[NVR];
    bool bin[NVR];
#pragma unroll
    for (int j = 0; j < NVR; ++j) {
        const int f = tid + 256 * j;
        bin[j] = f < 18 * 16;
        bkk[j] = f >> 4;
    }

    floatx16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    float4 ra, rb[3][NVR];
    auto load_a = [&](const WgStrip& q) {
        const int64_t pix = ((int64_t)q.b * H + q.y) * W + q.seg * 16;
        ra = bload4(rsa, (uint32_t)((pix - p0) * lda4) + aoff);
    };
    auto load_row = [&](const WgStrip& q, int yy, float4 (&r)[NVR]) {
        const int64_t pix = ((int64_t)q.b * H + yy) * W + q.seg * 16 - 1;   // window pixel kk = 0
        const bool rowok = (unsigned)yy < (unsigned)H;
#pragma unroll
        for (int j = 0; j < NVR; ++j) {
            const int xx = q.seg * 16 + bkk[j] - 1;
            const bool ok = bin[j] && rowok && (unsigned)xx < (unsigned)W;
            r[j] = bload4(rsb, ok ? (uint32_t)((pix + bkk[j] - pb) * ldb4 + (tid & 15) * 16) : kOOB);
        }
    };
    auto store_a = [&](int buf) {
        const auto sp = split_np<NP>(ra);
        const int off = WgM::off(tid >> 4, (tid & 15) * 4);
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(lds + buf * SA + p * PLA + off) = sp.p[p];
    };
    auto store_row = [&](int yy, const float4 (&r)[NVR]) {
        char* d = lds + 2 * SA + ((yy + 1) & 3) * SLOT;
#pragma unroll
        for (int j = 0; j < NVR; ++j)
            if (bin[j]) {
                const auto sp = split_np<NP>(r[j]);
                const int off = WgM::off(bkk[j], (tid & 15) * 4);
#pragma unroll
                for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(d + p * PLB + off) = sp.p[p];
            }
    };
    auto compute = [&](int buf, int y) {
        const char* sa = lds + buf * SA;
        const char* sb = lds + 2 * SA;
        bf16x8 fa[1][NP];
        mnc_frag_at<kWgRows, NP>(sa, PLA, cbk * 32, 0, fa[0]);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const int slot = (y + ky) & 3;   // row y + ky - 1
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int t = ky * 3 + kx;
                bf16x8 fb[NP];
                mnc_frag_at<kWgRows, NP>(sb, PLB, cib * 32, slot * 18 + kx, fb);
                if constexpr (NP == 3) {   // the six products of s3_mfma, smallest first
                    constexpr int P[6] = {2, 1, 0, 1, 0, 0};
                    constexpr int Q[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
                    for (int u = 0; u < 6; ++u)
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][P[u]], fb[Q[u]], acc[t], 0, 0, 0);
                } else {
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][0], fb[0], acc[t], 0, 0, 0);
                }
            }
        }
    };

    if (kbeg < kend) {   // (uniform; an empty slice writes a zero slab)
    // prologue: A and the three window rows of the first stage
    load_a(pos);
#pragma unroll
    for (int k = 0; k < 3; ++k) load_row(pos, pos.y - 1 + k, rb[k]);
    store_a(0);
#pragma unroll
    for (int k = 0; k < 3; ++k) store_row(pos.y - 1 + k, rb[k]);
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        WgStrip nx = pos;
        nx.next(H, W);
        const bool fresh = nx.y == 0;   // a new strip: three rows (uniform)
        if (more) {
            load_a(nx);
            if (fresh) {
#pragma unroll
                for (int k = 0; k < 3; ++k) load_row(nx, k - 1, rb[k]);
            } else {
                load_row(nx, nx.y + 1, rb[0]);
            }
        }
        compute(cur, pos.y);
        if (more) {
            store_a(cur ^ 1);
            if (fresh) {
                __syncthreads();   // the ring slots of the finished strip may still be read
#pragma unroll
                for (int k = 0; k < 3; ++k) store_row(k - 1, rb[k]);
            } else {
                store_row(nx.y + 1, rb[0]);   // slot of row y - 2: free since the last barrier
            }
        }
        __syncthreads();
        cur ^= 1;
        pos = nx;
    }
    }
    // slab z: C[z][co][tap*cin + ci] (row stride a.ldc = 9*cin)
    const int lane = tid & 63;
    float* dst = a.C + (int64_t)tile.z * a.slab_stride;
    const int cin = a.b_cin;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = t * cin + ci0 + cib * 32 + (lane & 31);
            const int co = co0 + cbk * 32 + 4 * (lane >> 5) + 8 * g;
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[(int64_t)(co + q) * a.ldc + n] = acc[t][4 * g + q];
        }
}

// ------------------------------------------------------------------------------------------------
// B1 window weight gradient on the bf16 twins (pre-split, NP = 1: plain NHWC bf16 rows).  The same
// decomposition as conv3x3_wgrad_win_body — a workgroup owns a 64 (co) x 64 (ci) channel pair over all
// nine taps and a split-K slice; wave w the 32x32 block (w & 1, w >> 1) of every tap — with stages of
// P pixels of one image row (P/16 k16 steps: 9 P/16 MFMAs per wave and barrier) and no conversion:
// the loaders move 16-B pieces (8 channels) global -> registers -> LDS.
//   A = dZ[P px][64 co]                  planes [P k-rows][64]        (S3M<64>: 192-B k-rows)
//   B = X rows y-1..y+1 x (P+2) px x 64 ci  planes [3 (P+2) k-rows][64]
// Tap (ky, kx) reads B's k-rows ky (P+2) + kx + 16 s .. of k16 step s (ds_read_b64_tr_b16 fragments).
// Per stage 64 P + 192 (P+2) elements for 64 x 576 x P MACs: X is fetched once per pixel and co-block
// (the im2col GEMM fetches it once per tap).  Requirements (host): cout, cin % 64, W % P, twin
// channel offsets % 8.
// ------------------------------------------------------------------------------------------------
template <int P>
__device__ __forceinline__ void conv3x3_wgrad_win_ps_body(const GemmArgs& a) {
    static_assert(P % 16 == 0, "stage");
    constexpr int KW = 3 * (P + 2);                    // B window k-rows
    constexpr int PLA = P * WgM::STRIDE, PLB = KW * WgM::STRIDE;   // bytes per operand image
    constexpr int NCA = P * 8, NCB = KW * 8;           // 16-B pieces (8 channels) per stage
    constexpr int NVA = (NCA + 255) / 256, NVB = (NCB + 255) / 256;
    __shared__ __attribute__((aligned(16))) char lds[2 * (PLA + PLB)];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int cbk = wave & 1, cib = wave >> 1;
    const TileId tile = xcd_tile();
    const int co0 = tile.x * 64, ci0 = tile.y * 64;
    const int H = a.H, W = a.W;
    const int nst = a.K / P;                           // stages (K = B*H*W, W % P == 0)
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nst, kbeg + a.kstages_per_split);
    const int segs = W / P;

    // operand bases: the slice's first pixel (A) / minus one row and one pixel (B, the window's reach)
    const int64_t p0 = (int64_t)kbeg * P;
    const int64_t pb = p0 - W - 1 > 0 ? p0 - W - 1 : 0;
    const int rowA = (int)a.lda * 2, rowB = (int)a.ldb * 2;   // bytes per twin row
    const __amdgpu_buffer_rsrc_t rsa =
        make_rsrc(ps_at(a.A, (p0 * a.lda + a.a_coff + co0) * 2));
    const __amdgpu_buffer_rsrc_t rsb =
        make_rsrc(ps_at(a.Bm, (pb * a.ldb + a.b_coff + ci0) * 2));
    int aoff[NVA], alds[NVA];
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
        const int f = tid + 256 * j;
        const int kr = f >> 3, g = f & 7;
        aoff[j] = f < NCA ? kr * rowA + g * 16 : -1;
        alds[j] = WgM::off(f < NCA ? kr : 0, g * 8);
    }
    int brel[NVB], bky[NVB], bkk[NVB], blds[NVB];
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
        const int f = tid + 256 * j;
        const int kr = f >> 3, g = f & 7;
        const bool in = f < NCB;
        bky[j] = in ? kr / (P + 2) : -(1 << 28);        // out-of-window slots: never in range
        bkk[j] = in ? kr - (kr / (P + 2)) * (P + 2) : 0;
        brel[j] = in ? ((bky[j] - 1) * W + bkk[j] - 1) * rowB + g * 16 : 0;
        blds[j] = WgM::off(in ? kr : 0, g * 8);
    }

    floatx16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    // stage position: pixels x0 .. x0+P-1 of row y of image b
    int sb_ = 0, sy = 0, sx0 = 0;
    {
        const int row = kbeg / segs;
        sx0 = (kbeg - row * segs) * P;
        sy = row % H;
        sb_ = row / H;
    }
    uint4 ra[NVA], rb[NVB];
    auto load = [&]() {
        const int64_t pix = ((int64_t)sb_ * H + sy) * W + sx0;
#pragma unroll
        for (int j = 0; j < NVA; ++j)
            ra[j] = bload16(rsa, aoff[j] >= 0 ? (uint32_t)((pix - p0) * rowA) + (uint32_t)aoff[j] : kOOB);
        const int sbase = (int)((pix - pb) * rowB);
#pragma unroll
        for (int j = 0; j < NVB; ++j) {
            const int yy = sy + bky[j] - 1, xx = sx0 + bkk[j] - 1;
            const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            rb[j] = bload16(rsb, ok ? (uint32_t)(sbase + brel[j]) : kOOB);
        }
        sx0 += P;
        if (sx0 == W) { sx0 = 0; if (++sy == H) { sy = 0; ++sb_; } }
    };
    auto store = [&](int buf) {
        char* da = lds + buf * (PLA + PLB);
#pragma unroll
        for (int j = 0; j < NVA; ++j)
            if (NCA % 256 == 0 || tid + 256 * j < NCA) *reinterpret_cast<uint4*>(da + alds[j]) = ra[j];
#pragma unroll
        for (int j = 0; j < NVB; ++j)
            if (NCB % 256 == 0 || tid + 256 * j < NCB) *reinterpret_cast<uint4*>(da + PLA + blds[j]) = rb[j];
    };
    auto compute = [&](int buf) {
        const char* sa = lds + buf * (PLA + PLB);
        const char* sb = sa + PLA;
#pragma unroll
        for (int q = 0; q < P / 16; ++q) {
            bf16x8 fa[1];
            mnc_frag_at<kWgRows, 1>(sa, PLA, cbk * 32, 16 * q, fa);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                bf16x8 fb[1];
                mnc_frag_at<kWgRows, 1>(sb, PLB, cib * 32, (t / 3) * (P + 2) + (t % 3) + 16 * q, fb);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[t], 0, 0, 0);
            }
        }
    };

    if (kbeg < kend) {
        load();
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        if (more) load();
        compute(cur);
        if (more) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    // slab z: C[z][co][tap*cin + ci] (row stride a.ldc = 9*cin)
    const int lane = tid & 63;
    const int cin = a.b_cin;
    float* dst = a.C + (int64_t)tile.z * a.slab_stride;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = t * cin + ci0 + cib * 32 + (lane & 31);
            const int co = co0 + cbk * 32 + 4 * (lane >> 5) + 8 * g;
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[(int64_t)(co + q) * a.ldc + n] = acc[t][4 * g + q];
        }
}


// ------------------------------------------------------------------------------------------------
// B1 window weight gradient with LDS-DMA staging (round 3).  The decomposition of
// conv3x3_wgrad_win_ps_body (64 co x 64 ci x 9 taps per workgroup, P-pixel stages of one image row),
// but the operands travel global -> LDS by buffer_load ... lds (no staging registers, no ds_write):
// one DMA wave-instruction moves 8 k-rows (pixels) x 128 B (64 channels) into a lane-linear LDS
// image of unpadded 128-B k-rows.  Bank conflicts of the transposed fragment reads
// (ds_read_b64_tr_b16: 4 consecutive k-rows x 64 B per 32-lane group; with 128-B rows, k-rows r and
// r + 2 would share banks) are removed by swizzling on the SOURCE side: LDS 16-B chunk c of k-row kr
// holds global chunk c ^ 4((kr >> 1) & 1), so any 4 consecutive k-rows cover disjoint bank ranges.
// A ring of NBUF = 3 stages keeps two stages in flight: iteration kt waits (counted vmcnt) for stage
// kt, passes ONE barrier (after which every wave has finished stage kt - 1, so its buffer is free),
// issues the DMA of stage kt + 2 into that buffer and computes stage kt.  Out-of-image halo pixels
// and the padding k-rows read past the buffer range: the DMA writes zeros for them.
// Per stage (P = 32): 4 + 13 DMA wave-instructions (17 KB), 18 MFMAs per wave; LDS 3 x 17 KB.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int wgd_off(int kr, int byte) {   // LDS byte of (k-row, byte in the row)
    return kr * 128 + ((((byte >> 4) ^ (((kr >> 1) & 1) << 2))) << 4) + (byte & 15);
}
__device__ __forceinline__ void wgd_frag(const char* s, int rb, int krow0, bf16x8& f) {
    const int lane = threadIdx.x & 63;
    const int g = (lane >> 4) & 1, h = lane >> 5, i = lane & 15;
    const int krow = krow0 + 8 * h + (i >> 2);
    const int byte = 2 * (rb + 16 * g + 4 * (i & 3));
    typedef __attribute__((address_space(3))) v4i16 lds_v4;
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(s + wgd_off(krow, byte)));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(s + wgd_off(krow + 4, byte)));
    const uint2 ul = __builtin_bit_cast(uint2, lo), uh = __builtin_bit_cast(uint2, hi);
    f = __builtin_bit_cast(bf16x8, make_uint4(ul.x, ul.y, uh.x, uh.y));
}
template <int P, int NBUF_ = 3>
struct WgdGeo {
    static constexpr int KW = 3 * (P + 2);            // B window k-rows
    static constexpr int NIA = P / 8;                 // DMA wave-instructions of A per stage
    static constexpr int NIB = (KW + 7) / 8;          // ... of B
    static constexpr int NI = NIA + NIB;
    static constexpr int SLOTS = (NI + 3) / 4;        // per wave (wave w issues j = w, w + 4, ...)
    static constexpr int WAIT = NI / 4;               // instructions every wave issues per stage
    static constexpr int SA = P * 128, SB = NIB * 8 * 128, STAGE = SA + SB;
    static constexpr int NBUF = NBUF_;   // 3: two stages in flight; 2: one (half the LDS)
};

// One LDS-DMA wave-instruction: buffer_load_dwordx4 ... lds (16 B per lane to M0 + 16 lane).  Issued
// by inline asm so the compiler's wait-count pass does not see it: otherwise, unable to prove that the
// fragment reads of the current ring slot do not alias the DMA's destination, it waits vmcnt(0)
// before them and drains the ring; the kernel counts these loads itself (wgd_wait_barrier).
typedef int i32x4_t __attribute__((ext_vector_type(4)));
struct DmaRsrc {
    i32x4_t d;
};
__device__ __forceinline__ DmaRsrc dma_rsrc(const void* base) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    DmaRsrc r;
    r.d[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r.d[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xFFFF));
    r.d[2] = (int)kRecords;
    r.d[3] = 0x00020000;
    return r;
}
__device__ __forceinline__ void dma16(const DmaRsrc& r, const void* lds_dst, uint32_t voff) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)lds_dst));
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r.d), "s"(m0)
                 : "memory", "m0");
}

template <int WAITN>
__device__ __forceinline__ void wgd_wait_barrier() {
    // the wave's DMAs of the stage about to be read have landed (at most WAITN newer ones pending),
    // then every wave's: a raw barrier (a __syncthreads fence would drain the in-flight DMAs too)
    if constexpr (WAITN == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(WAITN) : "memory");
}

template <int P, int NBUF = 3>
__device__ __forceinline__ void conv3x3_wgrad_win_dma_body(const GemmArgs& a) {
    static_assert(P % 16 == 0 && (NBUF == 2 || NBUF == 3), "stage / ring");
    using G = WgdGeo<P, NBUF>;
    __shared__ __attribute__((aligned(1024))) char lds[G::NBUF * G::STAGE];

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;   // (uniform: scalar branches)
    const int cbk = wave & 1, cib = wave >> 1;
    const TileId tile = xcd_tile();
    const int co0 = tile.x * 64, ci0 = tile.y * 64;
    const int H = a.H, W = a.W;
    const int nst = a.K / P;
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nst, kbeg + a.kstages_per_split);
    const int segs = W / P;

    const int64_t p0 = (int64_t)kbeg * P;
    const int64_t pb = p0 - W - 1 > 0 ? p0 - W - 1 : 0;
    const int rowA = (int)a.lda * 2, rowB = (int)a.ldb * 2;
    const DmaRsrc rsa = dma_rsrc(ps_at(a.A, (p0 * a.lda + a.a_coff + co0) * 2));
    const DmaRsrc rsb = dma_rsrc(ps_at(a.Bm, (pb * a.ldb + a.b_coff + ci0) * 2));

    // this wave's DMA slots: instruction j = wave + 4 t; lane -> k-row 8 j' + lane / 8, LDS chunk lane % 8
    const int lrow = lane >> 3, lch = lane & 7;
    int sj[G::SLOTS];        // instruction index (or -1)
    int soff[G::SLOTS];      // A: byte offset of the lane's piece from the stage's first pixel; B: relative window offset
    int sky[G::SLOTS], skk[G::SLOTS];
#pragma unroll
    for (int t = 0; t < G::SLOTS; ++t) {
        const int j = wave + 4 * t;
        sj[t] = j < G::NI ? j : -1;
        if (j < G::NIA) {
            const int kr = 8 * j + lrow;
            const int gch = lch ^ (((kr >> 1) & 1) << 2);
            soff[t] = kr * rowA + gch * 16;
            sky[t] = 0; skk[t] = 0;
        } else {
            const int kr = 8 * (j - G::NIA) + lrow;
            const int gch = lch ^ (((kr >> 1) & 1) << 2);
            const bool in = kr < G::KW;
            sky[t] = in ? kr / (P + 2) : -(1 << 28);   // padding k-rows: never in range
            skk[t] = in ? kr - (kr / (P + 2)) * (P + 2) : 0;
            soff[t] = in ? ((sky[t] - 1) * W + skk[t] - 1) * rowB + gch * 16 : 0;
        }
    }
    auto issue = [&](int stage, int buf) {   // DMA of stage `stage` (absolute) into ring slot buf
        const int row = stage / segs;
        const int sx0 = (stage - row * segs) * P, sy = row % H, sb = row / H;
        const int64_t pix = ((int64_t)sb * H + sy) * W + sx0;
        const uint32_t da = (uint32_t)((pix - p0) * rowA), db = (uint32_t)((pix - pb) * rowB);
        char* base = lds + buf * G::STAGE;
#pragma unroll
        for (int t = 0; t < G::SLOTS; ++t) {
            const int j = sj[t];
            if (j < 0) continue;   // wave-uniform
            if (j < G::NIA) {
                dma16(rsa, base + j * 1024, da + (uint32_t)soff[t]);
            } else {
                const int yy = sy + sky[t] - 1, xx = sx0 + skk[t] - 1;
                const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
                dma16(rsb, base + G::SA + (j - G::NIA) * 1024, ok ? db + (uint32_t)soff[t] : kOOB);
            }
        }
    };

    floatx16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    auto compute = [&](int buf) {
        const char* sa = lds + buf * G::STAGE;
        const char* sb = sa + G::SA;
#pragma unroll
        for (int q = 0; q < P / 16; ++q) {
            bf16x8 fa;
            wgd_frag(sa, cbk * 32, 16 * q, fa);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                bf16x8 fb;
                wgd_frag(sb, cib * 32, (t / 3) * (P + 2) + (t % 3) + 16 * q, fb);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[t], 0, 0, 0);
            }
        }
    };

    if (kbeg < kend) issue(kbeg, 0);
    if (NBUF == 3 && kbeg + 1 < kend) issue(kbeg + 1, 1);
    int buf = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        if (NBUF == 3 && kt + 1 < kend) wgd_wait_barrier<G::WAIT>();   // stage kt landed; kt + 1 may still fly
        else wgd_wait_barrier<0>();
        // the next DMA goes to the slot of stage kt - 1, which every wave has finished (barrier above)
        if (kt + NBUF - 1 < kend) issue(kt + NBUF - 1, buf == 0 ? NBUF - 1 : buf - 1);
        compute(buf);
        buf = buf == NBUF - 1 ? 0 : buf + 1;
    }
    // slab z: C[z][co][tap*cin + ci] (row stride a.ldc = 9*cin)
    const int cin = a.b_cin;
    float* dst = a.C + (int64_t)tile.z * a.slab_stride;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = t * cin + ci0 + cib * 32 + (lane & 31);
            const int co = co0 + cbk * 32 + 4 * (lane >> 5) + 8 * g;
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[(int64_t)(co + q) * a.ldc + n] = acc[t][4 * g + q];
        }
}


// ------------------------------------------------------------------------------------------------
// The LDS-DMA weight gradient walked down P-pixel-wide column strips (round 4; the strip order of
// conv3x3_wgrad_strip_body).  A slice is a sequence of STEPS: each step DMAs one window row (P + 2
// pixels, padded to whole 8-row DMA instructions) into a ring of 8 row slots (step i -> slot i & 7) and
// one A stage (dZ, P pixels) into a ring of NBUF = 3 stage slots; step i computes the stage whose
// rows came in steps i - 2, i - 1, i.  A strip (and the slice's first strip) opens with two steps that
// only load rows y0 - 1 and y0 (their A DMA reads the out-of-range offset: zeros, never read), so every
// step issues the same DMA instructions and the counted vmcnt of the round-3 kernel applies unchanged.
// Per stage: 1 + P/8 + ... = (P + 2)/8 + P/8 DMA instructions (9 at P = 32) against 3 (P + 2)/8 + P/8
// (17): X fetched once per strip (plus the 2-row preamble) instead of three times.
// ------------------------------------------------------------------------------------------------
template <int P>
struct WgsGeo {
    static constexpr int NIA = P / 8;                   // DMA instructions of A per step
    static constexpr int NIR = (P + 2 + 7) / 8;         // ... of one window row
    static constexpr int NI = NIA + NIR;
    static constexpr int SLOTS = (NI + 3) / 4;          // per wave
    static constexpr int WAIT = NI / 4;
    static constexpr int SA = P * 128, ROW = NIR * 8 * 128, KR = NIR * 8;   // bytes; k-rows per row slot
    static constexpr int NBUF = 3, NROW = 8;
};

template <int P>
__device__ __forceinline__ void conv3x3_wgrad_strip_dma_body(const GemmArgs& a) {
    static_assert(P % 16 == 0, "stage");
    using G = WgsGeo<P>;
    __shared__ __attribute__((aligned(1024))) char lds[G::NBUF * G::SA + G::NROW * G::ROW];
    char* const ldsB = lds + G::NBUF * G::SA;

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int cbk = wave & 1, cib = wave >> 1;
    const TileId tile = xcd_tile();
    const int co0 = tile.x * 64, ci0 = tile.y * 64;
    const int H = a.H, W = a.W;
    const int segs = W / P;
    const int nst = a.K / P;
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nst, kbeg + a.kstages_per_split);

    // strip walk: stage s -> strip s / H (= image b, column segment), row y = s % H
    const int s0 = min(kbeg, nst - 1);
    const int b0 = s0 / (segs * H);
    const int64_t p0 = (int64_t)b0 * H * W;   // the slice's first image (operand window base)
    const int64_t pb = p0 - W - 1 > 0 ? p0 - W - 1 : 0;
    const int rowA = (int)a.lda * 2, rowB = (int)a.ldb * 2;
    const DmaRsrc rsa = dma_rsrc(ps_at(a.A, (p0 * a.lda + a.a_coff + co0) * 2));
    const DmaRsrc rsb = dma_rsrc(ps_at(a.Bm, (pb * a.ldb + a.b_coff + ci0) * 2));

    const int lrow = lane >> 3, lch = lane & 7;
    int sj[G::SLOTS], soff[G::SLOTS], skr[G::SLOTS];
#pragma unroll
    for (int t = 0; t < G::SLOTS; ++t) {
        const int j = wave + 4 * t;
        sj[t] = j < G::NI ? j : -1;
        const int kr = 8 * (j < G::NIA ? j : j - G::NIA) + lrow;   // k-row within the A stage / row slot
        const int gch = lch ^ (((kr >> 1) & 1) << 2);
        skr[t] = kr;
        soff[t] = (j < G::NIA ? kr * rowA : (kr - 1) * rowB) + gch * 16;   // B: pixel x0 - 1 + kr
    }
    // steps: each strip of the slice contributes its stages + 2 (rows y0 - 1, y0 first)
    const int nsteps = kbeg < kend ? (kend - kbeg) + 2 * ((kend - 1) / H - kbeg / H + 1) : 0;
    // issue-side walk: strip index and the row the next step loads
    int w_strip = kbeg / H, w_row = kbeg % H - 1, w_ylo = kbeg % H;
    auto issue = [&](int step) {   // DMAs of the walk's current step into its slots, then advance
        const int sb = w_strip / segs, sx0 = (w_strip - sb * segs) * P;
        const int ya = w_row - 1;   // the stage this step computes (when >= w_ylo)
        const bool hasA = ya >= w_ylo;
        const int64_t rowpix = ((int64_t)sb * H + w_row) * W + sx0;
        const uint32_t da = hasA ? (uint32_t)((((int64_t)sb * H + ya) * W + sx0 - p0) * rowA) : 0u;
        const bool rowok = (unsigned)w_row < (unsigned)H;
        char* baseA = lds + (step % G::NBUF) * G::SA;
        char* baseB = ldsB + (step & (G::NROW - 1)) * G::ROW;
#pragma unroll
        for (int t = 0; t < G::SLOTS; ++t) {
            const int j = sj[t];
            if (j < 0) continue;   // wave-uniform
            if (j < G::NIA) {
                dma16(rsa, baseA + j * 1024, hasA ? da + (uint32_t)soff[t] : kOOB);
            } else {
                const int xx = sx0 + skr[t] - 1;
                const bool ok = rowok && skr[t] < P + 2 && (unsigned)xx < (unsigned)W;
                dma16(rsb, baseB + (j - G::NIA) * 1024,
                      ok ? (uint32_t)((rowpix - pb) * rowB) + (uint32_t)soff[t] : kOOB);
            }
        }
        // advance: the next row of this strip, or the next strip's preamble
        if (++w_row == H + 1) { ++w_strip; w_row = -1; w_ylo = 0; }
    };

    floatx16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    auto compute = [&](int step) {
        const char* sa = lds + (step % G::NBUF) * G::SA;
#pragma unroll
        for (int q = 0; q < P / 16; ++q) {
            bf16x8 fa;
            wgd_frag(sa, cbk * 32, 16 * q, fa);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const char* sr = ldsB + ((step - 2 + ky) & (G::NROW - 1)) * G::ROW;
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    bf16x8 fb;
                    wgd_frag(sr, cib * 32, kx + 16 * q, fb);
                    acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[ky * 3 + kx], 0, 0, 0);
                }
            }
        }
    };

    // compute steps: a step computes iff its A stage exists (bit step % NBUF of comp)
    int comp = 0;
    auto issue_step = [&](int step) {
        const int bit = 1 << (step % G::NBUF);
        comp = w_row - 1 >= w_ylo ? comp | bit : comp & ~bit;
        issue(step);
    };
    if (nsteps > 0) issue_step(0);
    if (nsteps > 1) issue_step(1);
    for (int i = 0; i < nsteps; ++i) {
        if (i + 1 < nsteps) wgd_wait_barrier<G::WAIT>();   // step i landed; i + 1 may still fly
        else wgd_wait_barrier<0>();
        const bool ci = (comp >> (i % G::NBUF)) & 1;   // (read before step i + 2 reuses the slot)
        // step i + 2 reuses the A slot of step i - 1 and the row slot of step i - 6: finished (barrier)
        if (i + 2 < nsteps) issue_step(i + 2);
        if (ci) compute(i);
    }
    // slab z: C[z][co][tap*cin + ci] (row stride a.ldc = 9*cin)
    const int cin = a.b_cin;
    float* dst = a.C + (int64_t)tile.z * a.slab_stride;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = t * cin + ci0 + cib * 32 + (lane & 31);
            const int co = co0 + cbk * 32 + 4 * (lane >> 5) + 8 * g;
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[(int64_t)(co + q) * a.ldc + n] = acc[t][4 * g + q];
        }
}

// ------------------------------------------------------------------------------------------------
// The same strip walk two output rows per step (round 5; P = 16 and 32).  One 16-pixel row per step left
// 9 MFMAs per wave between the DMA issue and the barrier (~0.40 MFMA-busy against 0.53 at P = 32); a
// stage is now a row PAIR (y, y + 1) of a strip: its step DMAs the two dZ rows and the window rows
// y + 1, y + 2 (rows y - 1, y came with the previous step, or with the strip's one-step preamble), so
// 18 (P = 16) or 36 (P = 32) MFMAs per wave share one barrier; within a K-slice each accumulator still
// takes the rows in order (slices now split at row pairs: the slab partials may differ from the one-row
// walk's by fp32 rounding).  Row slot of the
// window rows of step i: 2 i, 2 i + 1 (mod 8); output row y + q, kernel row ky reads slot 2 i - 2 + q + ky.
// Stage s -> strip s / HP, pair s % HP (HP = ceil(H / 2)); a pair's second row past H is DMA'd as zeros
// (its dZ is then 0 and adds nothing).  Host: kstages over B * (W / P) * HP pairs.
// ------------------------------------------------------------------------------------------------
template <int P>
struct Wgs2Geo {
    static constexpr int NIA = 2 * P / 8;               // DMA instructions of A per step (two dZ rows)
    static constexpr int NIR = (P + 2 + 7) / 8;         // ... of one window row
    static constexpr int NI = NIA + 2 * NIR;
    static constexpr int SLOTS = (NI + 3) / 4;          // per wave
    static constexpr int WAIT = NI / 4;
    static constexpr int SA = 2 * P * 128, ROW = NIR * 8 * 128;   // bytes
    static constexpr int NBUF = 3, NROW = 8;
};

template <int P>
__device__ __forceinline__ void conv3x3_wgrad_strip2_dma_body(const GemmArgs& a) {
    static_assert(P % 16 == 0, "stage");
    using G = Wgs2Geo<P>;
    __shared__ __attribute__((aligned(1024))) char lds[G::NBUF * G::SA + G::NROW * G::ROW];
    char* const ldsB = lds + G::NBUF * G::SA;

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int cbk = wave & 1, cib = wave >> 1;
    const TileId tile = xcd_tile();
    const int co0 = tile.x * 64, ci0 = tile.y * 64;
    const int H = a.H, W = a.W;
    const int segs = W / P, HP = (H + 1) / 2;
    const int nst = a.B * segs * HP;
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nst, kbeg + a.kstages_per_split);

    const int s0 = min(kbeg, nst - 1);
    const int b0 = s0 / (segs * HP);
    const int64_t p0 = (int64_t)b0 * H * W;   // the slice's first image (operand window base)
    const int64_t pb = p0 - W - 1 > 0 ? p0 - W - 1 : 0;
    const int rowA = (int)a.lda * 2, rowB = (int)a.ldb * 2;
    const DmaRsrc rsa = dma_rsrc(ps_at(a.A, (p0 * a.lda + a.a_coff + co0) * 2));
    const DmaRsrc rsb = dma_rsrc(ps_at(a.Bm, (pb * a.ldb + a.b_coff + ci0) * 2));

    // DMA slot t of this wave: instruction j = wave + 4 t; A (j < NIA): k-row kr of the two-row stage,
    // dZ row kr / P; window (j >= NIA): row rr of the step's two, k-row kr of that row slot
    const int lrow = lane >> 3, lch = lane & 7;
    int sj[G::SLOTS], soff[G::SLOTS], skr[G::SLOTS], srr[G::SLOTS];
#pragma unroll
    for (int t = 0; t < G::SLOTS; ++t) {
        const int j = wave + 4 * t;
        sj[t] = j < G::NI ? j : -1;
        if (j < G::NIA) {
            const int kr = 8 * j + lrow;
            const int gch = lch ^ (((kr >> 1) & 1) << 2);
            srr[t] = kr / P;
            skr[t] = kr;
            soff[t] = (srr[t] * W + kr - srr[t] * P) * rowA + gch * 16;
        } else {
            const int jj = j - G::NIA;
            const int rr = jj / G::NIR, kr = 8 * (jj - rr * G::NIR) + lrow;
            const int gch = lch ^ (((kr >> 1) & 1) << 2);
            srr[t] = rr;
            skr[t] = kr;
            soff[t] = (rr * W + kr - 1) * rowB + gch * 16;   // window pixel x0 - 1 + kr of row rr
        }
    }
    // steps: each strip of the slice opens with one preamble step (window rows y0 - 1, y0), then one
    // step per pair
    const int nsteps = kbeg < kend ? (kend - kbeg) + ((kend - 1) / HP - kbeg / HP + 1) : 0;
    int w_strip = kbeg / HP, w_pair = kbeg % HP;
    bool w_pre = true;
    int comp = 0;   // bit step % NBUF: the step computes (has an A stage)
    auto issue = [&](int step) {
        const int sb = w_strip / segs, sx0 = (w_strip - sb * segs) * P;
        const int y = 2 * w_pair;
        const int wr = w_pre ? y - 1 : y + 1;   // first window row this step loads
        const bool hasA = !w_pre;
        const int bit = 1 << (step % G::NBUF);
        comp = hasA ? comp | bit : comp & ~bit;
        const int64_t rowpix = ((int64_t)sb * H + wr) * W + sx0;
        const uint32_t da = hasA ? (uint32_t)((((int64_t)sb * H + y) * W + sx0 - p0) * rowA) : 0u;
        const uint32_t db = (uint32_t)((rowpix - pb) * rowB);
        char* baseA = lds + (step % G::NBUF) * G::SA;
#pragma unroll
        for (int t = 0; t < G::SLOTS; ++t) {
            const int j = sj[t];
            if (j < 0) continue;   // wave-uniform
            if (j < G::NIA) {
                const bool ok = hasA && y + srr[t] < H;
                dma16(rsa, baseA + j * 1024, ok ? da + (uint32_t)soff[t] : kOOB);
            } else {
                const int jj = j - G::NIA, rr = srr[t];
                const int xx = sx0 + skr[t] - 1;
                const bool ok = (unsigned)(wr + rr) < (unsigned)H && skr[t] < P + 2 && (unsigned)xx < (unsigned)W;
                char* dst = ldsB + ((2 * step + rr) & (G::NROW - 1)) * G::ROW + (jj - rr * G::NIR) * 1024;
                dma16(rsb, dst, ok ? db + (uint32_t)soff[t] : kOOB);
            }
        }
        // advance: the first pair after the preamble, the next pair, or the next strip's preamble
        if (w_pre) {
            w_pre = false;
        } else if (++w_pair == HP) {
            ++w_strip; w_pair = 0; w_pre = true;
        }
    };

    floatx16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    auto compute = [&](int step) {
        const char* sa = lds + (step % G::NBUF) * G::SA;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int qq = 0; qq < P / 16; ++qq) {
                bf16x8 fa;
                wgd_frag(sa, cbk * 32, q * P + 16 * qq, fa);
#pragma unroll
                for (int ky = 0; ky < 3; ++ky) {
                    const char* sr = ldsB + ((2 * step - 2 + q + ky) & (G::NROW - 1)) * G::ROW;
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) {
                        bf16x8 fb;
                        wgd_frag(sr, cib * 32, kx + 16 * qq, fb);
                        acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[ky * 3 + kx], 0, 0, 0);
                    }
                }
            }
    };

    if (nsteps > 0) issue(0);
    if (nsteps > 1) issue(1);
    for (int i = 0; i < nsteps; ++i) {
        if (i + 1 < nsteps) wgd_wait_barrier<G::WAIT>();   // step i landed; i + 1 may still fly
        else wgd_wait_barrier<0>();
        const bool ci = (comp >> (i % G::NBUF)) & 1;   // (read before step i + 2 reuses the slot)
        // step i + 2 reuses the A slot of step i - 1 and the row slots of steps i - 2 (rows 2 i - 4,
        // 2 i - 3), read last by step i - 1's compute: finished (barrier)
        if (i + 2 < nsteps) issue(i + 2);
        if (ci) compute(i);
    }
    // slab z: C[z][co][tap*cin + ci] (row stride a.ldc = 9*cin)
    const int cin = a.b_cin;
    float* dst = a.C + (int64_t)tile.z * a.slab_stride;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = t * cin + ci0 + cib * 32 + (lane & 31);
            const int co = co0 + cbk * 32 + 4 * (lane >> 5) + 8 * g;
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[(int64_t)(co + q) * a.ldc + n] = acc[t][4 * g + q];
        }
}

// LDS row image of the DMA kernels below: unpadded 64-B rows (32 bf16) whose 16-B chunk c of row w sits
// at c ^ ((w >> 2) & 3), the source-side swizzle that keeps the ds_read_b128 fragment reads of 16
// consecutive rows on disjoint banks.
__device__ __forceinline__ int wind_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// ------------------------------------------------------------------------------------------------
// Dense bf16 GEMM C[m][n] = sum_k A[m][k] B[n][k] with LDS-DMA staging (round 4): the ConvT forward
// (A = the low-res twin, K = cin) and config 5's dense forward GEMMs.  The register-staged gemm_body_ps keeps one stage in flight with 8 MFMAs per
// wave and stage (128 x 128): its load latency is exposed (the ConvT GEMMs ran at 430-630 TFLOP/s).
// Here a ring of 3 stages keeps two in flight with no staging registers (48 KB of LDS for 128 x 128:
// three workgroups per CU).  LDS rows are unpadded 64-B (32 bf16) with the source-side chunk swizzle
// (wind_off); a DMA wave-instruction fills 16 rows.  M / N tails and K tails
// (K % 8 == 0) read the out-of-range offset: zeros.
// ------------------------------------------------------------------------------------------------
template <int BM, int BN>
struct DenseDGeo {
    static constexpr int NIA = BM / 16, NIB = BN / 16, NI = NIA + NIB;
    static constexpr int SLOTS = (NI + 3) / 4, WAIT = NI / 4;
    static constexpr int SA = BM * 64, STAGE = (BM + BN) * 64, NBUF = 3;
};
template <int WM, int WN, int MI, int NJ, class Epi>
__device__ __forceinline__ void gemm_dense_dma_body(const GemmArgs& a) {
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    using G = DenseDGeo<BM, BN>;
    __shared__ __attribute__((aligned(1024))) char lds[G::NBUF * G::STAGE];

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const TileId tile = xcd_tile();
    const int m0 = tile.x * BM, n0 = tile.y * BN;
    const int K = a.K, S = (K + 31) / 32;
    const int rowa = (int)a.lda * 2, rowb = (int)a.ldb * 2;
    const int64_t abase = m0;
    const DmaRsrc rsa = dma_rsrc(reinterpret_cast<const char*>(a.A) + (abase * a.lda + a.a_coff) * 2);
    const DmaRsrc rsb = dma_rsrc(reinterpret_cast<const char*>(a.Bm) + ((int64_t)n0 * a.ldb + a.b_coff) * 2);

    const int lrow = lane >> 2, lch = lane & 3;
    int sj[G::SLOTS], soff[G::SLOTS], sch[G::SLOTS];
#pragma unroll
    for (int t = 0; t < G::SLOTS; ++t) {
        const int j = wave + 4 * t;
        sj[t] = j < G::NI ? j : -1;
        const int r = 16 * (j < G::NIA ? j : j - G::NIA) + lrow;
        const int gch = lch ^ ((r >> 2) & 3);
        sch[t] = 8 * gch;   // k offset of the lane's piece within the stage
        if (j < G::NIA) {
            const int m = m0 + r;
            soff[t] = m < a.M ? r * rowa + gch * 16 : -1;
        } else {
            soff[t] = n0 + r < a.N ? r * rowb + gch * 16 : -1;
        }
    }
    auto issue = [&](int stage, int buf) {
        const int k0 = stage * 32;
        const int adda = k0 * 2;
        char* base = lds + buf * G::STAGE;
#pragma unroll
        for (int t = 0; t < G::SLOTS; ++t) {
            const int j = sj[t];
            if (j < 0) continue;   // wave-uniform
            const bool ok = soff[t] >= 0 && k0 + sch[t] < K;
            if (j < G::NIA) dma16(rsa, base + j * 1024, ok ? (uint32_t)(soff[t] + adda) : kOOB);
            else dma16(rsb, base + G::SA + (j - G::NIA) * 1024, ok ? (uint32_t)(soff[t] + k0 * 2) : kOOB);
        }
    };

    floatx16 acc[MI][NJ];
    acc_zero(acc);
    const int h = lane >> 5;
    auto compute = [&](int buf) {
        const char* sa = lds + buf * G::STAGE;
        const char* sb = sa + G::SA;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            bf16x8 fa[MI][1], fb[NJ][1];
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                fb[j][0] = *reinterpret_cast<const bf16x8*>(sb + wind_off(wn * 32 * NJ + j * 32 + (lane & 31), 2 * q + h));
#pragma unroll
            for (int i = 0; i < MI; ++i)
                fa[i][0] = *reinterpret_cast<const bf16x8*>(sa + wind_off(wm * 32 * MI + i * 32 + (lane & 31), 2 * q + h));
            s3_mfma<1>(acc, fa, fb);
        }
    };

    if (S > 0) issue(0, 0);
    if (S > 1) issue(1, 1);
    int buf = 0;
    for (int s = 0; s < S; ++s) {
        if (s + 1 < S) wgd_wait_barrier<G::WAIT>();
        else wgd_wait_barrier<0>();
        if (s + 2 < S) issue(s + 2, buf == 0 ? G::NBUF - 1 : buf - 1);
        compute(buf);
        buf = buf == G::NBUF - 1 ? 0 : buf + 1;
    }
    __syncthreads();   // the ring is the epilogue's scratch
    gemm_epilogue_t<WM, WN, MI, NJ>(a, acc, tile, reinterpret_cast<float*>(lds), Epi{});
}

}  // namespace cad
