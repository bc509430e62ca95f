// MX-fp8 kernels (gemm_mx8.hpp) and their host launchers: the quantiser that writes MXFP8 operand
// twins, the dense (1x1 / im2col) forward GEMM and the window-tiled conv3x3 forward on them.  Used by
// the config-5 network's forward contractions (BASELINE.json configs[4]: "bf16 with fp8 MFMA
// conv-GEMM"; resunet.cpp, cad_resunet_set_fp8).  No reference counterpart.
#include <cstdio>
#include <stdexcept>

#include "epilogues.hpp"
#include "gemm_mx8.hpp"
#include "kernels.hpp"

namespace cad {

// one thread per (row, 32-element block): 32 source values -> 32 e4m3 bytes + one e8m0 byte
template <bool SRC_BF16>
__global__ void k_mx8_quantize(const void* __restrict__ src, int64_t lds, int scoff, int nblk, int64_t n,
                               uint8_t* __restrict__ q, int64_t ldq, int qcoff, uint8_t* __restrict__ s) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t row = i / nblk;
    const int blk = (int)(i - row * nblk);
    float v[32];
    if constexpr (SRC_BF16) {
        const uint4* p = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(src) + row * lds + scoff + 32 * blk);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 u = p[j];
            const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[8 * j + 2 * e] = __uint_as_float(w[e] << 16);
                v[8 * j + 2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
            }
        }
    } else {
        const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(src) + row * lds + scoff + 32 * blk);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float4 f = p[j];
            v[4 * j] = f.x; v[4 * j + 1] = f.y; v[4 * j + 2] = f.z; v[4 * j + 3] = f.w;
        }
    }
    uint32_t w[8];
    const uint32_t sc = mx8_quant_block(v, w);
    uint4* d = reinterpret_cast<uint4*>(q + row * ldq + qcoff + 32 * blk);
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
    s[row * (ldq >> 5) + (qcoff >> 5) + blk] = (uint8_t)sc;
}

// a list of fp32 weight tensors [rows][C] (row stride C) in one launch: the per-step quantisation of
// config 5's ~50 fp8 weights was ~50 launches of ~4 us of which most is launch latency; job j owns
// blocks [blk0, next blk0), the same per-(row, 32-block) work as k_mx8_quantize<false>
__global__ __launch_bounds__(256) void k_mx8_quantize_list(Mx8WList list) {
    int j = 0;
    while (j + 1 < list.njobs && (int)blockIdx.x >= list.job[j + 1].blk0) ++j;
    const Mx8WJob& jb = list.job[j];
    const int nblk = jb.C >> 5;
    const int64_t i = (int64_t)(blockIdx.x - jb.blk0) * 256 + threadIdx.x;
    if (i >= (int64_t)jb.rows * nblk) return;
    const int64_t row = i / nblk;
    const int blk = (int)(i - row * nblk);
    float v[32];
    const float4* p = reinterpret_cast<const float4*>(jb.src + row * jb.C + 32 * blk);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float4 f = p[e];
        v[4 * e] = f.x; v[4 * e + 1] = f.y; v[4 * e + 2] = f.z; v[4 * e + 3] = f.w;
    }
    uint32_t w[8];
    const uint32_t sc = mx8_quant_block(v, w);
    uint4* d = reinterpret_cast<uint4*>(jb.q + row * jb.ldq + 32 * blk);
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
    jb.s[row * (jb.ldq >> 5) + blk] = (uint8_t)sc;
}

template <int WM, int WN, class Epi>
__global__ __launch_bounds__(256, 2) void k_dense_x8(GemmArgs a, Mx8 x, Mx8 w) {
    dense_body_x8<WM, WN, 2, 2, Epi>(a, x, w);
}
template <int R, int CW, class Epi>
__global__ __launch_bounds__(256, 2) void k_conv3x3_win_x8(GemmArgs a, Mx8 x, Mx8 w) {
    conv3x3_win_x8_body<R, CW, R * CW == 128 ? 2 : 4, R * CW == 128 ? 2 : 1, Epi>(a, x, w);
}

namespace {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

void check_view(const Mx8& m, const char* what) {
    if (!m.q || !m.s || m.ld % 128 || m.coff % 64 || m.coff < 0)
        throw std::runtime_error(std::string("MX-fp8 operand layout: ") + what);
}

template <class Epi>
const char* epi_name() {
    return Epi::STATS ? (Epi::BF16 ? "EpiStoreStatsB16" : "EpiStoreStats") : (Epi::BF16 ? "EpiStoreB16" : "EpiStore");
}

template <int WM, int WN, class Epi>
void launch_dense(const GemmArgs& a, const Mx8& x, const Mx8& w, hipStream_t st) {
    const dim3 grid(cdiv(a.M, 64 * WM), cdiv(a.N, 64 * WN));
    if (prof_enabled()) {
        char name[160];
        std::snprintf(name, sizeof name, "void cad::k_dense_x8<%d, %d, cad::%s>(cad::GemmArgs, cad::Mx8, cad::Mx8)", WM, WN,
                      epi_name<Epi>());
        prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
        hipLaunchKernelGGL((k_dense_x8<WM, WN, Epi>), grid, dim3(256), 0, st, a, x, w);
        prof_pop(st);
    } else {
        hipLaunchKernelGGL((k_dense_x8<WM, WN, Epi>), grid, dim3(256), 0, st, a, x, w);
    }
}
template <class Epi>
void launch_dense_cfg(const GemmArgs& a, const Mx8& x, const Mx8& w, hipStream_t st) {
    if (a.N <= 64) launch_dense<4, 1, Epi>(a, x, w, st);
    else launch_dense<2, 2, Epi>(a, x, w, st);
}

struct WinX8 {
    int R = 0, CW = 0;
};
WinX8 pick_win_x8(int cin, int W, int N) {
    WinX8 p;
    if (cin % 64 || N % 64) return p;
    const int BM = N == 64 ? 256 : 128;
    if (BM == 128 && N % 128) return p;
    static const int c128[] = {64, 32, 16, 8}, c256[] = {128, 64};
    const int* cws = BM == 128 ? c128 : c256;
    for (int i = 0; i < (BM == 128 ? 4 : 2); ++i)
        if (W % cws[i] == 0) {
            p.CW = cws[i];
            p.R = BM / cws[i];
            return p;
        }
    return p;
}

template <int R, int CW, class Epi>
void launch_win_x8_1(const GemmArgs& a, const Mx8& x, const Mx8& w, hipStream_t st) {
    constexpr int BN = R * CW == 128 ? 128 : 64;
    const dim3 grid(a.B * cdiv(a.H, R) * (a.W / CW), cdiv(a.N, BN));
    if (prof_enabled()) {
        char name[160];
        std::snprintf(name, sizeof name, "void cad::k_conv3x3_win_x8<%d, %d, cad::%s>(cad::GemmArgs, cad::Mx8, cad::Mx8)", R,
                      CW, epi_name<Epi>());
        prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
        hipLaunchKernelGGL((k_conv3x3_win_x8<R, CW, Epi>), grid, dim3(256), 0, st, a, x, w);
        prof_pop(st);
    } else {
        hipLaunchKernelGGL((k_conv3x3_win_x8<R, CW, Epi>), grid, dim3(256), 0, st, a, x, w);
    }
}
template <class Epi>
void launch_win_x8(const WinX8& p, const GemmArgs& a, const Mx8& x, const Mx8& w, hipStream_t st) {
    if (p.R * p.CW == 128) {
        switch (p.CW) {
            case 64: launch_win_x8_1<2, 64, Epi>(a, x, w, st); return;
            case 32: launch_win_x8_1<4, 32, Epi>(a, x, w, st); return;
            case 16: launch_win_x8_1<8, 16, Epi>(a, x, w, st); return;
            case 8: launch_win_x8_1<16, 8, Epi>(a, x, w, st); return;
        }
    } else {
        switch (p.CW) {
            case 128: launch_win_x8_1<2, 128, Epi>(a, x, w, st); return;
            case 64: launch_win_x8_1<4, 64, Epi>(a, x, w, st); return;
        }
    }
    throw std::runtime_error("MX-fp8 window conv: block shape not built");
}
}  // namespace

void mx8_quantize(const void* src, bool src_bf16, int64_t lds, int scoff, int C, int64_t M, Mx8 dst, hipStream_t st) {
    if (C % 32 || dst.ld % 128 || dst.coff % 32 || scoff % 8 || lds % 8)
        throw std::runtime_error("mx8_quantize: layout");
    const int nblk = C / 32;
    const int64_t n = M * nblk;
    if (n == 0) return;
    CAD_NO_ALIAS("mx8_quantize", {aview(dst.q, M, dst.ld, dst.coff, C, 1, "q"), aview(dst.s, M, dst.ld / 32, dst.coff / 32, nblk, 1, "scales")},
                 {aview(src, M, lds, scoff, C, src_bf16 ? 2 : 4, "src")});
    auto* q = static_cast<uint8_t*>(const_cast<void*>(dst.q));
    auto* s = static_cast<uint8_t*>(const_cast<void*>(dst.s));
    const dim3 grid((unsigned)((n + 255) / 256));
    if (src_bf16)
        hipLaunchKernelGGL(k_mx8_quantize<true>, grid, dim3(256), 0, st, src, lds, scoff, nblk, n, q, dst.ld, dst.coff, s);
    else
        hipLaunchKernelGGL(k_mx8_quantize<false>, grid, dim3(256), 0, st, src, lds, scoff, nblk, n, q, dst.ld, dst.coff, s);
}

void mx8_quantize_weights(Mx8WList& list, hipStream_t st) {
    if (list.njobs <= 0) return;
    if (list.njobs > kMx8WMaxJobs) throw std::runtime_error("mx8_quantize_weights: too many jobs");
    int blocks = 0;
    for (int j = 0; j < list.njobs; ++j) {
        Mx8WJob& jb = list.job[j];
        if (jb.C % 32 || jb.ldq % 128 || jb.ldq < jb.C || jb.rows <= 0)
            throw std::runtime_error("mx8_quantize_weights: layout");
        CAD_NO_ALIAS("mx8_quantize_weights",
                     {aview(jb.q, jb.rows, jb.ldq, 0, jb.C, 1, "q"), aview(jb.s, jb.rows, jb.ldq / 32, 0, jb.C / 32, 1, "scales")},
                     {aview(jb.src, jb.rows, jb.C, 0, jb.C, 4, "w")});
        jb.blk0 = blocks;
        blocks += cdiv((int64_t)jb.rows * (jb.C / 32), 256);
    }
    hipLaunchKernelGGL(k_mx8_quantize_list, dim3(blocks), dim3(256), 0, st, list);
}

bool dense_x8_ok(int K, int N) { return K > 0 && K % 128 == 0 && N % 64 == 0; }
int dense_x8_stats_rows(int64_t M, int N) { return cdiv(M, N <= 64 ? 256 : 128); }

void dense_fwd_x8(Mx8 x, int K, Mx8 w, int N, float* y, int64_t ldy, int ycoff, int64_t M, float* stats, hipStream_t st,
                  bool y_bf16) {
    check_view(x, "dense x");
    check_view(w, "dense w");
    if (!dense_x8_ok(K, N)) throw std::runtime_error("dense MX-fp8 GEMM: K % 128 and N % 64 required");
    if (M > INT32_MAX) throw std::runtime_error("dense GEMM: too many rows");
    CAD_NO_ALIAS("dense_fwd_x8", {aview(y, M, ldy, ycoff, N, y_bf16 ? 2 : 4, "y")},
                 {aview(x.q, M, x.ld, x.coff, K, 1, "x"), aview(x.s, M, x.ld / 32, x.coff / 32, K / 32, 1, "x scales"),
                  aview(w.q, N, w.ld, w.coff, K, 1, "w"), aview(w.s, N, w.ld / 32, w.coff / 32, K / 32, 1, "w scales")});
    GemmArgs a{};
    a.M = (int)M; a.N = N; a.K = K;
    a.B = 1; a.H = 1; a.W = (int)M;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff;
    a.stats = stats;
    if (y_bf16) {
        if (stats) launch_dense_cfg<EpiStoreStatsB16>(a, x, w, st);
        else launch_dense_cfg<EpiStoreB16>(a, x, w, st);
    } else {
        if (stats) launch_dense_cfg<EpiStoreStats>(a, x, w, st);
        else launch_dense_cfg<EpiStore>(a, x, w, st);
    }
}

bool conv3x3_x8_ok(int cin, int W, int N) { return pick_win_x8(cin, W, N).R > 0; }
int conv3x3_x8_stats_rows(int cin, int B, int H, int W, int cout) {
    const WinX8 p = pick_win_x8(cin, W, cout);
    return p.R ? B * cdiv(H, p.R) * (W / p.CW) : 0;
}

void conv3x3_fwd_x8(Mx8 x, int cin, Mx8 w, int cout, float* y, int64_t ldy, int ycoff, int B, int H, int W, float* stats,
                    hipStream_t st, bool y_bf16) {
    check_view(x, "conv x");
    check_view(w, "conv w");
    const WinX8 p = pick_win_x8(cin, W, cout);
    if (!p.R) throw std::runtime_error("MX-fp8 window conv: cin % 64, N % 64 and a block width dividing W required");
    if (w.ld < 9 * (int64_t)cin) throw std::runtime_error("MX-fp8 window conv: weight rows shorter than 9 cin");
    CAD_NO_ALIAS("conv3x3_fwd_x8", {aview(y, (int64_t)B * H * W, ldy, ycoff, cout, y_bf16 ? 2 : 4, "y")},
                 {aview(x.q, (int64_t)B * H * W, x.ld, x.coff, cin, 1, "x"),
                  aview(x.s, (int64_t)B * H * W, x.ld / 32, x.coff / 32, cin / 32, 1, "x scales"),
                  aview(w.q, cout, w.ld, w.coff, 9 * cin, 1, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = cout; a.K = 9 * cin;
    a.B = B; a.H = H; a.W = W;
    a.a_cin = cin;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff;
    a.stats = stats;
    if (y_bf16) {
        if (stats) launch_win_x8<EpiStoreStatsB16>(p, a, x, w, st);
        else launch_win_x8<EpiStoreB16>(p, a, x, w, st);
    } else {
        if (stats) launch_win_x8<EpiStoreStats>(p, a, x, w, st);
        else launch_win_x8<EpiStore>(p, a, x, w, st);
    }
}

}  // namespace cad
