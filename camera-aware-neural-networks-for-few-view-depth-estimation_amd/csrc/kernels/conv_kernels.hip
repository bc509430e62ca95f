// Convolution / transposed-convolution kernels on the fp32 MFMA engine (gemm_mfma.hpp) and their
// host launchers.  Reference ops replaced: torch::nn::Conv2d(k3,p1,no bias) and
// ConvTranspose2d(k2,s2,bias) of src/models/baseline_unet.h:20-30,85 (forward) and their autograd
// backward (dgrad + wgrad), see SURVEY.md §8(a) a1, a3, a5.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

#include "gemm_mfma.hpp"
#include "gemm_s3.hpp"
#include "gemm_ps.hpp"
#include "kernels.hpp"

namespace cad {

// Row-major epilogues: C[m][c_coff + n] with row stride ldc; the engine stores through a buffer
// descriptor based at row_base (gemm_mfma.hpp gemm_epilogue).
struct EpiStore {
    static constexpr bool STATS = false;
    __device__ static const float* row_base(const GemmArgs& a, int m0, int) {
        return a.C + (int64_t)m0 * a.ldc + a.c_coff;
    }
};
struct EpiStoreStats : EpiStore {
    static constexpr bool STATS = true;
};
// conv3x3 dgrad whose output feeds a ReLU(BatchNorm) backward: per-tile (Σ dz, Σ dz·x̂) partials
// (GemmArgs e_*), so the BN backward skips its reduction pass over (g, y)
struct EpiStoreBnBwd : EpiStore {
    static constexpr bool STATS = true;
    static constexpr bool BNBWD = true;
};
// ConvTranspose2d(k2,s2) pixel shuffle: n = (q=(dy,dx), co) -> high-res pixel (2y+dy, 2x+dx).
// The column (q, co) is fixed per lane and sub-block, and rows advance in small steps, so the
// epilogue carries (x, y, b) incrementally instead of dividing per element (STRUCTURED epilogue).
struct EpiConvT {
    static constexpr bool STATS = false;
    static constexpr bool STRUCTURED = true;
    __device__ void operator()(const GemmArgs& a, int m, int n, float v, int) const {
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const int x = m % a.W, t = m / a.W, y = t % a.H, b = t / a.H;
        const int64_t hp = ((int64_t)b * (2 * a.H) + 2 * y + (q >> 1)) * (2 * a.W) + 2 * x + (q & 1);
        a.C[hp * a.ldc + a.c_coff + co] = v + a.bias[co];
    }
    // one lane's 16 accumulator rows of a 32x32 sub-block: rows mbase + (r&3) + 8(r>>2), column n
    __device__ void block(const GemmArgs& a, int mbase, int n, const floatx16& acc) const {
        if (n >= a.N) return;
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const float bias = a.bias[co];
        float* dst = a.C + a.c_coff + co;
        const int64_t W2 = 2 * a.W;
        int x = mbase % a.W, t = mbase / a.W, y = t % a.H, b = t / a.H;
        int cur = 0;   // row offset that (x, y, b) currently describe
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int off = (r & 3) + 8 * (r >> 2);
            x += off - cur;
            cur = off;
            while (x >= a.W) { x -= a.W; if (++y == a.H) { y = 0; ++b; } }
            if (mbase + off < a.M) {
                const int64_t hp = ((int64_t)b * (2 * a.H) + 2 * y + (q >> 1)) * W2 + 2 * x + (q & 1);
                dst[hp * a.ldc] = acc[r] + bias;
            }
        }
    }
    // 4 consecutive rows m..m+3 at column n (the 16x16 MFMA layout's quads)
    __device__ void quad(const GemmArgs& a, int m, int n, const float (&v)[4]) const {
        if (n >= a.N) return;
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const float bias = a.bias[co];
        float* dst = a.C + a.c_coff + co;
        const int64_t W2 = 2 * a.W;
        int x = m % a.W, t = m / a.W, y = t % a.H, b = t / a.H;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (m + r < a.M) {
                const int64_t hp = ((int64_t)b * (2 * a.H) + 2 * y + (q >> 1)) * W2 + 2 * x + (q & 1);
                dst[hp * a.ldc] = v[r] + bias;
            }
            if (++x == a.W) { x = 0; if (++y == a.H) { y = 0; ++b; } }
        }
    }
};
struct EpiSlab {   // split-K partial: slab z holds C[m][n] of K-slice z
    static constexpr bool STATS = false;
    __device__ static const float* row_base(const GemmArgs& a, int m0, int z) {
        return a.C + (int64_t)z * a.slab_stride + (int64_t)m0 * a.ldc;
    }
};

template <int WM, int WN, int KB, class Epi, bool BNA>
__global__ __launch_bounds__(256) void k_conv3x3_fwd(GemmArgs a) {
    using LA = KcIm2col3x3<64 * WM, KB, BNA>;
    using LB = KcDense<64 * WN, KB>;
    gemm_body<WM, WN, KB, LA, true, LB, true>(
        a,
        [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb, a.a_sc, a.a_sh); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, Epi{});
}

template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_fwd(GemmArgs a) {
    using LA = KcDense<64 * WM, KB>;
    using LB = KcDense<64 * WN, KB>;
    gemm_body<WM, WN, KB, LA, true, LB, true>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiConvT{});
}

template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_dgrad(GemmArgs a) {
    using LA = KcUpGather<64 * WM, KB>;
    using LB = KcDense<64 * WN, KB>;
    gemm_body<WM, WN, KB, LA, true, LB, true>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiStore{});
}

template <int WM, int WN, int KB, bool BNB>
__global__ __launch_bounds__(256) void k_conv3x3_wgrad(GemmArgs a) {
    using LA = MNcDense<64 * WM, KB>;
    using LB = MNcIm2col3x3<64 * WN, KB, BNB>;
    gemm_body<WM, WN, KB, LA, false, LB, false>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.b_cin, a.B, a.H, a.W, r0, t, kb, a.b_sc, a.b_sh); },
        EpiSlab{});
}

template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_wgrad(GemmArgs a) {
    using LA = MNcDense<64 * WM, KB>;
    using LB = MNcUpGather<64 * WN, KB>;
    gemm_body<WM, WN, KB, LA, false, LB, false>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.b_cin, a.B, a.H, a.W, r0, t, kb); },
        EpiSlab{});
}

// ---- S3 / B1 engines (gemm_s3.hpp): NP = 3 exact bf16 planes (fp32 accuracy) or 1 rounded plane
// (bf16 operands).  The __global__ wrappers carry distinct names per engine (rocprof symbols). ----
template <int NP, int WM, int WN, int MI, int NJ, int KB, class Epi>
__device__ __forceinline__ void conv3x3_fwd_np(const GemmArgs& a) {
    using LA = KcIm2col3x3<32 * MI * WM, KB, false>;
    using LB = KcDense<32 * NJ * WN, KB>;
    gemm_body_s3<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a,
        [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, Epi{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void convT_fwd_np(const GemmArgs& a) {
    using LA = KcDense<32 * MI * WM, KB>;
    using LB = KcDense<32 * NJ * WN, KB>;
    gemm_body_s3<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiConvT{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void convT_dgrad_np(const GemmArgs& a) {
    using LA = KcUpGather<32 * MI * WM, KB>;
    using LB = KcDense<32 * NJ * WN, KB>;
    gemm_body_s3<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiStore{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void conv3x3_wgrad_np(const GemmArgs& a) {
    using LA = MNcDense<32 * MI * WM, KB>;
    using LB = MNcIm2col3x3<32 * NJ * WN, KB, false>;
    gemm_body_s3m<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.b_cin, a.B, a.H, a.W, r0, t, kb); },
        EpiSlab{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void convT_wgrad_np(const GemmArgs& a) {
    using LA = MNcDense<32 * MI * WM, KB>;
    using LB = MNcUpGather<32 * NJ * WN, KB>;
    gemm_body_s3m<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.b_cin, a.B, a.H, a.W, r0, t, kb); },
        EpiSlab{});
}

template <int WM, int WN, int KB, class Epi>
__global__ __launch_bounds__(256) void k_conv3x3_fwd_s3(GemmArgs a) { conv3x3_fwd_np<3, WM, WN, 2, 2, KB, Epi>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_fwd_s3(GemmArgs a) { convT_fwd_np<3, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_dgrad_s3(GemmArgs a) { convT_dgrad_np<3, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_conv3x3_wgrad_s3(GemmArgs a) { conv3x3_wgrad_np<3, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_wgrad_s3(GemmArgs a) { convT_wgrad_np<3, WM, WN, 2, 2, KB>(a); }

template <int WM, int WN, int KB, class Epi>
__global__ __launch_bounds__(256) void k_conv3x3_fwd_bf16(GemmArgs a) { conv3x3_fwd_np<1, WM, WN, 2, 2, KB, Epi>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_fwd_bf16(GemmArgs a) { convT_fwd_np<1, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_dgrad_bf16(GemmArgs a) { convT_dgrad_np<1, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_conv3x3_wgrad_bf16(GemmArgs a) { conv3x3_wgrad_np<1, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_wgrad_bf16(GemmArgs a) { convT_wgrad_np<1, WM, WN, 2, 2, KB>(a); }
#define CAD_NP_LKERNELS(SUF, NP)                                                                             \
    template <int WM, int WN, int KB, class Epi>                                                             \
    __global__ __launch_bounds__(256, 2) void k_conv3x3_fwd_##SUF(GemmArgs a) { conv3x3_fwd_np<NP, WM, WN, 4, 2, KB, Epi>(a); } \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, 2) void k_convT_fwd_##SUF(GemmArgs a) { convT_fwd_np<NP, WM, WN, 4, 2, KB>(a); }     \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, 2) void k_convT_dgrad_##SUF(GemmArgs a) { convT_dgrad_np<NP, WM, WN, 4, 2, KB>(a); } \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, 2) void k_conv3x3_wgrad_##SUF(GemmArgs a) { conv3x3_wgrad_np<NP, WM, WN, 2, 4, KB>(a); } \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, 2) void k_convT_wgrad_##SUF(GemmArgs a) { convT_wgrad_np<NP, WM, WN, 2, 4, KB>(a); }
CAD_NP_LKERNELS(s3L, 3)
CAD_NP_LKERNELS(bf16L, 1)
#undef CAD_NP_LKERNELS

// ---- S3 with pre-split weights ("s3w"): the activation operand A is split in the loader, the
// weight operand B (split once per step) is staged without conversion — half the main-loop split
// work of s3 at 1.25x its operand bytes ----
template <int WM, int WN, int KB, class Epi>
__global__ __launch_bounds__(256) void k_conv3x3_fwd_s3w(GemmArgs a) {
    using LA = KcIm2col3x3<64 * WM, KB, false>;
    using LB = PsKcDense<64 * WN, KB, 3>;
    gemm_body_s3<3, WM, WN, 2, 2, KB, LA, LB>(
        a,
        [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, Epi{});
}
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_fwd_s3w(GemmArgs a) {
    using LA = KcDense<64 * WM, KB>;
    using LB = PsKcDense<64 * WN, KB, 3>;
    gemm_body_s3<3, WM, WN, 2, 2, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiConvT{});
}
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_dgrad_s3w(GemmArgs a) {
    using LA = KcUpGather<64 * WM, KB>;
    using LB = PsKcDense<64 * WN, KB, 3>;
    gemm_body_s3<3, WM, WN, 2, 2, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiStore{});
}

// ---- pre-split operand kernels (gemm_ps.hpp): A/B pointers are split tensors (kernels.hpp Split),
// lda/ldb their row length in channels, a_coff/b_coff channel offsets ----
template <int NP, int WM, int WN, int MI, int NJ, int KB, class Epi>
__device__ __forceinline__ void conv3x3_fwd_psb(const GemmArgs& a) {
    using LA = PsKcIm2col3x3<32 * MI * WM, KB, NP>;
    using LB = PsKcDense<32 * NJ * WN, KB, NP>;
    gemm_body_ps<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a,
        [&](LA& l, int r0, int t, int kb) {
            l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb, a.cimajor);
        },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb, a.cimajor, a.a_cin); },
        Epi{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void convT_fwd_psb(const GemmArgs& a) {
    using LA = PsKcDense<32 * MI * WM, KB, NP>;
    using LB = PsKcDense<32 * NJ * WN, KB, NP>;
    gemm_body_ps<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiConvT{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void convT_dgrad_psb(const GemmArgs& a) {
    using LA = PsKcUpGather<32 * MI * WM, KB, NP>;
    using LB = PsKcDense<32 * NJ * WN, KB, NP>;
    gemm_body_ps<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiStore{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void conv3x3_wgrad_psb(const GemmArgs& a) {
    using LA = PsMNcDense<32 * MI * WM, KB, NP>;
    using LB = PsMNcIm2col3x3<32 * NJ * WN, KB, NP>;
    gemm_body_psm<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.b_cin, a.B, a.H, a.W, r0, t, kb); },
        EpiSlab{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void convT_wgrad_psb(const GemmArgs& a) {
    using LA = PsMNcDense<32 * MI * WM, KB, NP>;
    using LB = PsMNcUpGather<32 * NJ * WN, KB, NP>;
    gemm_body_psm<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.b_cin, a.B, a.H, a.W, r0, t, kb); },
        EpiSlab{});
}
#define CAD_PS_KERNELS(SUF, NP, MI_, NJ_, NJW_, WPE)                                                               \
    template <int WM, int WN, int KB, class Epi>                                                             \
    __global__ __launch_bounds__(256, WPE) void k_conv3x3_fwd_##SUF(GemmArgs a) { conv3x3_fwd_psb<NP, WM, WN, MI_, NJ_, KB, Epi>(a); } \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, WPE) void k_convT_fwd_##SUF(GemmArgs a) { convT_fwd_psb<NP, WM, WN, MI_, NJ_, KB>(a); }     \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, WPE) void k_convT_dgrad_##SUF(GemmArgs a) { convT_dgrad_psb<NP, WM, WN, MI_, NJ_, KB>(a); } \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, WPE) void k_conv3x3_wgrad_##SUF(GemmArgs a) { conv3x3_wgrad_psb<NP, WM, WN, 2, NJW_, KB>(a); } \
    template <int WM, int WN, int KB>                                                                        \
    __global__ __launch_bounds__(256, WPE) void k_convT_wgrad_##SUF(GemmArgs a) { convT_wgrad_psb<NP, WM, WN, 2, NJW_, KB>(a); }
CAD_PS_KERNELS(s3p, 3, 2, 2, 2, 1)
CAD_PS_KERNELS(bf16p, 1, 2, 2, 2, 1)
// large tiles: 256x128 (conv / ConvT forward, dgrad: 2x2 waves of 128x64) and 128x256 (weight
// gradients: 2x2 waves of 64x128) — 0.75x the operand bytes per MAC of the 128x128 tile
CAD_PS_KERNELS(s3pL, 3, 4, 2, 4, 2)   // (256, 2): at most 256 VGPRs, two waves per SIMD
CAD_PS_KERNELS(bf16pL, 1, 4, 2, 4, 2)
#undef CAD_PS_KERNELS

// split pass: one thread per (row, 8-channel group)
template <int NP>
__global__ void k_split_rows(const float* __restrict__ x, int64_t ldx, int xcoff, int G, int64_t n,
                             char* __restrict__ out, int64_t ldo, int ocoff) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t row = i / G;
    const int g = (int)(i - row * G);
    const float* s = x + row * ldx + xcoff + 8 * g;
    const float4 a = *reinterpret_cast<const float4*>(s);
    const float4 b = *reinterpret_cast<const float4*>(s + 4);
    split8_store<NP>(out + row * ldo * 2 * NP + (int64_t)((ocoff >> 3) + g) * 16 * NP, a, b);
}

// deterministic split-K reduction: dst[e] = sum_z slab[z * zstep][e] for z < nsplit (fixed order).
// Two levels when there are many slabs (the 64-channel weight gradients: ~680 slices of a small
// M x N): level 1 sums each group of G consecutive slabs into the group's first slab (blockIdx.y =
// group), level 2 sums the group heads — a few dozen dependent loads per thread instead of ~680.
__global__ void k_slab_reduce(float* __restrict__ slab, int nsplit, int64_t stride, int zstep,
                              float* __restrict__ dst, int64_t n) {
    int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i >= n) return;
    const int z0 = blockIdx.y * nsplit;   // level 1: this group's slabs; level 2: gridDim.y == 1
    float4 s = *reinterpret_cast<const float4*>(slab + (int64_t)z0 * zstep * stride + i);
    for (int z = 1; z < nsplit; ++z) {
        float4 t = *reinterpret_cast<const float4*>(slab + (int64_t)(z0 + z) * zstep * stride + i);
        s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    float* out = dst ? dst + i : slab + (int64_t)z0 * zstep * stride + i;
    *reinterpret_cast<float4*>(out) = s;
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
namespace {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// tile shape by output width: narrow N -> tall tiles.  K-stage depth per (kernel kind, tile shape),
// measured on MI355X at the bench shapes (bs32 480x640 f=64): 32 pays for the conv3x3 forward/dgrad
// on the square tile (+1% plain, +8% with the BN-stats epilogue), 16 everywhere else (the wgrad and
// ConvT GEMMs lose 2-6% at 32, the tall/wide tiles ~10%).  CAD_KB_<KIND>_<CFG>=16|32 overrides,
// e.g. CAD_KB_WGRAD_C22=32.
// C22L / C22W (S3, B1 and pre-split engines): 256x128 / 128x256 tiles of 2x2 waves with 128x64 /
// 64x128 per wave — 0.75x the operand bytes and LDS traffic per MAC of C22, half the barriers per
// MFMA; for the pixel-major (forward, dgrad) and the weight-gradient contractions.  Off by default
// (CAD_BIGTILE=1 enables): measured on MI355X they tie C22 on S3 (189 vs 188 TFLOP/s) and B1
// (676 vs 693) at two waves per SIMD instead of three.
enum Cfg { C41, C22, C14, C22L, C22W };
enum Kind { K_FWD, K_FWDS, K_WGRAD, K_TFWD, K_TDGRAD, K_TWGRAD, K_NKIND };
int engine();
bool big_tiles() {
    static int on = -1;
    if (on < 0) {
        const char* e = std::getenv("CAD_BIGTILE");
        on = (e && e[0] == '1') ? 1 : 0;
    }
    return on && engine() != 0;
}
Cfg pick_cfg(int M, int N, bool wgrad = false) {
    if (N <= 64) return C41;
    if (M <= 64) return C14;
    if (big_tiles()) {
        if (!wgrad && M >= 4096) return C22L;
        if (wgrad && N >= 256) return C22W;
    }
    return C22;
}
int kb_for(Kind k, Cfg c) {
    static int kb[K_NKIND][3];
    static bool init = false;
    if (!init) {
        const char* kn[K_NKIND] = {"FWD", "FWDS", "WGRAD", "TFWD", "TDGRAD", "TWGRAD"};
        const char* cn[3] = {"C41", "C22", "C14"};
        for (int i = 0; i < K_NKIND; ++i)
            for (int j = 0; j < 3; ++j) {
                int v = (j == C22 && (i == K_FWD || i == K_FWDS)) ? 32 : 16;
                char name[40];
                snprintf(name, sizeof(name), "CAD_KB_%s_%s", kn[i], cn[j]);
                if (const char* e = std::getenv(name)) v = std::atoi(e);
                kb[i][j] = v == 32 ? 32 : 16;
            }
        init = true;
    }
    return kb[k][c];
}

template <template <int, int, int> class KT, int WM, int WN, int KB>
void launch_one(const GemmArgs& a, int splits, hipStream_t st, bool large = false) {
    using K = KT<WM, WN, KB>;
    auto fn = K::fn();
    if (large) {   // large tiles exist as 2x2-wave launches only (pick_cfg)
        if constexpr (WM == 2 && WN == 2 && K::HASL) fn = K::fnL();
        else throw std::runtime_error("large tile requested for a kernel without one");
    }
    const int mi = large ? K::LMI : 2, nj = large ? K::LNJ : 2;
    const dim3 grid(cdiv(a.M, 32 * mi * WM), cdiv(a.N, 32 * nj * WN), splits);
    if (prof_enabled()) {
        char name[160];
        snprintf(name, sizeof(name), large ? K::fmtL : K::fmt, WM, WN, KB);
        prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
        prof_pop(st);
    } else {
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
    }
}
template <template <int, int, int> class KT, int WM, int WN>
void launch_kb(int kb, const GemmArgs& a, int splits, hipStream_t st) {
    if (kb == 32) launch_one<KT, WM, WN, 32>(a, splits, st);
    else launch_one<KT, WM, WN, 16>(a, splits, st);
}
template <template <int, int, int> class KT>
void launch_cfg(Cfg c, int kb, const GemmArgs& a, int splits, hipStream_t st) {
    switch (c) {
        case C41: launch_kb<KT, 4, 1>(kb, a, splits, st); break;
        case C22: launch_kb<KT, 2, 2>(kb, a, splits, st); break;
        case C14: launch_kb<KT, 1, 4>(kb, a, splits, st); break;
        default: throw std::runtime_error("tile configuration not available on this engine");
    }
}
template <template <int, int, int> class KT, int KB>
void launch_cfg_kb(Cfg c, const GemmArgs& a, int splits, hipStream_t st) {
    switch (c) {
        case C41: launch_one<KT, 4, 1, KB>(a, splits, st); break;
        case C22: launch_one<KT, 2, 2, KB>(a, splits, st); break;
        case C14: launch_one<KT, 1, 4, KB>(a, splits, st); break;
        case C22L:
        case C22W: launch_one<KT, 2, 2, KB>(a, splits, st, true); break;
    }
}
// fmt = the symbol as rocprofv3 demangles it
// (kernel pointers behind functions: a specialization is instantiated only when launched)
#define CAD_KT(NAME, EXPR, FMT)                                                  \
    template <int WM, int WN, int KB> struct NAME {                              \
        static auto fn() { return EXPR; }                                        \
        static constexpr const char* fmt = FMT;                                  \
        static constexpr bool HASL = false;                                      \
        static auto fnL() { return EXPR; }                                       \
        static constexpr const char* fmtL = FMT;                                 \
        static constexpr int LMI = 2, LNJ = 2;                                   \
    };
// with a large-tile variant (launched for C22L / C22W): LMI x LNJ 32x32 blocks per wave
#define CAD_KTL(NAME, EXPR, FMT, EXPRL, FMTL, LMI_, LNJ_)                        \
    template <int WM, int WN, int KB> struct NAME {                              \
        static auto fn() { return EXPR; }                                        \
        static constexpr const char* fmt = FMT;                                  \
        static constexpr bool HASL = true;                                       \
        static auto fnL() { return EXPRL; }                                      \
        static constexpr const char* fmtL = FMTL;                                \
        static constexpr int LMI = LMI_, LNJ = LNJ_;                             \
    };
CAD_KT(KConvFwd, (k_conv3x3_fwd<WM, WN, KB, EpiStore, false>),
       "void cad::k_conv3x3_fwd<%d, %d, %d, cad::EpiStore, false>(cad::GemmArgs)")
CAD_KT(KConvFwdS, (k_conv3x3_fwd<WM, WN, KB, EpiStoreStats, false>),
       "void cad::k_conv3x3_fwd<%d, %d, %d, cad::EpiStoreStats, false>(cad::GemmArgs)")
CAD_KT(KConvFwdX, (k_conv3x3_fwd<WM, WN, KB, EpiStoreBnBwd, false>),
       "void cad::k_conv3x3_fwd<%d, %d, %d, cad::EpiStoreBnBwd, false>(cad::GemmArgs)")
CAD_KT(KConvFwdBN, (k_conv3x3_fwd<WM, WN, KB, EpiStore, true>),
       "void cad::k_conv3x3_fwd<%d, %d, %d, cad::EpiStore, true>(cad::GemmArgs)")
CAD_KT(KConvFwdSBN, (k_conv3x3_fwd<WM, WN, KB, EpiStoreStats, true>),
       "void cad::k_conv3x3_fwd<%d, %d, %d, cad::EpiStoreStats, true>(cad::GemmArgs)")
CAD_KT(KConvWgrad, (k_conv3x3_wgrad<WM, WN, KB, false>), "void cad::k_conv3x3_wgrad<%d, %d, %d, false>(cad::GemmArgs)")
CAD_KT(KConvWgradBN, (k_conv3x3_wgrad<WM, WN, KB, true>), "void cad::k_conv3x3_wgrad<%d, %d, %d, true>(cad::GemmArgs)")
CAD_KT(KConvTFwd, (k_convT_fwd<WM, WN, KB>), "void cad::k_convT_fwd<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTDgrad, (k_convT_dgrad<WM, WN, KB>), "void cad::k_convT_dgrad<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTWgrad, (k_convT_wgrad<WM, WN, KB>), "void cad::k_convT_wgrad<%d, %d, %d>(cad::GemmArgs)")
#define CAD_NP_KT(SUF, T)                                                                                      \
    CAD_KTL(KConvFwd##T, (k_conv3x3_fwd_##SUF<WM, WN, KB, EpiStore>),                                          \
            "void cad::k_conv3x3_fwd_" #SUF "<%d, %d, %d, cad::EpiStore>(cad::GemmArgs)",                      \
            (k_conv3x3_fwd_##SUF##L<WM, WN, KB, EpiStore>),                                                   \
            "void cad::k_conv3x3_fwd_" #SUF "L<%d, %d, %d, cad::EpiStore>(cad::GemmArgs)", 4, 2)               \
    CAD_KTL(KConvFwdS##T, (k_conv3x3_fwd_##SUF<WM, WN, KB, EpiStoreStats>),                                    \
            "void cad::k_conv3x3_fwd_" #SUF "<%d, %d, %d, cad::EpiStoreStats>(cad::GemmArgs)",                 \
            (k_conv3x3_fwd_##SUF##L<WM, WN, KB, EpiStoreStats>),                                              \
            "void cad::k_conv3x3_fwd_" #SUF "L<%d, %d, %d, cad::EpiStoreStats>(cad::GemmArgs)", 4, 2)          \
    CAD_KTL(KConvFwdX##T, (k_conv3x3_fwd_##SUF<WM, WN, KB, EpiStoreBnBwd>),                                    \
            "void cad::k_conv3x3_fwd_" #SUF "<%d, %d, %d, cad::EpiStoreBnBwd>(cad::GemmArgs)",                 \
            (k_conv3x3_fwd_##SUF##L<WM, WN, KB, EpiStoreBnBwd>),                                              \
            "void cad::k_conv3x3_fwd_" #SUF "L<%d, %d, %d, cad::EpiStoreBnBwd>(cad::GemmArgs)", 4, 2)          \
    CAD_KTL(KConvTFwd##T, (k_convT_fwd_##SUF<WM, WN, KB>), "void cad::k_convT_fwd_" #SUF "<%d, %d, %d>(cad::GemmArgs)", \
            (k_convT_fwd_##SUF##L<WM, WN, KB>), "void cad::k_convT_fwd_" #SUF "L<%d, %d, %d>(cad::GemmArgs)", 4, 2) \
    CAD_KTL(KConvTDgrad##T, (k_convT_dgrad_##SUF<WM, WN, KB>),                                                 \
            "void cad::k_convT_dgrad_" #SUF "<%d, %d, %d>(cad::GemmArgs)",                                     \
            (k_convT_dgrad_##SUF##L<WM, WN, KB>), "void cad::k_convT_dgrad_" #SUF "L<%d, %d, %d>(cad::GemmArgs)", 4, 2) \
    CAD_KTL(KConvWgrad##T, (k_conv3x3_wgrad_##SUF<WM, WN, KB>),                                                \
            "void cad::k_conv3x3_wgrad_" #SUF "<%d, %d, %d>(cad::GemmArgs)",                                   \
            (k_conv3x3_wgrad_##SUF##L<WM, WN, KB>), "void cad::k_conv3x3_wgrad_" #SUF "L<%d, %d, %d>(cad::GemmArgs)", 2, 4) \
    CAD_KTL(KConvTWgrad##T, (k_convT_wgrad_##SUF<WM, WN, KB>),                                                 \
            "void cad::k_convT_wgrad_" #SUF "<%d, %d, %d>(cad::GemmArgs)",                                     \
            (k_convT_wgrad_##SUF##L<WM, WN, KB>), "void cad::k_convT_wgrad_" #SUF "L<%d, %d, %d>(cad::GemmArgs)", 2, 4)
CAD_KT(KConvFwdW3, (k_conv3x3_fwd_s3w<WM, WN, KB, EpiStore>), "void cad::k_conv3x3_fwd_s3w<%d, %d, %d, cad::EpiStore>(cad::GemmArgs)")
CAD_KT(KConvFwdSW3, (k_conv3x3_fwd_s3w<WM, WN, KB, EpiStoreStats>),
       "void cad::k_conv3x3_fwd_s3w<%d, %d, %d, cad::EpiStoreStats>(cad::GemmArgs)")
CAD_KT(KConvTFwdW3, (k_convT_fwd_s3w<WM, WN, KB>), "void cad::k_convT_fwd_s3w<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTDgradW3, (k_convT_dgrad_s3w<WM, WN, KB>), "void cad::k_convT_dgrad_s3w<%d, %d, %d>(cad::GemmArgs)")
// in-loader split engines: KConvFwd3 ... (S3), KConvFwdB ... (B1); pre-split: KConvFwdP3 ..., KConvFwdP1 ...
CAD_NP_KT(s3, 3)
CAD_NP_KT(bf16, B)
CAD_NP_KT(s3p, P3)
CAD_NP_KT(bf16p, P1)
#undef CAD_NP_KT
#undef CAD_KT

// GEMM engine of every conv / ConvT contraction: 0 = exact f32 MFMA, 1 = S3 (bf16 matrix cores,
// exact 3-term split; gemm_s3.hpp) — the default: fp32 accuracy (tests/test_gpu_ops.py) at
// 1.35-1.4x the f32 engine's speed on MI355X; 2 = B1 (operands rounded to bf16, one product, fp32
// accumulation: the bf16 configs 3-5).  Process-wide; CAD_GEMM=f32|s3|bf16 sets the initial value.
int g_engine = -1;
int engine() {
    if (g_engine < 0) {
        const char* e = std::getenv("CAD_GEMM");
        g_engine = (e && e[0] == 'f') ? 0 : (e && e[0] == 'b') ? 2 : 1;
    }
    return g_engine;
}
// B1 stage depth (two k16 steps per LDS stage by default; CAD_BF16_KB=16|32)
// B1 stage depth override (CAD_BF16_KB=16|32|64; 0 = per-kernel defaults below)
int bf16_kb_env() {
    static int kb = -1;
    if (kb < 0) {
        const char* e = std::getenv("CAD_BF16_KB");
        const int v = e ? std::atoi(e) : 0;
        kb = (v == 16 || v == 32 || v == 64) ? v : 0;
    }
    return kb;
}
int ps_bf16_kb() { return bf16_kb_env() ? bf16_kb_env() : 32; }
int bf16_kb() {   // in-loader B1 kernels (KS<KB> staging: 16 or 32)
    return std::min(ps_bf16_kb(), 32);
}
template <template <int, int, int> class KT>
void launch_b1(Cfg c, const GemmArgs& a, int splits, hipStream_t st) {
    if (bf16_kb() == 16) launch_cfg_kb<KT, 16>(c, a, splits, st);
    else launch_cfg_kb<KT, 32>(c, a, splits, st);
}
// pre-split B1 kernels may also stage 64 k per stage (four k16 steps between barriers)
template <template <int, int, int> class KT>
void launch_b1p(Cfg c, int kb, const GemmArgs& a, int splits, hipStream_t st) {
    if (kb == 16) launch_cfg_kb<KT, 16>(c, a, splits, st);
    else if (kb == 64) launch_cfg_kb<KT, 64>(c, a, splits, st);
    else launch_cfg_kb<KT, 32>(c, a, splits, st);
}
int ps_planes() { return engine() == 1 ? 3 : engine() == 2 ? 1 : 0; }
// stage depth of a pre-split GEMM: S3 16 (three planes); B1 per kernel kind — 64 for the
// conv3x3 forward/dgrad on 128x128 tiles (measured on MI355X: 708 -> 790 TFLOP/s), 32 elsewhere
// (64 costs the weight-gradient and the tall/wide tiles 7-20%)
int ps_kb(bool fwd_kind = false, Cfg c = C41) {
    if (engine() == 1) return 16;
    if (bf16_kb_env()) return bf16_kb_env();
    return fwd_kind && c == C22 ? 64 : 32;
}
template <template <int, int, int> class KT3, template <int, int, int> class KT1>
void launch_ps(Cfg c, int kb, const GemmArgs& a, int splits, hipStream_t st) {
    if (engine() == 1) launch_cfg_kb<KT3, 16>(c, a, splits, st);
    else if (engine() == 2) launch_b1p<KT1>(c, kb, a, splits, st);
    else throw std::runtime_error("pre-split GEMM launched on the f32 engine");
}
constexpr int kS3KB = 16;   // S3 stage depth (LDS: 3 bf16 planes per operand)
// S3 stage depth: one bf16 k16 step per LDS stage (32 measured 12-13% slower: the LDS footprint
// costs a workgroup per CU); kept as a function for the launch sites
int s3_kb(Kind, Cfg) { return kS3KB; }
[[maybe_unused]] int s3_kb_env(Kind k, Cfg c) {
    static int kb[K_NKIND][3];
    static bool init = false;
    if (!init) {
        const char* kn[K_NKIND] = {"FWD", "FWDS", "WGRAD", "TFWD", "TDGRAD", "TWGRAD"};
        const char* cn[3] = {"C41", "C22", "C14"};
        for (int i = 0; i < K_NKIND; ++i)
            for (int j = 0; j < 3; ++j) {
                int v = kS3KB;
                char name[40];
                snprintf(name, sizeof(name), "CAD_S3KB_%s_%s", kn[i], cn[j]);
                if (const char* e = std::getenv(name)) v = std::atoi(e);
                kb[i][j] = v == 32 ? 32 : 16;
            }
        init = true;
    }
    return kb[k][c];
}
template <template <int, int, int> class KT>
void launch_s3(Cfg c, int, const GemmArgs& a, int splits, hipStream_t st) {
    launch_cfg_kb<KT, 16>(c, a, splits, st);
}

int tile_m(Cfg c) { return c == C41 || c == C22L ? 256 : c == C22 || c == C22W ? 128 : 64; }
int tile_n(Cfg c) { return c == C41 ? 64 : c == C22 || c == C22L ? 128 : 256; }

// split-K planning for the weight-gradient GEMMs: aim for >= ~2048 workgroups, >= 32 K-stages each.
// A K-slice is also a loader's buffer window (gemm_mfma.hpp: 32-bit offsets from the slice's first
// pixel): `kbytes` = bytes one K step spans in the widest operand; slices stay below 1 GB.
int plan_splits(const GemmArgs& a, Cfg c, int kb, int64_t slab_cap_floats, int64_t kbytes) {
    const int tiles = cdiv(a.M, tile_m(c)) * cdiv(a.N, tile_n(c));
    const int nk = cdiv(a.K, kb);
    int s = std::max(1, std::min(cdiv(2048, tiles), nk / 32));
    const int64_t per = (int64_t)a.M * a.N;
    if (slab_cap_floats > 0) s = (int)std::max<int64_t>(1, std::min<int64_t>(s, slab_cap_floats / per));
    const int64_t need = (int64_t)cdiv((int64_t)a.K * kbytes, (int64_t)1 << 30);
    if (need > s) {
        if (slab_cap_floats > 0 && need * per > slab_cap_floats)
            throw std::runtime_error("weight-gradient K-slice exceeds the 1 GB loader window and the split-K slab");
        s = (int)need;
    }
    return s;
}
}  // namespace

void conv3x3_fwd(const float* x, int64_t ldx, int xcoff, int cin, const float* w, int cout, float* y,
                 int64_t ldy, int ycoff, int B, int H, int W, float* stats, hipStream_t st,
                 const float* in_scale, const float* in_shift, const void* w_split) {
    GemmArgs a{};
    a.M = B * H * W; a.N = cout; a.K = 9 * cin;
    a.B = B; a.H = H; a.W = W;
    a.A = x; a.lda = ldx; a.a_coff = xcoff; a.a_cin = cin;
    a.Bm = w; a.ldb = 9 * cin; a.b_coff = 0;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff;
    a.stats = stats;
    a.a_sc = in_scale; a.a_sh = in_shift;
    const Cfg c = pick_cfg(a.M, a.N);
    if (engine() == 2 && !in_scale) {
        a.kstages_per_split = cdiv(a.K, bf16_kb());
        if (stats) launch_b1<KConvFwdSB>(c, a, 1, st); else launch_b1<KConvFwdB>(c, a, 1, st);
        return;
    }
    if (engine() == 1 && !in_scale) {
        const int kb = s3_kb(stats ? K_FWDS : K_FWD, c);
        a.kstages_per_split = cdiv(a.K, kb);
        if (w_split && a.K % 8 == 0) {   // pre-split weights: rows cout of K = 9 cin
            a.Bm = static_cast<const float*>(w_split); a.ldb = a.K; a.b_coff = 0;
            if (stats) launch_s3<KConvFwdSW3>(c, kb, a, 1, st); else launch_s3<KConvFwdW3>(c, kb, a, 1, st);
            return;
        }
        if (stats) launch_s3<KConvFwdS3>(c, kb, a, 1, st); else launch_s3<KConvFwd3>(c, kb, a, 1, st);
        return;
    }
    const int kb = kb_for(stats ? K_FWDS : K_FWD, c);
    a.kstages_per_split = cdiv(a.K, kb);
    if (in_scale) {
        if (stats) launch_cfg<KConvFwdSBN>(c, kb, a, 1, st); else launch_cfg<KConvFwdBN>(c, kb, a, 1, st);
    } else {
        if (stats) launch_cfg<KConvFwdS>(c, kb, a, 1, st); else launch_cfg<KConvFwd>(c, kb, a, 1, st);
    }
}

void set_gemm_engine(int e) { g_engine = (e == 1 || e == 2) ? e : 0; }
int gemm_engine() { return engine(); }

int conv3x3_stats_rows(int B, int H, int W, int cout) {
    Cfg c = pick_cfg(B * H * W, cout);
    return cdiv((int64_t)B * H * W, tile_m(c));
}

void convT_fwd(const float* x, int64_t ldx, int cin, const float* wf, const float* bias, int cout,
               float* y, int64_t ldy, int ycoff, int B, int H, int W, hipStream_t st, const void* wf_split) {
    GemmArgs a{};
    a.M = B * H * W; a.N = 4 * cout; a.K = cin;
    a.B = B; a.H = H; a.W = W;
    a.A = x; a.lda = ldx; a.a_coff = 0;
    a.Bm = wf; a.ldb = cin;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff; a.bias = bias;
    const Cfg c = pick_cfg(a.M, a.N);
    if (engine() == 2) {
        a.kstages_per_split = cdiv(a.K, bf16_kb());
        launch_b1<KConvTFwdB>(c, a, 1, st);
        return;
    }
    if (engine() == 1) {
        const int kb = s3_kb(K_TFWD, c);
        a.kstages_per_split = cdiv(a.K, kb);
        if (wf_split && a.K % 8 == 0) {   // rows 4 cout of K = cin
            a.Bm = static_cast<const float*>(wf_split);
            launch_s3<KConvTFwdW3>(c, kb, a, 1, st);
            return;
        }
        launch_s3<KConvTFwd3>(c, kb, a, 1, st);
        return;
    }
    const int kb = kb_for(K_TFWD, c);
    a.kstages_per_split = cdiv(a.K, kb);
    launch_cfg<KConvTFwd>(c, kb, a, 1, st);
}

static void set_bnbwd(GemmArgs& a, const BnBwdEpi* bn) {
    a.stats = bn->stats;
    a.e_y = bn->y; a.e_mean = bn->mean; a.e_invstd = bn->invstd; a.e_scale = bn->scale; a.e_shift = bn->shift;
}

void conv3x3_dgrad(const float* dz, int cout, const float* wd, int cin, float* dx, int64_t lddx,
                   int B, int H, int W, hipStream_t st, const void* wd_split, const BnBwdEpi* bn) {
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 9 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = dz; a.lda = cout; a.a_coff = 0; a.a_cin = cout;
    a.Bm = wd; a.ldb = 9 * cout;
    a.C = dx; a.ldc = lddx; a.c_coff = 0;
    if (bn) {
        if (lddx != cin || (engine() == 1 && wd_split))
            throw std::runtime_error("BN-backward dgrad epilogue: dense output, no pre-split-weight kernel");
        set_bnbwd(a, bn);
    }
    const Cfg c = pick_cfg(a.M, a.N);
    if (engine() == 2) {
        a.kstages_per_split = cdiv(a.K, bf16_kb());
        if (bn) launch_b1<KConvFwdXB>(c, a, 1, st); else launch_b1<KConvFwdB>(c, a, 1, st);
        return;
    }
    if (engine() == 1) {
        const int kb = s3_kb(K_FWD, c);
        a.kstages_per_split = cdiv(a.K, kb);
        if (wd_split && a.K % 8 == 0) {   // rows cin of K = 9 cout
            a.Bm = static_cast<const float*>(wd_split);
            launch_s3<KConvFwdW3>(c, kb, a, 1, st);
            return;
        }
        if (bn) launch_s3<KConvFwdX3>(c, kb, a, 1, st); else launch_s3<KConvFwd3>(c, kb, a, 1, st);
        return;
    }
    const int kb = kb_for(K_FWD, c);
    a.kstages_per_split = cdiv(a.K, kb);
    if (bn) launch_cfg<KConvFwdX>(c, kb, a, 1, st); else launch_cfg<KConvFwd>(c, kb, a, 1, st);
}

void convT_dgrad(const float* g, int64_t ldg, int gcoff, int cout, const float* wm, int cin, float* dx,
                 int B, int H, int W, hipStream_t st, const void* wm_split) {
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 4 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = g; a.lda = ldg; a.a_coff = gcoff; a.a_cin = cout;
    a.Bm = wm; a.ldb = 4 * cout;
    a.C = dx; a.ldc = cin; a.c_coff = 0;
    const Cfg c = pick_cfg(a.M, a.N);
    if (engine() == 2) {
        a.kstages_per_split = cdiv(a.K, bf16_kb());
        launch_b1<KConvTDgradB>(c, a, 1, st);
        return;
    }
    if (engine() == 1) {
        const int kb = s3_kb(K_TDGRAD, c);
        a.kstages_per_split = cdiv(a.K, kb);
        if (wm_split && a.K % 8 == 0) {   // rows cin of K = 4 cout
            a.Bm = static_cast<const float*>(wm_split);
            launch_s3<KConvTDgradW3>(c, kb, a, 1, st);
            return;
        }
        launch_s3<KConvTDgrad3>(c, kb, a, 1, st);
        return;
    }
    const int kb = kb_for(K_TDGRAD, c);
    a.kstages_per_split = cdiv(a.K, kb);
    launch_cfg<KConvTDgrad>(c, kb, a, 1, st);
}

int64_t wgrad_slab_floats(int M, int N, int Kpix) {
    GemmArgs a{};
    a.M = M; a.N = N; a.K = Kpix;
    const Cfg c = pick_cfg(M, N, true);
    return (int64_t)plan_splits(a, c, 16, 0, 0) * M * N;   // kb 16: the larger split count
}

static void finish_slabs(float* slab, int splits, int64_t per, float* dw, hipStream_t st) {
    const unsigned bx = (unsigned)cdiv(per / 4, 256);
    constexpr int G = 24;   // slabs per level-1 group
    static const bool two_level = !(std::getenv("CAD_SLAB2") && std::getenv("CAD_SLAB2")[0] == '0');
    if (two_level && splits >= 2 * G && bx < 512) {
        const int groups = splits / G;   // whole groups; the remainder slabs join level 2 one by one
        hipLaunchKernelGGL(k_slab_reduce, dim3(bx, groups), dim3(256), 0, st, slab, G, per, 1, (float*)nullptr, per);
        // level 2: group heads z = 0, G, 2G, ... then the remainder slabs groups*G .. splits-1
        hipLaunchKernelGGL(k_slab_reduce, dim3(bx, 1), dim3(256), 0, st, slab, groups, per, G, (float*)nullptr, per);
        const int rem = splits - groups * G;
        if (rem == 0) {
            hipLaunchKernelGGL(k_slab_reduce, dim3(bx, 1), dim3(256), 0, st, slab, 1, per, 1, dw, per);
        } else {
            // move the level-2 total next to the remainder and sum those (fixed order)
            float* tail = slab + (int64_t)(groups * G - 1) * per;
            hipLaunchKernelGGL(k_slab_reduce, dim3(bx, 1), dim3(256), 0, st, slab, 1, per, 1, tail, per);
            hipLaunchKernelGGL(k_slab_reduce, dim3(bx, 1), dim3(256), 0, st, tail, rem + 1, per, 1, dw, per);
        }
        return;
    }
    hipLaunchKernelGGL(k_slab_reduce, dim3(bx, 1), dim3(256), 0, st, slab, splits, per, 1, dw, per);
}

void conv3x3_wgrad(const float* dz, int cout, const float* x, int64_t ldx, int xcoff, int cin, float* dw,
                   int B, int H, int W, float* slab, int64_t slab_cap, hipStream_t st,
                   const float* x_scale, const float* x_shift) {
    GemmArgs a{};
    a.M = cout; a.N = 9 * cin; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = dz; a.lda = cout; a.a_coff = 0;
    a.Bm = x; a.ldb = ldx; a.b_coff = xcoff; a.b_cin = cin;
    a.b_sc = x_scale; a.b_sh = x_shift;
    const Cfg c = pick_cfg(a.M, a.N, true);
    const bool s3 = engine() == 1 && !x_scale, b1 = engine() == 2 && !x_scale;
    const int kb = b1 ? bf16_kb() : s3 ? s3_kb(K_WGRAD, c) : kb_for(K_WGRAD, c);
    int s = plan_splits(a, c, kb, slab_cap, 4 * std::max<int64_t>(a.lda, ldx));
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    if (b1) launch_b1<KConvWgradB>(c, a, s, st);
    else if (s3) launch_s3<KConvWgrad3>(c, kb, a, s, st);
    else if (x_scale) launch_cfg<KConvWgradBN>(c, kb, a, s, st);
    else launch_cfg<KConvWgrad>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

void convT_wgrad(const float* x, int cin, const float* g, int64_t ldg, int gcoff, int cout, float* dw,
                 int B, int H, int W, float* slab, int64_t slab_cap, hipStream_t st) {
    GemmArgs a{};
    a.M = cin; a.N = 4 * cout; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = x; a.lda = cin; a.a_coff = 0;
    a.Bm = g; a.ldb = ldg; a.b_coff = gcoff; a.b_cin = cout;
    const Cfg c = pick_cfg(a.M, a.N, true);
    const bool s3 = engine() == 1, b1 = engine() == 2;
    const int kb = b1 ? bf16_kb() : s3 ? s3_kb(K_TWGRAD, c) : kb_for(K_TWGRAD, c);
    int s = plan_splits(a, c, kb, slab_cap, 4 * std::max<int64_t>(a.lda, 4 * ldg));
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    if (b1) launch_b1<KConvTWgradB>(c, a, s, st);
    else if (s3) launch_s3<KConvTWgrad3>(c, kb, a, s, st);
    else launch_cfg<KConvTWgrad>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

// ------------------------------------------------------------------------------------------
// pre-split launchers
// ------------------------------------------------------------------------------------------
int split_planes() { return ps_planes(); }

void split_rows(const float* x, int64_t ldx, int xcoff, int C, int64_t M, void* out, int64_t ldo, int ocoff,
                hipStream_t st) {
    if (C % 8 || xcoff % 4 || ldx % 4 || ocoff % 8 || ldo % 8) throw std::runtime_error("split_rows: alignment");
    const int G = C / 8;
    const int64_t n = M * G;
    if (n == 0) return;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (ps_planes() == 3)
        hipLaunchKernelGGL(k_split_rows<3>, grid, dim3(256), 0, st, x, ldx, xcoff, G, n, (char*)out, ldo, ocoff);
    else if (ps_planes() == 1)
        hipLaunchKernelGGL(k_split_rows<1>, grid, dim3(256), 0, st, x, ldx, xcoff, G, n, (char*)out, ldo, ocoff);
    else
        throw std::runtime_error("split_rows on the f32 engine");
}

namespace {
// channel-major K order for the pre-split conv3x3 forward/dgrad (GemmArgs::cimajor); CAD_CIMAJOR=0 disables
int cimajor_ok(int cin, int kb) {
    static int on = -1;
    if (on < 0) {
        const char* e = std::getenv("CAD_CIMAJOR");
        on = (e && e[0] == '0') ? 0 : 1;
    }
    return on && cin % kb == 0 ? 1 : 0;
}
void ps_check(const Split& s, int channels, const char* what) {
    if (!s.p || s.ld % 8 || s.coff % 8 || channels % 8) throw std::runtime_error(std::string("pre-split operand: ") + what);
}
}  // namespace

void conv3x3_fwd_ps(Split x, int cin, Split w, int cout, float* y, int64_t ldy, int ycoff, int B, int H, int W,
                    float* stats, hipStream_t st) {
    ps_check(x, cin, "conv3x3_fwd x");
    ps_check(w, 9 * cin, "conv3x3_fwd w");
    GemmArgs a{};
    a.M = B * H * W; a.N = cout; a.K = 9 * cin;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)x.p; a.lda = x.ld; a.a_coff = x.coff; a.a_cin = cin;
    a.Bm = (const float*)w.p; a.ldb = w.ld; a.b_coff = w.coff;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff;
    a.stats = stats;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(true, c);
    a.kstages_per_split = cdiv(a.K, kb);
    a.cimajor = cimajor_ok(cin, kb);
    if (stats) launch_ps<KConvFwdSP3, KConvFwdSP1>(c, kb, a, 1, st);
    else launch_ps<KConvFwdP3, KConvFwdP1>(c, kb, a, 1, st);
}

void conv3x3_dgrad_ps(Split dz, int cout, Split wd, int cin, float* dx, int64_t lddx, int B, int H, int W,
                      hipStream_t st, const BnBwdEpi* bn) {
    ps_check(dz, cout, "conv3x3_dgrad dz");
    ps_check(wd, 9 * cout, "conv3x3_dgrad w");
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 9 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)dz.p; a.lda = dz.ld; a.a_coff = dz.coff; a.a_cin = cout;
    a.Bm = (const float*)wd.p; a.ldb = wd.ld; a.b_coff = wd.coff;
    a.C = dx; a.ldc = lddx; a.c_coff = 0;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(true, c);
    a.kstages_per_split = cdiv(a.K, kb);
    a.cimajor = cimajor_ok(cout, kb);
    if (bn) {
        if (lddx != cin) throw std::runtime_error("BN-backward dgrad epilogue: dense output only");
        set_bnbwd(a, bn);
        launch_ps<KConvFwdXP3, KConvFwdXP1>(c, kb, a, 1, st);
    } else {
        launch_ps<KConvFwdP3, KConvFwdP1>(c, kb, a, 1, st);
    }
}

void conv3x3_wgrad_ps(Split dz, int cout, Split x, int cin, float* dw, int B, int H, int W, float* slab,
                      int64_t slab_cap, hipStream_t st) {
    ps_check(dz, cout, "conv3x3_wgrad dz");
    ps_check(x, cin, "conv3x3_wgrad x");
    GemmArgs a{};
    a.M = cout; a.N = 9 * cin; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)dz.p; a.lda = dz.ld; a.a_coff = dz.coff;
    a.Bm = (const float*)x.p; a.ldb = x.ld; a.b_coff = x.coff; a.b_cin = cin;
    const Cfg c = pick_cfg(a.M, a.N, true);
    const int kb = ps_kb();
    int s = plan_splits(a, c, kb, slab_cap, 2 * kMaxPlanes * std::max<int64_t>(dz.ld, x.ld));
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    launch_ps<KConvWgradP3, KConvWgradP1>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

void convT_fwd_ps(Split x, int cin, Split wf, const float* bias, int cout, float* y, int64_t ldy, int ycoff, int B,
                  int H, int W, hipStream_t st) {
    ps_check(x, cin, "convT_fwd x");
    ps_check(wf, cin, "convT_fwd w");
    GemmArgs a{};
    a.M = B * H * W; a.N = 4 * cout; a.K = cin;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)x.p; a.lda = x.ld; a.a_coff = x.coff;
    a.Bm = (const float*)wf.p; a.ldb = wf.ld; a.b_coff = wf.coff;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff; a.bias = bias;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb();
    a.kstages_per_split = cdiv(a.K, kb);
    launch_ps<KConvTFwdP3, KConvTFwdP1>(c, kb, a, 1, st);
}

void convT_dgrad_ps(Split g, int cout, Split wm, int cin, float* dx, int B, int H, int W, hipStream_t st) {
    ps_check(g, cout, "convT_dgrad g");
    ps_check(wm, 4 * cout, "convT_dgrad w");
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 4 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)g.p; a.lda = g.ld; a.a_coff = g.coff; a.a_cin = cout;
    a.Bm = (const float*)wm.p; a.ldb = wm.ld; a.b_coff = wm.coff;
    a.C = dx; a.ldc = cin; a.c_coff = 0;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb();
    a.kstages_per_split = cdiv(a.K, kb);
    launch_ps<KConvTDgradP3, KConvTDgradP1>(c, kb, a, 1, st);
}

void convT_wgrad_ps(Split x, int cin, Split g, int cout, float* dw, int B, int H, int W, float* slab,
                    int64_t slab_cap, hipStream_t st) {
    ps_check(x, cin, "convT_wgrad x");
    ps_check(g, cout, "convT_wgrad g");
    GemmArgs a{};
    a.M = cin; a.N = 4 * cout; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)x.p; a.lda = x.ld; a.a_coff = x.coff;
    a.Bm = (const float*)g.p; a.ldb = g.ld; a.b_coff = g.coff; a.b_cin = cout;
    const Cfg c = pick_cfg(a.M, a.N, true);
    const int kb = ps_kb();
    int s = plan_splits(a, c, kb, slab_cap, 2 * kMaxPlanes * std::max<int64_t>(x.ld, 4 * g.ld));
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    launch_ps<KConvTWgradP3, KConvTWgradP1>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

}  // namespace cad
