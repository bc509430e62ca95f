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
#include "gemm_win.hpp"
#include "kernels.hpp"
#include "epilogues.hpp"

namespace cad {

template <int WM, int WN, int KB, class Epi>
__global__ __launch_bounds__(256) void k_conv3x3_fwd(GemmArgs a) {
    using LA = KcIm2col3x3<64 * WM, KB>;
    using LB = KcDense<64 * WN, KB>;
    gemm_body<WM, WN, KB, LA, true, LB, true>(
        a,
        [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
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

template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_conv3x3_wgrad(GemmArgs a) {
    using LA = MNcDense<64 * WM, KB>;
    using LB = MNcIm2col3x3<64 * WN, KB>;
    gemm_body<WM, WN, KB, LA, false, LB, false>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.b_cin, a.B, a.H, a.W, r0, t, kb); },
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
    using LA = KcIm2col3x3<32 * MI * WM, KB>;
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
    using LB = MNcIm2col3x3<32 * NJ * WN, KB>;
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

// window-tiled conv3x3 forward/dgrad (gemm_win.hpp): BM = R*CW output pixels of one image; 128x128
// tiles (WM = WN = 2) or, for N <= 64, 256x64 (WM = 4, WN = 1)
template <int R, int CW, class Epi>
__global__ __launch_bounds__(256, 3) void k_conv3x3_win_s3(GemmArgs a) {
    conv3x3_win_body<3, R, CW, R * CW == 128 ? 2 : 4, R * CW == 128 ? 2 : 1, Epi>(a);
}

// window-tiled conv3x3 forward/dgrad on the pre-split bf16 twins (B1)
template <int R, int CW, class Epi>
__global__ __launch_bounds__(256, 3) void k_conv3x3_win_bf16p(GemmArgs a) {
    conv3x3_win_ps_body<R, CW, R * CW == 128 ? 2 : 4, R * CW == 128 ? 2 : 1, Epi>(a);
}
// ... with 4 x 2 blocks of 32 x 32 per wave: 256 x 128 tiles (N % 128 == 0; BN64 = false) or
// 512 x 64 tiles (N == 64).  Blocks at most 16 pixels wide (levels 3-4 of 480 x 640) run the same
// tile as 8 x 4 blocks of 16 x 16 (v_mfma_f32_16x16x32_bf16): measured on MI355X (tools/winlab.py,
// configs[3] shapes) 4-6 % faster there, 1-6 % slower on the wider blocks of levels 0-2.
template <int R, int CW, class Epi, bool BN64 = false>
__global__ __launch_bounds__(256, 2) void k_conv3x3_win_bf16p4(GemmArgs a) {
    conv3x3_win_ps_body<R, CW, BN64 ? 4 : 2, BN64 ? 1 : 2, Epi, 4, 2, (CW <= 16) || (CAD_WIN16 != 0)>(a);
}

// ... 256 x 96 tiles (2 x 3 blocks of 32 x 32 per wave, four waves down M) for N % 96 == 0: the 96 and
// 192-channel levels at f = 96
template <int R, int CW, class Epi>
__global__ __launch_bounds__(256, 2) void k_conv3x3_win_bf16p3(GemmArgs a) {
    conv3x3_win_ps_body<R, CW, 4, 1, Epi, 2, 3>(a);
}

// window-tiled conv3x3 weight gradient (gemm_win.hpp): 64 co x 64 ci x 9 taps per workgroup, split-K
__global__ __launch_bounds__(256, 2) void k_conv3x3_wgrad_win_s3(GemmArgs a) { conv3x3_wgrad_win_body<3>(a); }
__global__ __launch_bounds__(256, 2) void k_conv3x3_wgrad_strip_s3(GemmArgs a) { conv3x3_wgrad_strip_body<3>(a); }
template <int P>
__global__ __launch_bounds__(256, 2) void k_conv3x3_wgrad_win_bf16p(GemmArgs a) { conv3x3_wgrad_win_ps_body<P>(a); }
// ... with LDS-DMA staging (3-stage ring, conv3x3_wgrad_win_dma_body)
template <int P, int NBUF>
__global__ __launch_bounds__(256, 2) void k_conv3x3_wgrad_win_bf16d(GemmArgs a) { conv3x3_wgrad_win_dma_body<P, NBUF>(a); }
template <int P>
__global__ __launch_bounds__(256, 2) void k_conv3x3_wgrad_strip_bf16d(GemmArgs a) { conv3x3_wgrad_strip_dma_body<P>(a); }
// ... two output rows per step (P = 16 levels)
template <int P>
__global__ __launch_bounds__(256, 2) void k_conv3x3_wgrad_strip2_bf16d(GemmArgs a) { conv3x3_wgrad_strip2_dma_body<P>(a); }

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
template <int NP, int WM, int WN, int MI, int NJ, int KB, class Epi = EpiConvT>
__device__ __forceinline__ void convT_fwd_psb(const GemmArgs& a) {
    using LA = PsKcDense<32 * MI * WM, KB, NP>;
    using LB = PsKcDense<32 * NJ * WN, KB, NP>;
    gemm_body_ps<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, Epi{});
}
template <int NP, int WM, int WN, int MI, int NJ, int KB, class Epi = EpiStore>
__device__ __forceinline__ void convT_dgrad_psb(const GemmArgs& a) {
    using LA = PsKcUpGather<32 * MI * WM, KB, NP>;
    using LB = PsKcDense<32 * NJ * WN, KB, NP>;
    gemm_body_ps<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.a_cin, a.B, a.H, a.W, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, Epi{});
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
// dense GEMMs on twins (config-5 network: 1x1 and im2col convolutions): C[m][n] = sum_k A[m][k] B[n][k]
template <int NP, int WM, int WN, int MI, int NJ, int KB, class Epi>
__device__ __forceinline__ void dense_nt_psb(const GemmArgs& a) {
    using LA = PsKcDense<32 * MI * WM, KB, NP>;
    using LB = PsKcDense<32 * NJ * WN, KB, NP>;
    gemm_body_ps<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, Epi{});
}
// ... and their weight gradients: C[m][n] = sum_k A[k][m] B[k][n] (k = pixel)
template <int NP, int WM, int WN, int MI, int NJ, int KB>
__device__ __forceinline__ void dense_tn_psb(const GemmArgs& a) {
    using LA = PsMNcDense<32 * MI * WM, KB, NP>;
    using LB = PsMNcDense<32 * NJ * WN, KB, NP>;
    gemm_body_psm<NP, WM, WN, MI, NJ, KB, LA, LB>(
        a, [&](LA& l, int r0, int t, int kb) { l.init(a.A, a.lda, a.a_coff, a.M, a.K, r0, t, kb); },
        [&](LB& l, int r0, int t, int kb) { l.init(a.Bm, a.ldb, a.b_coff, a.N, a.K, r0, t, kb); }, EpiSlab{});
}
template <int WM, int WN, int KB, class Epi>
__global__ __launch_bounds__(256) void k_dense_bf16p(GemmArgs a) { dense_nt_psb<1, WM, WN, 2, 2, KB, Epi>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_dense_wgrad_bf16p(GemmArgs a) { dense_tn_psb<1, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB, class Epi>
__global__ __launch_bounds__(256) void k_conv3x3_fwd_bf16p(GemmArgs a) { conv3x3_fwd_psb<1, WM, WN, 2, 2, KB, Epi>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_fwd_bf16p(GemmArgs a) { convT_fwd_psb<1, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_fwd_bf16pt(GemmArgs a) {
    convT_fwd_psb<1, WM, WN, 2, 2, KB, EpiConvTB16>(a);
}
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_dgrad_bf16p(GemmArgs a) { convT_dgrad_psb<1, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_dgrad_bf16pb(GemmArgs a) {
    convT_dgrad_psb<1, WM, WN, 2, 2, KB, EpiStoreB16>(a);
}
// ... 256 x 128 tiles (2 x 2 waves of 4 x 2 blocks): each A row-stage feeds twice the MFMA work (the
// ConvT GEMMs' K is cin or 4 cout, 128..2048: short main loops that the 128 x 128 tile left issue-bound)
template <int KB>
__global__ __launch_bounds__(256, 2) void k_convT_fwd_bf16pt4(GemmArgs a) {
    convT_fwd_psb<1, 2, 2, 4, 2, KB, EpiConvTB16>(a);
}
template <int KB>
__global__ __launch_bounds__(256, 2) void k_convT_dgrad_bf16pb4(GemmArgs a) {
    convT_dgrad_psb<1, 2, 2, 4, 2, KB, EpiStoreB16>(a);
}
// ... with LDS-DMA staging (gemm_dense_dma_body: 3-stage ring)
__global__ __launch_bounds__(256, 2) void k_convT_fwd_bf16dt(GemmArgs a) {
    gemm_dense_dma_body<2, 2, 2, 2, EpiConvTB16>(a);
}
// dense (1x1-conv / im2col) forward GEMMs of the config-5 network on the same DMA body
template <class Epi>
__global__ __launch_bounds__(256, 2) void k_dense_bf16d(GemmArgs a) {
    gemm_dense_dma_body<2, 2, 2, 2, Epi>(a);
}
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_conv3x3_wgrad_bf16p(GemmArgs a) { conv3x3_wgrad_psb<1, WM, WN, 2, 2, KB>(a); }
template <int WM, int WN, int KB>
__global__ __launch_bounds__(256) void k_convT_wgrad_bf16p(GemmArgs a) { convT_wgrad_psb<1, WM, WN, 2, 2, KB>(a); }

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
    // unrolled: the slabs' loads in flight together, the adds in slab order (same sums bit for bit)
#pragma unroll 8
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

// Tile shape by output width: narrow N -> tall tiles (256x64), narrow M -> wide tiles (64x256),
// else 128x128.  K-stage depth per engine and kernel kind, measured on MI355X at the bench shapes
// (bs32 480x640 f=64):
//   f32: 32 for the conv3x3 forward/dgrad on the square tile (+1% plain, +8% with the BN-stats
//        epilogue), 16 elsewhere (the wgrad and ConvT GEMMs lose 2-6% at 32, the tall/wide tiles ~10%);
//   S3:  16 (three bf16 planes per operand; 32 measured 12-13% slower: the LDS footprint costs a
//        workgroup per CU);
//   B1 in-loader split: 32 (two k16 steps per stage);
//   B1 pre-split: 64 for the conv3x3 forward/dgrad on 128x128 tiles (708 -> 790 TFLOP/s), 32
//        elsewhere (64 costs the weight-gradient and the tall/wide tiles 7-20%).
enum Cfg { C41, C22, C14 };
Cfg pick_cfg(int M, int N) {
    if (N <= 64) return C41;
    if (M <= 64) return C14;
    return C22;
}
int tile_m(Cfg c) { return c == C41 ? 256 : c == C22 ? 128 : 64; }
int tile_n(Cfg c) { return c == C41 ? 64 : c == C22 ? 128 : 256; }

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
int f32_kb(bool conv_fwd_kind, Cfg c) { return conv_fwd_kind && c == C22 ? 32 : 16; }
constexpr int kS3KB = 16;
constexpr int kB1KB = 32;
int ps_kb(bool conv_fwd_kind, Cfg c) { return conv_fwd_kind && c == C22 ? 64 : 32; }

template <template <int, int, int> class KT, int WM, int WN, int KB>
void launch_one(const GemmArgs& a, int splits, hipStream_t st) {
    using K = KT<WM, WN, KB>;
    const dim3 grid(cdiv(a.M, 64 * WM), cdiv(a.N, 64 * WN), splits);
    if (prof_enabled()) {
        char name[160];
        snprintf(name, sizeof(name), K::fmt, WM, WN, KB);
        prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
        hipLaunchKernelGGL(K::fn(), grid, dim3(256), 0, st, a);
        prof_pop(st);
    } else {
        hipLaunchKernelGGL(K::fn(), grid, dim3(256), 0, st, a);
    }
}
template <template <int, int, int> class KT, int KB>
void launch_cfg(Cfg c, const GemmArgs& a, int splits, hipStream_t st) {
    switch (c) {
        case C41: launch_one<KT, 4, 1, KB>(a, splits, st); break;
        case C22: launch_one<KT, 2, 2, KB>(a, splits, st); break;
        case C14: launch_one<KT, 1, 4, KB>(a, splits, st); break;
    }
}
// stage depth kb among the ones a kernel family is built for (KBs)
template <template <int, int, int> class KT, int... KBs>
void launch_kb(Cfg c, int kb, const GemmArgs& a, int splits, hipStream_t st) {
    const bool done = ((kb == KBs ? (launch_cfg<KT, KBs>(c, a, splits, st), true) : false) || ...);
    if (!done) throw std::runtime_error("GEMM stage depth not built for this kernel family");
}
// fmt = the symbol as rocprofv3 demangles it
// (kernel pointers behind functions: a specialization is instantiated only when launched)
#define CAD_KT(NAME, EXPR, FMT)                                                  \
    template <int WM, int WN, int KB> struct NAME {                              \
        static auto fn() { return EXPR; }                                        \
        static constexpr const char* fmt = FMT;                                  \
    };
CAD_KT(KConvFwd, (k_conv3x3_fwd<WM, WN, KB, EpiStore>), "void cad::k_conv3x3_fwd<%d, %d, %d, cad::EpiStore>(cad::GemmArgs)")
CAD_KT(KConvFwdS, (k_conv3x3_fwd<WM, WN, KB, EpiStoreStats>),
       "void cad::k_conv3x3_fwd<%d, %d, %d, cad::EpiStoreStats>(cad::GemmArgs)")
CAD_KT(KConvWgrad, (k_conv3x3_wgrad<WM, WN, KB>), "void cad::k_conv3x3_wgrad<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTFwd, (k_convT_fwd<WM, WN, KB>), "void cad::k_convT_fwd<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTDgrad, (k_convT_dgrad<WM, WN, KB>), "void cad::k_convT_dgrad<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTWgrad, (k_convT_wgrad<WM, WN, KB>), "void cad::k_convT_wgrad<%d, %d, %d>(cad::GemmArgs)")
#define CAD_NP_KT(SUF, T)                                                                                  \
    CAD_KT(KConvFwd##T, (k_conv3x3_fwd_##SUF<WM, WN, KB, EpiStore>),                                       \
           "void cad::k_conv3x3_fwd_" #SUF "<%d, %d, %d, cad::EpiStore>(cad::GemmArgs)")                   \
    CAD_KT(KConvFwdS##T, (k_conv3x3_fwd_##SUF<WM, WN, KB, EpiStoreStats>),                                 \
           "void cad::k_conv3x3_fwd_" #SUF "<%d, %d, %d, cad::EpiStoreStats>(cad::GemmArgs)")              \
    CAD_KT(KConvTFwd##T, (k_convT_fwd_##SUF<WM, WN, KB>), "void cad::k_convT_fwd_" #SUF "<%d, %d, %d>(cad::GemmArgs)") \
    CAD_KT(KConvTDgrad##T, (k_convT_dgrad_##SUF<WM, WN, KB>),                                              \
           "void cad::k_convT_dgrad_" #SUF "<%d, %d, %d>(cad::GemmArgs)")                                  \
    CAD_KT(KConvWgrad##T, (k_conv3x3_wgrad_##SUF<WM, WN, KB>),                                             \
           "void cad::k_conv3x3_wgrad_" #SUF "<%d, %d, %d>(cad::GemmArgs)")                                \
    CAD_KT(KConvTWgrad##T, (k_convT_wgrad_##SUF<WM, WN, KB>),                                              \
           "void cad::k_convT_wgrad_" #SUF "<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KDenseP1, (k_dense_bf16p<WM, WN, KB, EpiStore>), "void cad::k_dense_bf16p<%d, %d, %d, cad::EpiStore>(cad::GemmArgs)")
CAD_KT(KDenseSP1, (k_dense_bf16p<WM, WN, KB, EpiStoreStats>),
       "void cad::k_dense_bf16p<%d, %d, %d, cad::EpiStoreStats>(cad::GemmArgs)")
CAD_KT(KDenseP1B, (k_dense_bf16p<WM, WN, KB, EpiStoreB16>), "void cad::k_dense_bf16p<%d, %d, %d, cad::EpiStoreB16>(cad::GemmArgs)")
CAD_KT(KDenseSP1B, (k_dense_bf16p<WM, WN, KB, EpiStoreStatsB16>),
       "void cad::k_dense_bf16p<%d, %d, %d, cad::EpiStoreStatsB16>(cad::GemmArgs)")
CAD_KT(KConvFwdP1B, (k_conv3x3_fwd_bf16p<WM, WN, KB, EpiStoreB16>),
       "void cad::k_conv3x3_fwd_bf16p<%d, %d, %d, cad::EpiStoreB16>(cad::GemmArgs)")
CAD_KT(KConvFwdSP1B, (k_conv3x3_fwd_bf16p<WM, WN, KB, EpiStoreStatsB16>),
       "void cad::k_conv3x3_fwd_bf16p<%d, %d, %d, cad::EpiStoreStatsB16>(cad::GemmArgs)")
CAD_KT(KDenseWgradP1, (k_dense_wgrad_bf16p<WM, WN, KB>), "void cad::k_dense_wgrad_bf16p<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTFwdP1T, (k_convT_fwd_bf16pt<WM, WN, KB>), "void cad::k_convT_fwd_bf16pt<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KConvTDgradP1B, (k_convT_dgrad_bf16pb<WM, WN, KB>), "void cad::k_convT_dgrad_bf16pb<%d, %d, %d>(cad::GemmArgs)")
CAD_KT(KDenseAddP1, (k_dense_bf16p<WM, WN, KB, EpiStoreAdd>), "void cad::k_dense_bf16p<%d, %d, %d, cad::EpiStoreAdd>(cad::GemmArgs)")
// in-loader split engines: KConvFwd3 ... (S3), KConvFwdB ... (B1); pre-split B1: KConvFwdP1 ...
CAD_NP_KT(s3, 3)
CAD_NP_KT(bf16, B)
CAD_NP_KT(bf16p, P1)
#undef CAD_NP_KT
#undef CAD_KT

// `splits` launches of one contraction on the current engine with in-loader operand conversion:
// F = f32 kernel, T3 = S3, TB = B1; `fwd_kind` selects the deeper f32 stage of the conv3x3
// forward/dgrad.  a.kstages_per_split must be set.
template <template <int, int, int> class F, template <int, int, int> class T3, template <int, int, int> class TB>
void launch_on_engine(Cfg c, int kb, const GemmArgs& a, int splits, hipStream_t st) {
    if (engine() == 1) launch_kb<T3, kS3KB>(c, kb, a, splits, st);
    else if (engine() == 2) launch_kb<TB, kB1KB>(c, kb, a, splits, st);
    else launch_kb<F, 16, 32>(c, kb, a, splits, st);
}
int engine_kb(bool fwd_kind, Cfg c) { return engine() == 1 ? kS3KB : engine() == 2 ? kB1KB : f32_kb(fwd_kind, c); }
template <template <int, int, int> class F, template <int, int, int> class T3, template <int, int, int> class TB>
void launch_engine(Cfg c, bool fwd_kind, GemmArgs& a, hipStream_t st) {
    const int kb = engine_kb(fwd_kind, c);
    a.kstages_per_split = cdiv(a.K, kb);
    launch_on_engine<F, T3, TB>(c, kb, a, 1, st);
}

// Window-tiled conv3x3 forward/dgrad (S3 engine): the block shape for a given layer, or R = 0 when
// the im2col kernel serves it (channels not a multiple of 16: enc1.conv1; no CW dividing W)
struct WinPick {
    int R = 0, CW = 0;
    bool big = false;   // B1 4 x 2 blocks per wave (k_conv3x3_win_bf16p4): 256 x 128, or 512 x 64 tiles
    bool n96 = false;   // B1 256 x 96 tiles (k_conv3x3_win_bf16p3)
    int bn() const { return n96 ? 96 : big ? (R * CW == 256 ? 128 : 64) : R * CW == 128 ? 128 : 64; }
};
WinPick pick_win(int cin, int W, int N) {
    WinPick w;
    if (engine() != 1 || cin % 16) return w;
    const int BM = N <= 64 ? 256 : 128;
    if (N % (BM == 128 ? 128 : 64)) return w;
    static const int c128[] = {64, 32, 16, 8}, c256[] = {128, 64};
    const int* cws = BM == 128 ? c128 : c256;
    const int ncw = BM == 128 ? 4 : 2;
    for (int i = 0; i < ncw; ++i)
        if (W % cws[i] == 0) {
            w.CW = cws[i];
            w.R = BM / cws[i];
            return w;
        }
    return w;
}
int win_blocks(const WinPick& w, int B, int H, int W) { return B * cdiv(H, w.R) * (W / w.CW); }
// PS = false: S3 window kernel (fp32 operands, in-loader split); true: B1 on the pre-split twins
template <bool PS, int R, int CW, class Epi, bool BIG = false, bool N96 = false>
void launch_win1(const GemmArgs& a, hipStream_t st) {
    constexpr int BN = N96 ? 96 : BIG ? (R * CW == 256 ? 128 : 64) : R * CW == 128 ? 128 : 64;
    if (a.N % BN) throw std::runtime_error("window conv: N not a multiple of the tile");
    const dim3 grid(win_blocks(WinPick{R, CW}, a.B, a.H, a.W), cdiv(a.N, BN));
    void (*fn)(GemmArgs);
    if constexpr (N96) fn = k_conv3x3_win_bf16p3<R, CW, Epi>;
    else if constexpr (BIG) fn = k_conv3x3_win_bf16p4<R, CW, Epi, BN == 64>;
    else fn = PS ? (void (*)(GemmArgs))k_conv3x3_win_bf16p<R, CW, Epi> : (void (*)(GemmArgs))k_conv3x3_win_s3<R, CW, Epi>;
    if (prof_enabled()) {
        char name[160];
        snprintf(name, sizeof(name), "void cad::k_conv3x3_win_%s<%d, %d, cad::%s%s>(cad::GemmArgs)",
                 N96 ? "bf16p3" : BIG ? "bf16p4" : PS ? "bf16p" : "s3", R, CW,
                 Epi::STATS ? "EpiStoreStats" : is_bnsums<Epi>::value ? "EpiStoreBnSums" : "EpiStore",
                 Epi::BF16 ? "B16" : "");
        prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
        prof_pop(st);
    } else {
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
    }
}
template <class Epi, bool PS = false>
void launch_win(const WinPick& w, const GemmArgs& a, hipStream_t st) {
    if constexpr (PS) {
        if (w.n96) {   // 256 x 96
            switch (w.CW) {
                case 128: launch_win1<PS, 2, 128, Epi, true, true>(a, st); return;
                case 64: launch_win1<PS, 4, 64, Epi, true, true>(a, st); return;
                case 32: launch_win1<PS, 8, 32, Epi, true, true>(a, st); return;
                case 16: launch_win1<PS, 16, 16, Epi, true, true>(a, st); return;
                case 8: launch_win1<PS, 32, 8, Epi, true, true>(a, st); return;
            }
            throw std::runtime_error("window conv: block shape not built");
        }
        if (w.big && w.R * w.CW == 256) {
            switch (w.CW) {
                case 128: launch_win1<PS, 2, 128, Epi, true>(a, st); return;
                case 64: launch_win1<PS, 4, 64, Epi, true>(a, st); return;
                case 32: launch_win1<PS, 8, 32, Epi, true>(a, st); return;
                case 16: launch_win1<PS, 16, 16, Epi, true>(a, st); return;
                case 8: launch_win1<PS, 32, 8, Epi, true>(a, st); return;
            }
            throw std::runtime_error("window conv: block shape not built");
        }
        if (w.big) {   // 512 x 64
            switch (w.CW) {
                case 128: launch_win1<PS, 4, 128, Epi, true>(a, st); return;
                case 64: launch_win1<PS, 8, 64, Epi, true>(a, st); return;
            }
            throw std::runtime_error("window conv: block shape not built");
        }
    }
    if (w.R * w.CW == 128) {
        switch (w.CW) {
            case 64: launch_win1<PS, 2, 64, Epi>(a, st); return;
            case 32: launch_win1<PS, 4, 32, Epi>(a, st); return;
            case 16: launch_win1<PS, 8, 16, Epi>(a, st); return;
            case 8: launch_win1<PS, 16, 8, Epi>(a, st); return;
        }
    } else {
        switch (w.CW) {
            case 128: launch_win1<PS, 2, 128, Epi>(a, st); return;
            case 64: launch_win1<PS, 4, 64, Epi>(a, st); return;
        }
    }
    throw std::runtime_error("window conv: block shape not built");
}
// B1 window kernel on the pre-split twins: 32-channel stages
WinPick pick_win_ps(int cin, int W, int N, int acoff) {
    WinPick w;
    if (engine() != 2 || cin % 32 || acoff % 8) return w;
    if (N % 128 == 0) {   // 256 x 128 tiles
        static const int cb[] = {128, 64, 32, 16, 8};
        for (int cw : cb)
            if (W % cw == 0) {
                w.CW = cw;
                w.R = 256 / cw;
                w.big = true;
                return w;
            }
        return w;
    }
    static const bool big64 = [] {   // A/B: CAD_WIN64=0 -> 256 x 64 tiles for N = 64
        const char* e = std::getenv("CAD_WIN64");
        return !(e && e[0] == '0');
    }();
    if (N == 64 && big64 && (W % 128 == 0 || W % 64 == 0)) {   // 512 x 64 tiles
        w.CW = W % 128 == 0 ? 128 : 64;
        w.R = 512 / w.CW;
        w.big = true;
        return w;
    }
    if (N % 96 == 0) {   // 256 x 96 tiles (f = 96: 96 and 192 channels)
        static const int cb[] = {128, 64, 32, 16, 8};
        for (int cw : cb)
            if (W % cw == 0) {
                w.CW = cw;
                w.R = 256 / cw;
                w.big = true;
                w.n96 = true;
                return w;
            }
        return w;
    }
    const int BM = N <= 64 ? 256 : 128;
    if (N % (BM == 128 ? 128 : 64)) return w;
    static const int c128[] = {64, 32, 16, 8}, c256[] = {128, 64};
    const int* cws = BM == 128 ? c128 : c256;
    const int ncw = BM == 128 ? 4 : 2;
    for (int i = 0; i < ncw; ++i)
        if (W % cws[i] == 0) {
            w.CW = cws[i];
            w.R = BM / cws[i];
            return w;
        }
    return w;
}

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

// deterministic split-K reduction of `splits` slabs of `per` floats into dw; two levels when there
// are many slabs (the L0 weight gradients: ~680): kSlabGroup slabs per level-1 group summed into the
// group's first slab, then the group heads, then the remainder slabs in order
constexpr int kSlabGroup = 24;
void slab_reduce(float* slab, int nsplit, int64_t per, int zstep, float* dst, unsigned bx, unsigned by, hipStream_t st) {
    // profiled (0 FLOP) so a launch profile shows which reduction plan ran
    if (prof_enabled()) prof_push("cad::k_slab_reduce(float*, int, long, int, float*, long)", 0.0, st);
    hipLaunchKernelGGL(k_slab_reduce, dim3(bx, by), dim3(256), 0, st, slab, nsplit, per, zstep, dst, per);
    if (prof_enabled()) prof_pop(st);
}
void finish_slabs(float* slab, int splits, int64_t per, float* dw, hipStream_t st) {
    const unsigned bx = (unsigned)cdiv(per / 4, 256);
    constexpr int G = kSlabGroup;
    if (splits >= 2 * G && bx < 512) {
        const int groups = splits / G;   // whole groups; the remainder slabs join level 2 one by one
        slab_reduce(slab, G, per, 1, nullptr, bx, groups, st);
        // level 2: group heads z = 0, G, 2G, ... then the remainder slabs groups*G .. splits-1.  Without
        // a remainder the level-2 total goes straight to dw; with one it lands next to the remainder (in
        // the consumed slab groups*G-1, not a group head) and is summed with it in order
        const int rem = splits - groups * G;
        if (rem == 0) {
            slab_reduce(slab, groups, per, G, dw, bx, 1, st);
        } else {
            float* tail = slab + (int64_t)(groups * G - 1) * per;
            slab_reduce(slab, groups, per, G, tail, bx, 1, st);
            slab_reduce(tail, rem + 1, per, 1, dw, bx, 1, st);
        }
        return;
    }
    slab_reduce(slab, splits, per, 1, dw, bx, 1, st);
}

// Weight gradient of the few-channel image layer on S3 (enc1.conv1: cin = 3 or 4, K = 27 / 36): the
// im2col GEMM runs it on 64 x 256 tiles of which one wave's 64 x 64 block is live (busy 0.25, 1.6 ms at
// bs32 480x640).  Here every wave of a workgroup owns the whole 64 (co) x 32 NJ (tap, ci) output for
// its own pixel range — a split-K inside the workgroup — and builds its MFMA fragments straight from
// global memory (dZ: 8 consecutive pixels of one co per lane; X: the 8 shifted pixels of one (tap, ci)),
// split exactly into three bf16 planes (the six S3 products, fp32 accumulation).  The four waves'
// accumulators are summed in LDS in wave order; workgroup partials go through the slab reduction.
template <int NJ>
__global__ __launch_bounds__(256) void k_wgrad_narrow_s3(const float* __restrict__ dz, int64_t ldz,
                                                         const float* __restrict__ x, int64_t ldx, int xoff, int cin,
                                                         int cout, int B, int H, int W, int ppw,
                                                         float* __restrict__ out) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c = lane & 31;
    const int NK = 9 * cin;
    const int cob = blockIdx.y * 64;
    const int M = B * H * W;
    const int p0 = (blockIdx.x * 4 + wave) * ppw, p1 = min(M, p0 + ppw);
    int ntap[NJ], nci[NJ];
    bool nok[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int n = 32 * j + c;
        nok[j] = n < NK;
        ntap[j] = nok[j] ? n / cin : 0;
        nci[j] = nok[j] ? n - ntap[j] * cin : 0;
    }
    floatx16 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int k0 = p0; k0 < p1; k0 += 16) {
        const int pb = k0 + 8 * h;   // this lane's 8 pixels pb .. pb + 7
        float av[2][8], bv[NJ][8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const bool ok = pb + e < p1;
#pragma unroll
            for (int i = 0; i < 2; ++i) av[i][e] = ok ? dz[(int64_t)(pb + e) * ldz + cob + 32 * i + c] : 0.f;
        }
        int xx = pb % W, r = pb / W, yy = r % H;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int p = pb + e;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int dy = ntap[j] / 3 - 1, dx = ntap[j] % 3 - 1;
                const bool ok = nok[j] && p < p1 && (unsigned)(yy + dy) < (unsigned)H && (unsigned)(xx + dx) < (unsigned)W;
                bv[j][e] = ok ? x[(int64_t)(p + dy * W + dx) * ldx + xoff + nci[j]] : 0.f;
            }
            if (++xx == W) { xx = 0; if (++yy == H) yy = 0; }
        }
        bf16x8 fa[2][3], fb[NJ][3];
        auto pack = [](const float (&v)[8], bf16x8 (&f)[3]) {
            const auto sa = split_np<3>(make_float4(v[0], v[1], v[2], v[3]));
            const auto sb = split_np<3>(make_float4(v[4], v[5], v[6], v[7]));
#pragma unroll
            for (int q = 0; q < 3; ++q)
                f[q] = __builtin_bit_cast(bf16x8, make_uint4(sa.p[q].x, sa.p[q].y, sb.p[q].x, sb.p[q].y));
        };
#pragma unroll
        for (int i = 0; i < 2; ++i) pack(av[i], fa[i]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) pack(bv[j], fb[j]);
        constexpr int P[6] = {2, 1, 0, 1, 0, 0};
        constexpr int Q[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][P[u]], fb[j][Q[u]], acc[i][j], 0, 0, 0);
    }
    // the four waves' partials, summed in wave order (one 32-row block i at a time: 16 NJ values per lane)
    __shared__ float red[3][NJ * 16][64];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (i) __syncthreads();   // the previous round's reads are done
        if (wave > 0)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) red[wave - 1][j * 16 + r][lane] = acc[i][j][r];
        __syncthreads();
        if (wave == 0)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int sidx = j * 16 + r;
                    const float v = ((acc[i][j][r] + red[0][sidx][lane]) + red[1][sidx][lane]) + red[2][sidx][lane];
                    // accumulator layout: row (co) 32 i + 8 (r / 4) + 4 h + r % 4, column n = 32 j + c
                    const int co = cob + 32 * i + 8 * (r >> 2) + 4 * h + (r & 3), n = 32 * j + c;
                    if (n < NK) out[((int64_t)blockIdx.x * cout + co) * NK + n] = v;
                }
    }
}
bool wgrad_narrow_s3(const float* dz, int64_t ldz, const float* x, int64_t ldx, int xoff, int cin, int cout, float* dw,
                     int B, int H, int W, float* slab, int64_t slab_cap, hipStream_t st) {
    static const bool on = [] {
        const char* e = std::getenv("CAD_WGNARROW");   // A/B: CAD_WGNARROW=0 keeps the im2col GEMM
        return !(e && e[0] == '0');
    }();
    if (!on || engine() != 1 || cin < 1 || cin > 10 || cout % 64) return false;
    const int64_t M = (int64_t)B * H * W;
    if (M >= ((int64_t)1 << 31) - 64) return false;
    const int64_t per = (int64_t)cout * 9 * cin;
    if (per % 4) return false;
    int s = (int)std::min<int64_t>(2048, std::max<int64_t>(1, M / 1024));
    if (slab_cap > 0) s = (int)std::max<int64_t>(1, std::min<int64_t>(s, slab_cap / per));
    const int ppw = (int)cdiv(cdiv(M, (int64_t)s * 4), 16) * 16;
    s = (int)cdiv(M, (int64_t)ppw * 4);
    if (s > 1 && (int64_t)s * per > slab_cap) return false;
    float* out = s == 1 ? dw : slab;
    const dim3 grid(s, cout / 64);
    if (prof_enabled()) prof_push("cad::k_wgrad_narrow_s3", 2.0 * M * per, st);
    if (9 * cin <= 32)
        hipLaunchKernelGGL(k_wgrad_narrow_s3<1>, grid, dim3(256), 0, st, dz, ldz, x, ldx, xoff, cin, cout, B, H, W, ppw, out);
    else if (9 * cin <= 64)
        hipLaunchKernelGGL(k_wgrad_narrow_s3<2>, grid, dim3(256), 0, st, dz, ldz, x, ldx, xoff, cin, cout, B, H, W, ppw, out);
    else
        hipLaunchKernelGGL(k_wgrad_narrow_s3<3>, grid, dim3(256), 0, st, dz, ldz, x, ldx, xoff, cin, cout, B, H, W, ppw, out);
    if (prof_enabled()) prof_pop(st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
    return true;
}

// window-tiled weight gradient (S3): cout, cin multiples of 64, W a multiple of 16
bool use_wgrad_win(int cout, int cin, int W) {
    return engine() == 1 && cout % 64 == 0 && cin % 64 == 0 && W % 16 == 0;
}
// CAD_WGSTRIP=0: the row-major S3 window weight gradient (k_conv3x3_wgrad_win_s3) instead of the
// strip-order one (A/B switch)
bool wg_strip() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_WGSTRIP");
        return !(e && e[0] == '0');
    }();
    return on;
}
void launch_wgrad_win(GemmArgs& a, float* dw, float* slab, int64_t slab_cap, int64_t kbytes, hipStream_t st) {
    const int cin = a.b_cin;
    const int tiles = (a.M / 64) * (cin / 64);
    const int nst = a.K / 16;
    const bool strip = wg_strip();
    int s = std::max(1, std::min(cdiv(2048, tiles), nst / 32));
    const int64_t per = (int64_t)a.M * a.N;
    if (slab_cap > 0) s = (int)std::max<int64_t>(1, std::min<int64_t>(s, slab_cap / per));
    // operand window of a slice: its pixels (strip order: from its first image's start, one image more)
    const int64_t img = (int64_t)a.H * a.W;
    auto span_ok = [&](int splits) {
        const int64_t px = (int64_t)cdiv(nst, splits) * 16;
        const int64_t span = strip ? (cdiv(px, img) + 1) * img : px;
        return span * kbytes <= ((int64_t)1 << 30);
    };
    if (!span_ok(s)) {
        int need = s;
        while (!span_ok(need) && need < nst) ++need;
        if (!span_ok(need) || (int64_t)need * per > slab_cap)
            throw std::runtime_error("weight-gradient K-slice exceeds the 1 GB window and the slab");
        s = need;
    }
    a.kstages_per_split = cdiv(nst, s);
    s = cdiv(nst, a.kstages_per_split);
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    const dim3 grid(a.M / 64, cin / 64, s);
    const char* name = strip ? "void cad::k_conv3x3_wgrad_strip_s3(cad::GemmArgs)" : "void cad::k_conv3x3_wgrad_win_s3(cad::GemmArgs)";
    if (prof_enabled()) prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
    if (strip) hipLaunchKernelGGL(k_conv3x3_wgrad_strip_s3, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_conv3x3_wgrad_win_s3, grid, dim3(256), 0, st, a);
    if (prof_enabled()) prof_pop(st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

// weight-gradient GEMM (M x N over K = pixels): split-K slabs, then the deterministic reduction
template <template <int, int, int> class F, template <int, int, int> class T3, template <int, int, int> class TB>
void launch_wgrad(GemmArgs& a, float* dw, float* slab, int64_t slab_cap, int64_t kbytes, hipStream_t st) {
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = engine() == 1 ? kS3KB : engine() == 2 ? kB1KB : 16;
    int s = plan_splits(a, c, kb, slab_cap, kbytes);
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    launch_on_engine<F, T3, TB>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}
}  // namespace

void set_gemm_engine(int e) { g_engine = (e == 1 || e == 2) ? e : 0; }
int gemm_engine() { return engine(); }

int conv3x3_stats_rows(int cin, int B, int H, int W, int cout, bool ps) {
    const WinPick w = ps ? pick_win_ps(cin, W, cout, 0) : pick_win(cin, W, cout);
    if (w.R) return win_blocks(w, B, H, W);
    return cdiv((int64_t)B * H * W, tile_m(pick_cfg(B * H * W, cout)));
}

void conv3x3_fwd(const float* x, int64_t ldx, int xcoff, int cin, const float* w, int cout, float* y,
                 int64_t ldy, int ycoff, int B, int H, int W, float* stats, hipStream_t st) {
    CAD_NO_ALIAS("conv3x3_fwd", {aview(y, (int64_t)B * H * W, ldy, ycoff, cout, 4, "y")},
                 {aview(x, (int64_t)B * H * W, ldx, xcoff, cin, 4, "x"), aview(w, cout, 9 * cin, 0, 9 * cin, 4, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = cout; a.K = 9 * cin;
    a.B = B; a.H = H; a.W = W;
    a.A = x; a.lda = ldx; a.a_coff = xcoff; a.a_cin = cin;
    a.Bm = w; a.ldb = 9 * cin; a.b_coff = 0;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff;
    a.stats = stats;
    if (const WinPick w = pick_win(cin, W, cout); w.R) {
        if (stats) launch_win<EpiStoreStats>(w, a, st);
        else launch_win<EpiStore>(w, a, st);
        return;
    }
    const Cfg c = pick_cfg(a.M, a.N);
    if (stats) launch_engine<KConvFwdS, KConvFwdS3, KConvFwdSB>(c, true, a, st);
    else launch_engine<KConvFwd, KConvFwd3, KConvFwdB>(c, true, a, st);
}

void convT_fwd(const float* x, int64_t ldx, int cin, const float* wf, const float* bias, int cout,
               float* y, int64_t ldy, int ycoff, int B, int H, int W, hipStream_t st) {
    CAD_NO_ALIAS("convT_fwd", {aview(y, (int64_t)B * 4 * H * W, ldy, ycoff, cout, 4, "y")},
                 {aview(x, (int64_t)B * H * W, ldx, 0, cin, 4, "x"), aview(wf, 4 * cout, cin, 0, cin, 4, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = 4 * cout; a.K = cin;
    a.B = B; a.H = H; a.W = W;
    a.A = x; a.lda = ldx; a.a_coff = 0;
    a.Bm = wf; a.ldb = cin;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff; a.bias = bias;
    launch_engine<KConvTFwd, KConvTFwd3, KConvTFwdB>(pick_cfg(a.M, a.N), false, a, st);
}

void conv3x3_dgrad(const float* dz, int cout, const float* wd, int cin, float* dx, int64_t lddx,
                   int B, int H, int W, hipStream_t st) {
    CAD_NO_ALIAS("conv3x3_dgrad", {aview(dx, (int64_t)B * H * W, lddx, 0, cin, 4, "dx")},
                 {aview(dz, (int64_t)B * H * W, cout, 0, cout, 4, "dz"), aview(wd, cin, 9 * cout, 0, 9 * cout, 4, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 9 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = dz; a.lda = cout; a.a_coff = 0; a.a_cin = cout;
    a.Bm = wd; a.ldb = 9 * cout;
    a.C = dx; a.ldc = lddx; a.c_coff = 0;
    if (const WinPick w = pick_win(cout, W, cin); w.R) {
        launch_win<EpiStore>(w, a, st);
        return;
    }
    launch_engine<KConvFwd, KConvFwd3, KConvFwdB>(pick_cfg(a.M, a.N), true, a, st);
}

void convT_dgrad(const float* g, int64_t ldg, int gcoff, int cout, const float* wm, int cin, float* dx,
                 int B, int H, int W, hipStream_t st) {
    CAD_NO_ALIAS("convT_dgrad", {aview(dx, (int64_t)B * H * W, cin, 0, cin, 4, "dx")},
                 {aview(g, (int64_t)B * 4 * H * W, ldg, gcoff, cout, 4, "g"), aview(wm, cin, 4 * cout, 0, 4 * cout, 4, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 4 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = g; a.lda = ldg; a.a_coff = gcoff; a.a_cin = cout;
    a.Bm = wm; a.ldb = 4 * cout;
    a.C = dx; a.ldc = cin; a.c_coff = 0;
    launch_engine<KConvTDgrad, KConvTDgrad3, KConvTDgradB>(pick_cfg(a.M, a.N), false, a, st);
}

int64_t wgrad_slab_floats(int M, int N, int Kpix) {
    GemmArgs a{};
    a.M = M; a.N = N; a.K = Kpix;
    return (int64_t)plan_splits(a, pick_cfg(M, N), 16, 0, 0) * M * N;   // kb 16: the larger split count
}

void conv3x3_wgrad(const float* dz, int cout, const float* x, int64_t ldx, int xcoff, int cin, float* dw,
                   int B, int H, int W, float* slab, int64_t slab_cap, hipStream_t st) {
    CAD_NO_ALIAS("conv3x3_wgrad",
                 {aview(dw, cout, 9 * cin, 0, 9 * cin, 4, "dw"), aview(slab, 1, slab_cap, 0, slab ? slab_cap : 0, 4, "slab")},
                 {aview(dz, (int64_t)B * H * W, cout, 0, cout, 4, "dz"), aview(x, (int64_t)B * H * W, ldx, xcoff, cin, 4, "x")});
    GemmArgs a{};
    a.M = cout; a.N = 9 * cin; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = dz; a.lda = cout; a.a_coff = 0;
    a.Bm = x; a.ldb = ldx; a.b_coff = xcoff; a.b_cin = cin;
    if (use_wgrad_win(cout, cin, W)) {
        launch_wgrad_win(a, dw, slab, slab_cap, 4 * std::max<int64_t>(a.lda, ldx), st);
        return;
    }
    if (wgrad_narrow_s3(dz, cout, x, ldx, xcoff, cin, cout, dw, B, H, W, slab, slab_cap, st)) return;
    launch_wgrad<KConvWgrad, KConvWgrad3, KConvWgradB>(a, dw, slab, slab_cap, 4 * std::max<int64_t>(a.lda, ldx), st);
}

void convT_wgrad(const float* x, int cin, const float* g, int64_t ldg, int gcoff, int cout, float* dw,
                 int B, int H, int W, float* slab, int64_t slab_cap, hipStream_t st) {
    CAD_NO_ALIAS("convT_wgrad",
                 {aview(dw, cin, 4 * cout, 0, 4 * cout, 4, "dw"), aview(slab, 1, slab_cap, 0, slab ? slab_cap : 0, 4, "slab")},
                 {aview(x, (int64_t)B * H * W, cin, 0, cin, 4, "x"), aview(g, (int64_t)B * 4 * H * W, ldg, gcoff, cout, 4, "g")});
    GemmArgs a{};
    a.M = cin; a.N = 4 * cout; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = x; a.lda = cin; a.a_coff = 0;
    a.Bm = g; a.ldb = ldg; a.b_coff = gcoff; a.b_cin = cout;
    launch_wgrad<KConvTWgrad, KConvTWgrad3, KConvTWgradB>(a, dw, slab, slab_cap, 4 * std::max<int64_t>(a.lda, 4 * ldg),
                                                           st);
}

// ------------------------------------------------------------------------------------------
// pre-split launchers (B1 engine: operands written as bf16 twins by their producers)
// ------------------------------------------------------------------------------------------
int split_planes() { return engine() == 2 ? 1 : 0; }

void split_rows(const float* x, int64_t ldx, int xcoff, int C, int64_t M, void* out, int64_t ldo, int ocoff,
                hipStream_t st) {
    if (C % 8 || xcoff % 4 || ldx % 4 || ocoff % 8 || ldo % 8) throw std::runtime_error("split_rows: alignment");
    if (split_planes() != 1) throw std::runtime_error("split_rows needs the bf16 engine");
    CAD_NO_ALIAS("split_rows", {aview(out, M, ldo, ocoff, C, 2, "out")}, {aview(x, M, ldx, xcoff, C, 4, "x")});
    const int G = C / 8;
    const int64_t n = M * G;
    if (n == 0) return;
    hipLaunchKernelGGL(k_split_rows<1>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, ldx, xcoff, G, n,
                       (char*)out, ldo, ocoff);
}

namespace {
void ps_check(const Split& s, int channels, const char* what) {
    if (!s.p || s.ld % 8 || s.coff % 8 || channels % 8) throw std::runtime_error(std::string("pre-split operand: ") + what);
    if (engine() != 2) throw std::runtime_error("pre-split GEMM launched off the bf16 engine");
}
}  // namespace

void conv3x3_fwd_ps(Split x, int cin, Split w, int cout, float* y, int64_t ldy, int ycoff, int B, int H, int W,
                    float* stats, hipStream_t st, bool y_bf16) {
    ps_check(x, cin, "conv3x3_fwd x");
    ps_check(w, 9 * cin, "conv3x3_fwd w");
    CAD_NO_ALIAS("conv3x3_fwd_ps", {aview(y, (int64_t)B * H * W, ldy, ycoff, cout, y_bf16 ? 2 : 4, "y")},
                 {aview(x.p, (int64_t)B * H * W, x.ld, x.coff, cin, 2, "x"), aview(w.p, cout, w.ld, w.coff, 9 * cin, 2, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = cout; a.K = 9 * cin;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)x.p; a.lda = x.ld; a.a_coff = x.coff; a.a_cin = cin;
    a.Bm = (const float*)w.p; a.ldb = w.ld; a.b_coff = w.coff;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff;
    a.stats = stats;
    if (const WinPick wp = pick_win_ps(cin, W, cout, x.coff); wp.R && w.coff == 0) {
        if (y_bf16) {
            if (stats) launch_win<EpiStoreStatsB16, true>(wp, a, st);
            else launch_win<EpiStoreB16, true>(wp, a, st);
        } else {
            if (stats) launch_win<EpiStoreStats, true>(wp, a, st);
            else launch_win<EpiStore, true>(wp, a, st);
        }
        return;
    }
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(true, c);
    a.kstages_per_split = cdiv(a.K, kb);
    // channel-major K order: the nine taps of a channel block re-read the same input rows back to back
    a.cimajor = cin % kb == 0;
    if (y_bf16) {
        if (stats) launch_kb<KConvFwdSP1B, 32, 64>(c, kb, a, 1, st);
        else launch_kb<KConvFwdP1B, 32, 64>(c, kb, a, 1, st);
    } else {
        if (stats) launch_kb<KConvFwdSP1, 32, 64>(c, kb, a, 1, st);
        else launch_kb<KConvFwdP1, 32, 64>(c, kb, a, 1, st);
    }
}

// conv2's input gradient with bn1's backward column sums from the window epilogue (EpiStoreBnSums):
// returns the number of tiles whose partials it wrote (0: no window kernel for this shape or the
// partials do not fit; nothing launched, the caller takes the unfused path).  S3 engine only: measured
// on MI355X (tools/ab_step.py, same box) fp32 configs[1] 225.7 -> 223.9 ms/step; the bf16 engine's
// form (bf16 dL/da1, the same epilogue on the B1 window kernels) made configs[3] 64.1 -> 68.2 ms/step —
// the per-element y load and fp64 sums in the epilogue cost its cheap GEMMs more than the
// column-reduction pass they replace
namespace {
template <bool OB16, bool PS>
int dgrad_bnsums_launch(const WinPick& wp, GemmArgs& a, const BnSums& bn, hipStream_t st) {
    const int tiles = win_blocks(wp, a.B, a.H, a.W);
    if (!bn.part || (int64_t)tiles * 2 * a.N > bn.part_cap) return 0;
    a.bn_g = bn.y; a.bn_ldg = bn.ldy;
    a.bn_mean = bn.mean; a.bn_invstd = bn.invstd; a.bn_scale = bn.scale; a.bn_shift = bn.shift;
    a.bn_part = bn.part;
    if (bn.y_bf16) launch_win<EpiStoreBnSums<OB16, true>, PS>(wp, a, st);
    else launch_win<EpiStoreBnSums<OB16, false>, PS>(wp, a, st);
    return tiles;
}
}  // namespace

int conv3x3_dgrad_bnsums(const float* dz, int cout, const float* wd, int cin, float* dx, int64_t lddx, int B, int H,
                         int W, const BnSums& bn, hipStream_t st) {
    const WinPick w = pick_win(cout, W, cin);
    if (!w.R || bn.y_bf16) return 0;
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 9 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = dz; a.lda = cout; a.a_coff = 0; a.a_cin = cout;
    a.Bm = wd; a.ldb = 9 * cout;
    a.C = dx; a.ldc = lddx; a.c_coff = 0;
    return dgrad_bnsums_launch<false, false>(w, a, bn, st);
}

bool conv3x3_dgrad_split_ok(Split dz, int cout, Split wd, int cin, int W, int split_n) {
    return split_n > 0 && split_n % 32 == 0 && split_n < cin && pick_win_ps(cout, W, cin, dz.coff).R && wd.coff == 0;
}

bool conv3x3_dgrad_ps(Split dz, int cout, Split wd, int cin, float* dx, int64_t lddx, int B, int H, int W,
                      hipStream_t st, bool dx_bf16, void* hi, int64_t ldhi, int split_n) {
    // the split store needs 32-column blocks on one side of split_n; otherwise dx is written whole
    // (in fp32: a bf16 lower half needs the split, conv3x3_dgrad_split_ok)
    if (hi && (!conv3x3_dgrad_split_ok(dz, cout, wd, cin, W, split_n) || ldhi < cin - split_n)) {
        if (dx_bf16) throw std::runtime_error("conv3x3_dgrad_ps: bf16 split store not possible for this shape");
        hi = nullptr;
    }
    ps_check(dz, cout, "conv3x3_dgrad dz");
    ps_check(wd, 9 * cout, "conv3x3_dgrad w");
    CAD_NO_ALIAS("conv3x3_dgrad_ps",
                 {aview(dx, (int64_t)B * H * W, lddx, 0, hi ? split_n : cin, dx_bf16 ? 2 : 4, "dx"),
                  aview(hi, (int64_t)B * H * W, ldhi, 0, hi ? cin - split_n : 0, 2, "hi (split store)")},
                 {aview(dz.p, (int64_t)B * H * W, dz.ld, dz.coff, cout, 2, "dz"), aview(wd.p, cin, wd.ld, wd.coff, 9 * cout, 2, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 9 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)dz.p; a.lda = dz.ld; a.a_coff = dz.coff; a.a_cin = cout;
    a.Bm = (const float*)wd.p; a.ldb = wd.ld; a.b_coff = wd.coff;
    a.C = dx; a.ldc = lddx; a.c_coff = 0;
    if (const WinPick wp = pick_win_ps(cout, W, cin, dz.coff); wp.R && wd.coff == 0) {
        if (hi) {
            a.C2 = hi; a.ldc2 = ldhi; a.split_n = split_n;
            if (dx_bf16) launch_win<EpiStoreSplit2B16, true>(wp, a, st);
            else launch_win<EpiStoreSplitB16, true>(wp, a, st);
            return true;
        }
        if (dx_bf16) launch_win<EpiStoreB16, true>(wp, a, st);
        else launch_win<EpiStore, true>(wp, a, st);
        return false;
    }
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(true, c);
    a.kstages_per_split = cdiv(a.K, kb);
    a.cimajor = cout % kb == 0;
    if (dx_bf16) launch_kb<KConvFwdP1B, 32, 64>(c, kb, a, 1, st);
    else launch_kb<KConvFwdP1, 32, 64>(c, kb, a, 1, st);
    return false;
}

// B1 window weight gradient (conv3x3_wgrad_win_ps_body): stage = P pixels of an image row
#ifndef CAD_WGWIN_P
#define CAD_WGWIN_P 32
#endif
#ifdef CAD_NO_WGWIN   // A/B builds (make VARIANT=... EXTRA=-DCAD_NO_WGWIN): the im2col kernel only
constexpr bool g_no_wgwin = true;
#else
constexpr bool g_no_wgwin = false;
#endif
int wgrad_win_ps_stage(int cout, int cin, int W) {
    if (cout % 64 || cin % 64) return 0;
    static const int pref = [] {
        const char* e = std::getenv("CAD_WGP");   // A/B tuning: preferred stage width (64 | 32)
        return (e && e[0] == '6') ? 64 : CAD_WGWIN_P;
    }();
    for (int p : {pref, 32, 16})
        if (W % p == 0) return p;
    return 0;
}
// LDS-DMA weight-gradient kernel (k_conv3x3_wgrad_win_bf16d): default (MI355X, configs[3] shapes:
// 1016 vs 996 TFLOP/s at 32-pixel stages, 890 vs 830 at 16); CAD_WGDMA=0 selects the register-staged
// one (A/B switch)
bool wg_dma() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_WGDMA");
        return !(e && e[0] == '0');
    }();
    return on;
}
// ring depth of the DMA kernel (CAD_WGBUF=2|3; A/B tuning switch)
int wg_nbuf() {
    static const int n = [] {
        const char* e = std::getenv("CAD_WGBUF");
        return (e && e[0] == '2') ? 2 : 3;
    }();
    return n;
}
// strip weight gradients two output rows per step (conv3x3_wgrad_strip2_dma_body; 16- and 32-pixel
// stages): measured on MI355X (tools/winlab.py, configs[3] shapes) 886 -> 1106 TFLOP/s at level 3,
// 753 -> 820 / 977 -> 1053 / 1024 -> 1110 at levels 0-2; configs[3] 63.07 -> 61.32 ms/step (same box).
// Within a K-slice each accumulator takes the rows in the same order as the one-row walk, but slices
// now split at row pairs, so the split-K partials (and the slab sums) can differ by fp32 rounding.
// CAD_WGSTRIP2=0: one row per step (A/B switch)
bool wg_strip2() {
    static const bool on = [] {
        const char* e = std::getenv("CAD_WGSTRIP2");
        return !(e && e[0] == '0');
    }();
    return on;
}
template <int P>
void launch_wgrad_win_ps1(GemmArgs& a, float* dw, float* slab, int64_t slab_cap, hipStream_t st) {
    const int cin = a.b_cin;
    const int tiles = (a.M / 64) * (cin / 64);
    const bool dma = wg_dma();
    const bool strip = dma && wg_strip();
    const bool strip2 = strip && (P == 16 || P == 32) && wg_strip2();
    const int RS = strip2 ? 2 : 1;   // output rows per stage
    const int nst = strip2 ? a.B * (a.W / P) * cdiv(a.H, 2) : a.K / P;
    static const int wgs = [] {   // A/B: CAD_WGSLABS = workgroups the split-K aims for (default 2048)
        const char* e = std::getenv("CAD_WGSLABS");
        return e && e[0] ? std::max(64, std::atoi(e)) : 2048;
    }();
    int s = std::max(1, std::min(cdiv(wgs, tiles), nst / 16));
    const int64_t per = (int64_t)a.M * a.N;
    if (slab_cap > 0) s = (int)std::max<int64_t>(1, std::min<int64_t>(s, slab_cap / per));
    // a K-slice is a loader window of 32-bit byte offsets: keep it below 1 GB in either operand (the
    // strip walk's window starts at the slice's first image: one image more)
    const int64_t kbytes = 2 * std::max<int64_t>(a.lda, a.ldb);
    const int64_t img = (int64_t)a.H * a.W;
    auto span_ok = [&](int splits) {
        const int64_t px = (int64_t)cdiv(nst, splits) * P * RS;
        const int64_t span = strip ? (cdiv(px, img) + 1) * img : px;
        return span * kbytes <= ((int64_t)1 << 30);
    };
    if (!span_ok(s)) {
        int need = s;
        while (!span_ok(need) && need < nst) ++need;
        if (!span_ok(need) || (int64_t)need * per > slab_cap)
            throw std::runtime_error("weight-gradient K-slice exceeds the 1 GB window and the slab");
        s = need;
    }
    a.kstages_per_split = cdiv(nst, s);
    s = cdiv(nst, a.kstages_per_split);
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    const dim3 grid(a.M / 64, cin / 64, s);
    const int nbuf = wg_nbuf();
    char name[96];
    if (strip2) std::snprintf(name, sizeof name, "void cad::k_conv3x3_wgrad_strip2_bf16d<%d>(cad::GemmArgs)", P);
    else if (strip) std::snprintf(name, sizeof name, "void cad::k_conv3x3_wgrad_strip_bf16d<%d>(cad::GemmArgs)", P);
    else if (dma) std::snprintf(name, sizeof name, "void cad::k_conv3x3_wgrad_win_bf16d<%d, %d>(cad::GemmArgs)", P, nbuf);
    else std::snprintf(name, sizeof name, "void cad::k_conv3x3_wgrad_win_bf16p<%d>(cad::GemmArgs)", P);
    if (prof_enabled()) prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
    if (strip2) hipLaunchKernelGGL(k_conv3x3_wgrad_strip2_bf16d<P == 32 ? 32 : 16>, grid, dim3(256), 0, st, a);
    else if (strip) hipLaunchKernelGGL(k_conv3x3_wgrad_strip_bf16d<P>, grid, dim3(256), 0, st, a);
    else if (dma && nbuf == 2) hipLaunchKernelGGL((k_conv3x3_wgrad_win_bf16d<P, 2>), grid, dim3(256), 0, st, a);
    else if (dma) hipLaunchKernelGGL((k_conv3x3_wgrad_win_bf16d<P, 3>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_conv3x3_wgrad_win_bf16p<P>, grid, dim3(256), 0, st, a);
    if (prof_enabled()) prof_pop(st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

// 32-channel weight gradient as a 64-channel one on pixel pairs (config 5's dec0: cout = cin = 32 at full
// resolution, which the 64-channel window tiles do not take; the im2col kernel ran it at ~215 TFLOP/s).
// Dense twins (ld = 32) read as rows of 64 channels are images of W / 2 pixel pairs: channel e 32 + c of
// pair x' is channel c of pixel 2 x' + e.  The 64 x 64 x 9 window weight gradient of that view,
// P[(e, co)][(ky, t)][(f, ci)] = sum dZ[y][2x' + e][co] X[y + ky - 1][2x' + 2t + f][ci] (t = -1, 0, 1),
// holds every horizontal offset dx = 2t + f - e of the 3x3 kernel once per output parity e (the
// zero padding at x' = -1, W/2 is that of pixels -2, -1, W, W + 1): dW[co][ky][dx][ci] =
// P(e = 0, the (t, f) with 2t + f = dx) + P(e = 1, 2t + f = dx + 1).  Twice the MFMAs of the 32-channel
// product (the other blocks are discarded) at the window kernels' rate.
__global__ void k_wgrad_pair_fold(const float* __restrict__ pr, float* __restrict__ dw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // dw[co][tap][ci], 32 x 9 x 32
    if (i >= 32 * 288) return;
    const int co = i / 288, n = i - co * 288, tap = n >> 5, ci = n & 31;
    const int ky = tap / 3, dx = tap - 3 * ky - 1;
    const int q0 = dx + 2, t0 = (q0 >> 1) - 1, f0 = q0 & 1;   // e = 0: 2t + f = dx (with q = 2(t + 1) + f)
    const int q1 = dx + 3, t1 = (q1 >> 1) - 1, f1 = q1 & 1;   // e = 1: 2t + f = dx + 1
    const float v0 = pr[(int64_t)co * 576 + (ky * 3 + t0 + 1) * 64 + f0 * 32 + ci];
    const float v1 = pr[(int64_t)(32 + co) * 576 + (ky * 3 + t1 + 1) * 64 + f1 * 32 + ci];
    dw[i] = v0 + v1;
}
bool wg_pair32() {   // CAD_WGPAIR=0: the im2col kernel for the 32-channel weight gradient (A/B switch)
    static const bool on = [] {
        const char* e = std::getenv("CAD_WGPAIR");
        return !(e && e[0] == '0');
    }();
    return on;
}

void conv3x3_wgrad_ps(Split dz, int cout, Split x, int cin, float* dw, int B, int H, int W, float* slab,
                      int64_t slab_cap, hipStream_t st) {
    ps_check(dz, cout, "conv3x3_wgrad dz");
    ps_check(x, cin, "conv3x3_wgrad x");
    CAD_NO_ALIAS("conv3x3_wgrad_ps",
                 {aview(dw, cout, 9 * cin, 0, 9 * cin, 4, "dw"), aview(slab, 1, slab_cap, 0, slab ? slab_cap : 0, 4, "slab")},
                 {aview(dz.p, (int64_t)B * H * W, dz.ld, dz.coff, cout, 2, "dz"),
                  aview(x.p, (int64_t)B * H * W, x.ld, x.coff, cin, 2, "x")});
    constexpr int64_t kPairPer = 64 * 576;
    if (!g_no_wgwin && cout == 32 && cin == 32 && dz.ld == 32 && x.ld == 32 && dz.coff == 0 && x.coff == 0 &&
        W % 2 == 0 && slab && slab_cap >= 2 * kPairPer && wg_pair32()) {
        const int P = wgrad_win_ps_stage(64, 64, W / 2);
        if (P) {
            GemmArgs a{};
            a.M = 64; a.N = 576; a.K = B * H * (W / 2);
            a.B = B; a.H = H; a.W = W / 2;
            a.A = (const float*)dz.p; a.lda = 64; a.a_coff = 0;
            a.Bm = (const float*)x.p; a.ldb = 64; a.b_coff = 0; a.b_cin = 64;
            float* pr = slab + (slab_cap - kPairPer);   // the pair product, after the split-K slabs
            switch (P) {
                case 64: launch_wgrad_win_ps1<64>(a, pr, slab, slab_cap - kPairPer, st); break;
                case 32: launch_wgrad_win_ps1<32>(a, pr, slab, slab_cap - kPairPer, st); break;
                default: launch_wgrad_win_ps1<16>(a, pr, slab, slab_cap - kPairPer, st); break;
            }
            hipLaunchKernelGGL(k_wgrad_pair_fold, dim3(cdiv(32 * 288, 256)), dim3(256), 0, st, pr, dw);
            return;
        }
    }
    GemmArgs a{};
    a.M = cout; a.N = 9 * cin; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)dz.p; a.lda = dz.ld; a.a_coff = dz.coff;
    a.Bm = (const float*)x.p; a.ldb = x.ld; a.b_coff = x.coff; a.b_cin = cin;
    if (!g_no_wgwin)
        switch (wgrad_win_ps_stage(cout, cin, W)) {
            case 64: launch_wgrad_win_ps1<64>(a, dw, slab, slab_cap, st); return;
            case 32: launch_wgrad_win_ps1<32>(a, dw, slab, slab_cap, st); return;
            case 16: launch_wgrad_win_ps1<16>(a, dw, slab, slab_cap, st); return;
        }
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(false, c);
    int s = plan_splits(a, c, kb, slab_cap, 2 * kMaxPlanes * std::max<int64_t>(dz.ld, x.ld));
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    launch_kb<KConvWgradP1, 32>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

int dense_stats_rows(int64_t M, int N) { return cdiv(M, tile_m(pick_cfg((int)M, N))); }

void launch_dense_dma(void (*fn)(GemmArgs), const char* name, const GemmArgs& a, hipStream_t st);
void dense_fwd_ps(Split x, int K, Split w, int N, float* y, int64_t ldy, int ycoff, int64_t M, float* stats,
                  hipStream_t st, bool y_bf16, const float* add, const float* mask, int64_t ldadd) {
    if (mask && !add) throw std::runtime_error("dense GEMM: a mask needs the added matrix");
    if (ldadd == 0) ldadd = ldy;
    if (add && ldadd != ldy && (mask || ycoff || ldadd < N))
        throw std::runtime_error("dense GEMM: an added matrix of its own stride takes no mask / offset");
    ps_check(x, K, "dense x");
    ps_check(w, K, "dense w");
    // add == y (same rows): the epilogue's in-place accumulate, declared
    CAD_NO_ALIAS("dense_fwd_ps", {aview(y, M, ldy, ycoff, N, y_bf16 ? 2 : 4, "y")},
                 {aview(x.p, M, x.ld, x.coff, K, 2, "x"), aview(w.p, N, w.ld, w.coff, K, 2, "w"),
                  aview(add == y && ldadd == ldy ? nullptr : add, M, ldadd, ldadd == ldy ? ycoff : 0, N, 4, "add"),
                  aview(mask, M, ldy, ycoff, N, 4, "mask")});
    if (M > INT32_MAX) throw std::runtime_error("dense GEMM: too many rows");
    GemmArgs a{};
    a.M = (int)M; a.N = N; a.K = K;
    a.B = 1; a.H = 1; a.W = (int)M;
    a.A = (const float*)x.p; a.lda = x.ld; a.a_coff = x.coff;
    a.Bm = (const float*)w.p; a.ldb = w.ld; a.b_coff = w.coff;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff;
    a.stats = stats;
    a.bias = add;
    a.C2 = const_cast<float*>(mask);
    a.ldc2 = ldadd;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(true, c);
    a.kstages_per_split = cdiv(a.K, kb);
    // the LDS-DMA dense GEMM on 128 x 128 tiles (config 5's 1x1 / im2col forward GEMMs: 571.5 -> 575.2
    // img/s on one box); CAD_DENSEDMA=0 keeps the register-staged gemm_body_ps kernels
    static const bool ddma = [] {
        const char* e = std::getenv("CAD_DENSEDMA");
        return !(e && e[0] == '0');
    }();
    if (ddma && c == C22 && K % 8 == 0 && x.ld % 8 == 0 && x.coff % 8 == 0 && w.ld % 8 == 0 && w.coff % 8 == 0) {
        if (add && (stats || y_bf16)) throw std::runtime_error("dense GEMM: the added matrix needs fp32 output");
        if (add && mask)
            launch_dense_dma(k_dense_bf16d<EpiStoreAddMask>, "void cad::k_dense_bf16d<cad::EpiStoreAddMask>(cad::GemmArgs)", a, st);
        else if (add && ldadd != ldy)
            launch_dense_dma(k_dense_bf16d<EpiStoreAddLd>, "void cad::k_dense_bf16d<cad::EpiStoreAddLd>(cad::GemmArgs)", a, st);
        else if (add) launch_dense_dma(k_dense_bf16d<EpiStoreAdd>, "void cad::k_dense_bf16d<cad::EpiStoreAdd>(cad::GemmArgs)", a, st);
        else if (y_bf16 && stats)
            launch_dense_dma(k_dense_bf16d<EpiStoreStatsB16>, "void cad::k_dense_bf16d<cad::EpiStoreStatsB16>(cad::GemmArgs)", a, st);
        else if (y_bf16) launch_dense_dma(k_dense_bf16d<EpiStoreB16>, "void cad::k_dense_bf16d<cad::EpiStoreB16>(cad::GemmArgs)", a, st);
        else if (stats) launch_dense_dma(k_dense_bf16d<EpiStoreStats>, "void cad::k_dense_bf16d<cad::EpiStoreStats>(cad::GemmArgs)", a, st);
        else launch_dense_dma(k_dense_bf16d<EpiStore>, "void cad::k_dense_bf16d<cad::EpiStore>(cad::GemmArgs)", a, st);
        return;
    }
    if (add && ldadd != ldy) {   // (the register-staged kernels: the GEMM, then an add pass)
        if (stats || y_bf16) throw std::runtime_error("dense GEMM: the added matrix needs fp32 output");
        a.bias = nullptr;
        launch_kb<KDenseP1, 32, 64>(c, kb, a, 1, st);
        add_strided(y, ldy, add, ldadd, 0, N, 1, 1, (int)M, 1, st);
    } else if (add) {
        if (stats || y_bf16) throw std::runtime_error("dense GEMM: the added matrix needs fp32 output");
        launch_kb<KDenseAddP1, 32, 64>(c, kb, a, 1, st);
        if (mask) mask_inplace(y, ldy, ycoff, mask, N, M, st);   // (the register-staged kernels: a pass)
    } else if (y_bf16) {
        if (stats) launch_kb<KDenseSP1B, 32, 64>(c, kb, a, 1, st);
        else launch_kb<KDenseP1B, 32, 64>(c, kb, a, 1, st);
    } else {
        if (stats) launch_kb<KDenseSP1, 32, 64>(c, kb, a, 1, st);
        else launch_kb<KDenseP1, 32, 64>(c, kb, a, 1, st);
    }
}

void dense_wgrad_ps(Split dz, int N, Split x, int K, float* dw, int64_t ldw, int64_t M, float* slab, int64_t slab_cap,
                    hipStream_t st) {
    ps_check(dz, N, "dense wgrad dz");
    ps_check(x, K, "dense wgrad x");
    CAD_NO_ALIAS("dense_wgrad_ps", {aview(dw, N, ldw, 0, K, 4, "dw"), aview(slab, 1, slab_cap, 0, slab ? slab_cap : 0, 4, "slab")},
                 {aview(dz.p, M, dz.ld, dz.coff, N, 2, "dz"), aview(x.p, M, x.ld, x.coff, K, 2, "x")});
    if (ldw != K) throw std::runtime_error("dense wgrad: dw rows must be dense");
    if (M > INT32_MAX) throw std::runtime_error("dense GEMM: too many rows");
    GemmArgs a{};
    a.M = N; a.N = K; a.K = (int)M;
    a.B = 1; a.H = 1; a.W = (int)M;
    a.A = (const float*)dz.p; a.lda = dz.ld; a.a_coff = dz.coff;
    a.Bm = (const float*)x.p; a.ldb = x.ld; a.b_coff = x.coff;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(false, c);
    int s = plan_splits(a, c, kb, slab_cap, 2 * kMaxPlanes * std::max<int64_t>(dz.ld, x.ld));
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    launch_kb<KDenseWgradP1, 32>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

// CAD_BIGT bit 1: ConvT forward, bit 2: ConvT dgrad on the 256 x 128 tiles (bf16 outputs).  Measured at
// configs[3] (4 launches per step each): dgrad 1.20 -> 1.11 ms, forward 1.47 -> 1.49 ms; default 2
int bigt_mask() {
    static const int m = [] {
        const char* e = std::getenv("CAD_BIGT");
        return e && e[0] ? std::atoi(e) : 2;
    }();
    return m;
}
void launch_big(void (*fn)(GemmArgs), const char* name, const GemmArgs& a, hipStream_t st) {
    const dim3 grid(cdiv(a.M, 256), cdiv(a.N, 128), 1);
    if (prof_enabled()) {
        prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
        prof_pop(st);
    } else {
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
    }
}
// CAD_CONVTDMA bit 1: the bf16 ConvT forward on the LDS-DMA dense GEMM.  Measured at configs[3] (4
// launches per step): 1.47 -> 1.42 ms (default on).  (Its up-gather input-gradient form, 1.13 ms
// against the 256 x 128 tiles' 1.11, was removed in round 5.)
int convt_dma() {
    static const int m = [] {
        const char* e = std::getenv("CAD_CONVTDMA");
        return e && e[0] ? std::atoi(e) : 1;
    }();
    return m;
}
void launch_dense_dma(void (*fn)(GemmArgs), const char* name, const GemmArgs& a, hipStream_t st) {
    const dim3 grid(cdiv(a.M, 128), cdiv(a.N, 128), 1);
    if (prof_enabled()) {
        prof_push(name, 2.0 * a.M * a.N * (double)a.K, st);
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
        prof_pop(st);
    } else {
        hipLaunchKernelGGL(fn, grid, dim3(256), 0, st, a);
    }
}
void convT_fwd_ps(Split x, int cin, Split wf, const float* bias, int cout, float* y, int64_t ldy, int ycoff, int B,
                  int H, int W, hipStream_t st, bool y_bf16) {
    ps_check(x, cin, "convT_fwd x");
    ps_check(wf, cin, "convT_fwd w");
    CAD_NO_ALIAS("convT_fwd_ps", {aview(y, (int64_t)B * 4 * H * W, ldy, ycoff, cout, y_bf16 ? 2 : 4, "y")},
                 {aview(x.p, (int64_t)B * H * W, x.ld, x.coff, cin, 2, "x"), aview(wf.p, 4 * cout, wf.ld, wf.coff, cin, 2, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = 4 * cout; a.K = cin;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)x.p; a.lda = x.ld; a.a_coff = x.coff;
    a.Bm = (const float*)wf.p; a.ldb = wf.ld; a.b_coff = wf.coff;
    a.C = y; a.ldc = ldy; a.c_coff = ycoff; a.bias = bias;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(false, c);
    a.kstages_per_split = cdiv(a.K, kb);
    if (y_bf16 && (convt_dma() & 1) && a.N >= 128 && a.K % 8 == 0 && a.lda % 8 == 0 && a.a_coff % 8 == 0) {
        launch_dense_dma(k_convT_fwd_bf16dt, "void cad::k_convT_fwd_bf16dt(cad::GemmArgs)", a, st);
        return;
    }
    if (y_bf16 && (bigt_mask() & 1) && a.N >= 128 && a.M >= 4096) {
        launch_big(k_convT_fwd_bf16pt4<32>, "void cad::k_convT_fwd_bf16pt4<32>(cad::GemmArgs)", a, st);
        return;
    }
    if (y_bf16) launch_kb<KConvTFwdP1T, 32>(c, kb, a, 1, st);
    else launch_kb<KConvTFwdP1, 32>(c, kb, a, 1, st);
}

void convT_dgrad_ps(Split g, int cout, Split wm, int cin, float* dx, int B, int H, int W, hipStream_t st, bool dx_bf16) {
    ps_check(g, cout, "convT_dgrad g");
    ps_check(wm, 4 * cout, "convT_dgrad w");
    CAD_NO_ALIAS("convT_dgrad_ps", {aview(dx, (int64_t)B * H * W, cin, 0, cin, dx_bf16 ? 2 : 4, "dx")},
                 {aview(g.p, (int64_t)B * 4 * H * W, g.ld, g.coff, cout, 2, "g"), aview(wm.p, cin, wm.ld, wm.coff, 4 * cout, 2, "w")});
    GemmArgs a{};
    a.M = B * H * W; a.N = cin; a.K = 4 * cout;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)g.p; a.lda = g.ld; a.a_coff = g.coff; a.a_cin = cout;
    a.Bm = (const float*)wm.p; a.ldb = wm.ld; a.b_coff = wm.coff;
    a.C = dx; a.ldc = cin; a.c_coff = 0;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(false, c);
    a.kstages_per_split = cdiv(a.K, kb);
    if (dx_bf16 && (bigt_mask() & 2) && a.N >= 128 && a.M >= 4096) {
        launch_big(k_convT_dgrad_bf16pb4<32>, "void cad::k_convT_dgrad_bf16pb4<32>(cad::GemmArgs)", a, st);
        return;
    }
    if (dx_bf16) launch_kb<KConvTDgradP1B, 32>(c, kb, a, 1, st);
    else launch_kb<KConvTDgradP1, 32>(c, kb, a, 1, st);
}

void convT_wgrad_ps(Split x, int cin, Split g, int cout, float* dw, int B, int H, int W, float* slab,
                    int64_t slab_cap, hipStream_t st) {
    ps_check(x, cin, "convT_wgrad x");
    ps_check(g, cout, "convT_wgrad g");
    CAD_NO_ALIAS("convT_wgrad_ps",
                 {aview(dw, cin, 4 * cout, 0, 4 * cout, 4, "dw"), aview(slab, 1, slab_cap, 0, slab ? slab_cap : 0, 4, "slab")},
                 {aview(x.p, (int64_t)B * H * W, x.ld, x.coff, cin, 2, "x"),
                  aview(g.p, (int64_t)B * 4 * H * W, g.ld, g.coff, cout, 2, "g")});
    GemmArgs a{};
    a.M = cin; a.N = 4 * cout; a.K = B * H * W;
    a.B = B; a.H = H; a.W = W;
    a.A = (const float*)x.p; a.lda = x.ld; a.a_coff = x.coff;
    a.Bm = (const float*)g.p; a.ldb = g.ld; a.b_coff = g.coff; a.b_cin = cout;
    const Cfg c = pick_cfg(a.M, a.N);
    const int kb = ps_kb(false, c);
    int s = plan_splits(a, c, kb, slab_cap, 2 * kMaxPlanes * std::max<int64_t>(x.ld, 4 * g.ld));
    a.kstages_per_split = cdiv(cdiv(a.K, kb), s);
    s = cdiv(cdiv(a.K, kb), a.kstages_per_split);
    const int64_t per = (int64_t)a.M * a.N;
    a.ldc = a.N; a.slab_stride = per;
    a.C = s == 1 ? dw : slab;
    launch_kb<KConvTWgradP1, 32>(c, kb, a, s, st);
    if (s > 1) finish_slabs(slab, s, per, dw, st);
}

}  // namespace cad
