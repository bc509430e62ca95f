// Memory-bound NN kernels of the U-Net step: BatchNorm2d (train/eval),
// ReLU, MaxPool2d(2), ConvTranspose bias grad, the 1x1 depth head with sigmoid*max_depth, layout
// conversion of the NCHW rgb batch, weight repacks.  All NHWC fp32, float4-vectorised, and every
// reduction is deterministic (fixed-order partial slabs reduced in fp64; no atomics).
//
// Reference semantics:
//   BatchNorm2d: torch/nn/options/batchnorm.h:20-34 defaults (eps 1e-5, momentum 0.1, affine),
//     batch statistics for normalisation (biased var), unbiased var for running_var.
//   MaxPool2d(2): first maximum in kernel scan order wins (strict >), NaN propagates.
//   head: baseline_unet.h:191-192  x = out_conv(x); x = sigmoid(x) * max_depth
#include <algorithm>
#include <stdexcept>
#include <type_traits>
#include <utility>

#include "gemm_s3.hpp"   // split_np (pre-split twins written by the elementwise passes)
#include "ew_load.hpp"
#include "kernels.hpp"
#include "mx8_quant.hpp"

namespace cad {
// The BN apply and the head's dot product are written with explicit fma / mul so that every pass
// that evaluates them (bn_relu_fwd, the fused level-0 pass, the head kernels, the backward's
// rebuilds) rounds identically, whatever contraction the compiler would pick per kernel.
__device__ __forceinline__ float bn_relu1(float y, float s, float t) { return fmaxf(__fmaf_rn(y, s, t), 0.f); }
__device__ __forceinline__ float head_dot4(float4 a, float4 w) {
    return __fmaf_rn(a.w, w.w, __fmaf_rn(a.z, w.z, __fmaf_rn(a.y, w.y, __fmul_rn(a.x, w.x))));
}
namespace {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline int ew_blocks(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(n, 256)), 8192); }
}  // namespace

// ------------------------------------------------------------------------------------------
// generic deterministic column reduction: part[s][o][c] = sum_{rows r in slice s} op(r, c)[o]
// ------------------------------------------------------------------------------------------
// an Op may take its per-thread coefficients per slice (prep_slice(c4, r0, r1): the rows r0 .. r1 - 1 of
// the workgroup's slice) instead of per channel quad only (prep(c4))
template <class Op, class = void>
struct has_prep_slice : std::false_type {};
template <class Op>
struct has_prep_slice<Op, std::void_t<decltype(std::declval<const Op&>().prep_slice(0, int64_t{0}, int64_t{0}))>>
    : std::true_type {};
template <class Op>
__device__ __forceinline__ auto prep_of(const Op& op, int c4, int64_t r0, int64_t r1) {
    if constexpr (has_prep_slice<Op>::value) return op.prep_slice(c4, r0, r1);
    else return op.prep(c4);
}
template <int NOUT, class Op>
__global__ void k_colreduce(Op op, int64_t R, int C, int64_t rows_per_slice, double* part) {
    const int CX = blockDim.x, RY = blockDim.y;
    const int C4 = C >> 2;
    const int c4 = blockIdx.x * CX + threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_slice;
    const int64_t r1 = min(R, r0 + rows_per_slice);
    double acc[NOUT][4];
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[o][e] = 0.0;
    if (c4 < C4) {
        const auto pc = prep_of(op, c4, r0, r1);   // per-thread channel coefficients, loaded once
        for (int64_t r = r0 + threadIdx.y; r < r1; r += RY) op(r, c4, acc, pc);
    }
    extern __shared__ double red[];   // [RY][CX][NOUT*4]
    double* mine = red + ((int64_t)threadIdx.y * CX + threadIdx.x) * NOUT * 4;
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
        for (int e = 0; e < 4; ++e) mine[o * 4 + e] = acc[o][e];
    __syncthreads();
    if (threadIdx.y == 0 && c4 < C4) {
        for (int y = 1; y < RY; ++y) {
            const double* o2 = red + ((int64_t)y * CX + threadIdx.x) * NOUT * 4;
#pragma unroll
            for (int o = 0; o < NOUT; ++o)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[o][e] += o2[o * 4 + e];
        }
#pragma unroll
        for (int o = 0; o < NOUT; ++o)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                part[((int64_t)blockIdx.y * NOUT + o) * C + c4 * 4 + e] = acc[o][e];
    }
}

// tot[n] = sum_s part[s][n] (fixed order), optional float copy dst[n] = scale * tot[n]
constexpr int kFinalLanes = 16;   // slice lanes of k_colfinal (block 64 x 16)
__global__ void k_colfinal(const double* part, int S, int N, double* tot, float* dst, float scale) {
    const int n = blockIdx.x * 64 + threadIdx.x;
    const int sy = threadIdx.y;
    double s = 0.0;
    // unrolled so the independent loads of a thread are in flight together (the adds stay in order:
    // the same sum bit for bit); one load per iteration left it latency-bound (~20 us per launch)
    if (n < N)
#pragma unroll 8
        for (int i = sy; i < S; i += kFinalLanes) s += part[(int64_t)i * N + n];
    __shared__ double red[kFinalLanes][64];
    red[sy][threadIdx.x] = s;
    __syncthreads();
    if (sy == 0 && n < N) {
        s = 0.0;
        for (int y = 0; y < kFinalLanes; ++y) s += red[y][threadIdx.x];
        if (tot) tot[n] = s;
        if (dst) dst[n] = (float)(s * scale);
    }
}

namespace {
struct NoPrep {};
struct OpSum {
    const float* x; int64_t ld; int coff;
    __device__ NoPrep prep(int) const { return {}; }
    __device__ void operator()(int64_t r, int c4, double (&acc)[1][4], NoPrep) const {
        float4 v = *reinterpret_cast<const float4*>(x + r * ld + coff + c4 * 4);
        acc[0][0] += v.x; acc[0][1] += v.y; acc[0][2] += v.z; acc[0][3] += v.w;
    }
};
struct OpSumB16 {
    const float* x; int64_t ld; int coff;
    __device__ NoPrep prep(int) const { return {}; }
    __device__ void operator()(int64_t r, int c4, double (&acc)[1][4], NoPrep) const {
        const float4 v = load4<true>(x, r * ld + coff + c4 * 4);
        acc[0][0] += v.x; acc[0][1] += v.y; acc[0][2] += v.z; acc[0][3] += v.w;
    }
};
struct OpSumD {   // fp64 rows (per-tile partials of a recomputed convolution's BN backward)
    const double* x; int C;
    __device__ NoPrep prep(int) const { return {}; }
    __device__ void operator()(int64_t r, int c4, double (&acc)[1][4], NoPrep) const {
        const double* p = x + r * C + c4 * 4;
        acc[0][0] += p[0]; acc[0][1] += p[1]; acc[0][2] += p[2]; acc[0][3] += p[3];
    }
};
// BN tile partials (BnTilePartials, gemm_mfma.hpp): per tile row r, S = part[r][c], M2 = part[r][C + c],
// n = cnt[r]; column sums of S and of M2 + S^2 / n (= sum y^2 of the tile) in fp64
struct OpBnTile {
    const float* part; const float* cnt; int C;
    __device__ NoPrep prep(int) const { return {}; }
    __device__ void operator()(int64_t r, int c4, double (&acc)[2][4], NoPrep) const {
        const float4 s = *reinterpret_cast<const float4*>(part + r * 2 * C + c4 * 4);
        const float4 q = *reinterpret_cast<const float4*>(part + r * 2 * C + C + c4 * 4);
        const double n = cnt[r];
        if (n <= 0.0) return;
        const double sa[4] = {s.x, s.y, s.z, s.w}, qa[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            acc[0][e] += sa[e];
            acc[1][e] += qa[e] + sa[e] * sa[e] / n;
        }
    }
};
struct BnCoef {
    float sc[4], sh[4], mu[4], is[4], hw[4];
};
// HG: the upstream gradient is the depth head's, g[r][c] = dp[r] * w[c] with
// dp = dpred * max_depth * s (1 - s) (k_head_da's values, rebuilt per row instead of read)
// the folded max-pool backward (PoolAdd): row r of the full-resolution gradient receives the pooled
// gradient of its window where r is that window's recorded argmax — the same fp32 add the scatter
// (k_maxpool_bwd_scatter) makes
__device__ __forceinline__ float4 pool_add(const PoolAdd& pa, int C, int64_t r, int c, float4 gv) {
    const uint32_t rr = (uint32_t)r, W = (uint32_t)pa.W, H = (uint32_t)pa.H;
    const uint32_t t = fdiv(pa.divW, rr), b = fdiv(pa.divH, t);
    const uint32_t x = rr - t * W, y = t - b * H;
    const uint32_t op = (b * (H >> 1) + (y >> 1)) * (W >> 1) + (x >> 1);
    const int k = (int)(((y & 1) << 1) | (x & 1));
    const uchar4 a = *reinterpret_cast<const uchar4*>(pa.idx + (int64_t)op * C + c);
    if (a.x == k || a.y == k || a.z == k || a.w == k) {
        const float4 d = *reinterpret_cast<const float4*>(pa.d + (int64_t)op * C + c);
        if (a.x == k) gv.x += d.x;
        if (a.y == k) gv.y += d.y;
        if (a.z == k) gv.z += d.z;
        if (a.w == k) gv.w += d.w;
    }
    return gv;
}

// GB: g holds bf16 values (the bf16 engine's conv2 dgrad output); PA: max-pool backward folded in
template <bool YB, bool HG = false, bool GB = false, bool PA = false>
struct OpBnBwd {
    const float *g, *y, *mean, *invstd, *scale, *shift, *gmul;
    int64_t ldg; int gcoff, C; int64_t HW; bool relu;
    HeadGrad hg;
    PoolAdd pa;
    FastDiv dHW;   // row -> sample of gmul (rows < 2^32)
    __device__ BnCoef prep(int c4) const {
        BnCoef k;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int c = c4 * 4 + e;
            k.sc[e] = scale[c]; k.sh[e] = shift[c]; k.mu[e] = mean[c]; k.is[e] = invstd[c];
            if constexpr (HG) k.hw[e] = hg.w[c];
        }
        return k;
    }
    __device__ void operator()(int64_t r, int c4, double (&acc)[2][4], const BnCoef& k) const {
        float4 gv;
        if constexpr (HG) {
            const float s = hg.sig[r];
            const float dp = hg.dpred[r] * hg.md * ((1.f - s) * s);
            gv = make_float4(dp * k.hw[0], dp * k.hw[1], dp * k.hw[2], dp * k.hw[3]);
        } else {
            gv = load4<GB>(g, r * ldg + gcoff + c4 * 4);
            if constexpr (PA) gv = pool_add(pa, C, r, c4 * 4, gv);
            if (gmul) {
                const float4 m = *reinterpret_cast<const float4*>(gmul + (int64_t)fdiv(dHW, (uint32_t)r) * C + c4 * 4);
                gv.x *= m.x; gv.y *= m.y; gv.z *= m.z; gv.w *= m.w;
            }
        }
        float4 yv = load4<YB>(y, r * C + c4 * 4);
        const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, ya[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float z = __fmaf_rn(ya[e], k.sc[e], k.sh[e]);
            const float dz = (!relu || z > 0.f) ? ga[e] : 0.f;
            const float xh = (ya[e] - k.mu[e]) * k.is[e];
            acc[0][e] += dz;
            acc[1][e] += (double)dz * xh;
        }
    }
};
// OpBnBwd<YB, false, GB, true> walked over POOLED pixels (round 5): row op = pooled pixel, whose 2 x 2
// window's four full-resolution rows it visits with the argmax codes and the pooled gradient loaded
// once (the per-row walk re-derived the window by two divisions and re-read both for each of its four
// rows).  Each row takes the same fp32 add as pool_add; the fp64 sums run in another order.
__device__ __forceinline__ int64_t pool_window(const PoolAdd& pa, uint32_t op) {
    const uint32_t Wo = (uint32_t)pa.W >> 1, Ho = (uint32_t)pa.H >> 1;
    const uint32_t t = fdiv(pa.divW, op), b = fdiv(pa.divH, t);
    const uint32_t xo = op - t * Wo, yo = t - b * Ho;
    return ((int64_t)b * pa.H + 2 * yo) * pa.W + 2 * xo;   // full-res row of the window's (0, 0)
}
__device__ __forceinline__ float4 pool_add_k(uchar4 a, float4 d, int k, float4 gv) {
    if (a.x == k) gv.x += d.x;
    if (a.y == k) gv.y += d.y;
    if (a.z == k) gv.z += d.z;
    if (a.w == k) gv.w += d.w;
    return gv;
}
template <bool YB, bool GB>
struct OpBnBwdPoolQ {
    const float *g, *y, *mean, *invstd, *scale, *shift;
    int64_t ldg; int gcoff, C;
    PoolAdd pa;   // divW / divH: by the POOLED width / height
    __device__ BnCoef prep(int c4) const {
        BnCoef k;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int c = c4 * 4 + e;
            k.sc[e] = scale[c]; k.sh[e] = shift[c]; k.mu[e] = mean[c]; k.is[e] = invstd[c];
        }
        return k;
    }
    __device__ void operator()(int64_t op, int c4, double (&acc)[2][4], const BnCoef& k) const {
        const int c = c4 * 4;
        const int64_t p00 = pool_window(pa, (uint32_t)op);
        const uchar4 a = *reinterpret_cast<const uchar4*>(pa.idx + op * C + c);
        const float4 d = *reinterpret_cast<const float4*>(pa.d + op * C + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t r = p00 + (q >> 1) * pa.W + (q & 1);
            const float4 gv = pool_add_k(a, d, q, load4<GB>(g, r * ldg + gcoff + c));
            const float4 yv = load4<YB>(y, r * C + c);
            const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, ya[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float z = __fmaf_rn(ya[e], k.sc[e], k.sh[e]);
                const float dz = z > 0.f ? ga[e] : 0.f;
                const float xh = (ya[e] - k.mu[e]) * k.is[e];
                acc[0][e] += dz;
                acc[1][e] += (double)dz * xh;
            }
        }
    }
};
// OpBnBwd of a FiLM block (gmul = gamma[b][c]) that also forms the FiLM affine's sums in the same pass
// over (g, y): acc[2] = sum g a, acc[3] = sum g with g the raw gradient of the FiLM output and a =
// relu(y scale + shift) (k_film_reduce's sums; slices aligned to samples by the caller)
struct FilmCoef : BnCoef {
    float4 m;   // the slice's FiLM gamma (its rows lie in one sample: bn_relu_bwd's sample-aligned slices)
};
template <bool YB, bool GB>
struct OpBnBwdFilm {
    const float *g, *y, *mean, *invstd, *scale, *shift, *gmul;
    int64_t ldg; int gcoff, C; int64_t HW;
    FastDiv dHW;   // row -> sample (rows < 2^32)
    __device__ FilmCoef prep_slice(int c4, int64_t r0, int64_t) const {
        FilmCoef k;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int c = c4 * 4 + e;
            k.sc[e] = scale[c]; k.sh[e] = shift[c]; k.mu[e] = mean[c]; k.is[e] = invstd[c];
        }
        k.m = *reinterpret_cast<const float4*>(gmul + (int64_t)fdiv(dHW, (uint32_t)r0) * C + c4 * 4);
        return k;
    }
    __device__ void operator()(int64_t r, int c4, double (&acc)[4][4], const FilmCoef& k) const {
        const float4 gr = load4<GB>(g, r * ldg + gcoff + c4 * 4);
        const float4 m = k.m;
        const float4 yv = load4<YB>(y, r * C + c4 * 4);
        const float g0[4] = {gr.x, gr.y, gr.z, gr.w}, ga[4] = {gr.x * m.x, gr.y * m.y, gr.z * m.z, gr.w * m.w};
        const float ya[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float z = __fmaf_rn(ya[e], k.sc[e], k.sh[e]);
            const float dz = z > 0.f ? ga[e] : 0.f;
            const float xh = (ya[e] - k.mu[e]) * k.is[e];
            acc[0][e] += dz;
            acc[1][e] += (double)dz * xh;
            acc[2][e] += (double)g0[e] * fmaxf(z, 0.f);
            acc[3][e] += g0[e];
        }
    }
};
struct OpHeadBwd {
    const float *a, *dpred, *sig; float md; int C;
    __device__ NoPrep prep(int) const { return {}; }
    __device__ void operator()(int64_t r, int c4, double (&acc)[2][4], NoPrep) const {
        const float s = sig[r];
        const float dp = dpred[r] * md * ((1.f - s) * s);
        float4 v = *reinterpret_cast<const float4*>(a + r * C + c4 * 4);
        acc[0][0] += (double)dp * v.x; acc[0][1] += (double)dp * v.y;
        acc[0][2] += (double)dp * v.z; acc[0][3] += (double)dp * v.w;
        if (c4 == 0) acc[1][0] += dp;
    }
};
// the same sums with the head input a = relu(y * scale + shift) rebuilt from the level-0 BN input
// (bn_relu_head_fwd's values; the fp32 activation is never stored)
struct AffCoef {
    float sc[4], sh[4];
};
template <bool YB>
struct OpHeadBwdY {
    const float *y, *scale, *shift, *dpred, *sig; float md; int C;
    __device__ AffCoef prep(int c4) const {
        AffCoef k;
#pragma unroll
        for (int e = 0; e < 4; ++e) { k.sc[e] = scale[c4 * 4 + e]; k.sh[e] = shift[c4 * 4 + e]; }
        return k;
    }
    __device__ void operator()(int64_t r, int c4, double (&acc)[2][4], const AffCoef& k) const {
        const float s = sig[r];
        const float dp = dpred[r] * md * ((1.f - s) * s);
        const float4 yv = load4<YB>(y, r * C + c4 * 4);
        const float ya[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[0][e] += (double)dp * bn_relu1(ya[e], k.sc[e], k.sh[e]);
        if (c4 == 0) acc[1][0] += dp;
    }
};

template <int NOUT, class Op>
int launch_colreduce(const Op& op, int64_t R, int C, double* part, hipStream_t st) {
    const int C4 = C >> 2;
    const int CX = std::min(C4, 64);
    const int RY = std::max(1, 256 / CX);
    const int S = colsum_slices(R);
    const int64_t rps = (R + S - 1) / S;
    const size_t shm = (size_t)RY * CX * NOUT * 4 * sizeof(double);
    hipLaunchKernelGGL((k_colreduce<NOUT, Op>), dim3(cdiv(C4, CX), S), dim3(CX, RY), shm, st, op, R, C, rps, part);
    return S;
}
// ... with caller-chosen slices (S slices of rps rows)
template <int NOUT, class Op>
void launch_colreduce_slices(const Op& op, int64_t R, int C, int S, int64_t rps, double* part, hipStream_t st) {
    const int C4 = C >> 2;
    const int CX = std::min(C4, 64);
    const int RY = std::max(1, 256 / CX);
    const size_t shm = (size_t)RY * CX * NOUT * 4 * sizeof(double);
    hipLaunchKernelGGL((k_colreduce<NOUT, Op>), dim3(cdiv(C4, CX), S), dim3(CX, RY), shm, st, op, R, C, rps, part);
}
void launch_colfinal(const double* part, int S, int N, double* tot, float* dst, float scale, hipStream_t st) {
    hipLaunchKernelGGL(k_colfinal, dim3(cdiv(N, 64)), dim3(64, kFinalLanes), 0, st, part, S, N, tot, dst, scale);
}
}  // namespace

// Up to 2048 slices of >= CAD_COLSLICE_ROWS rows: a level-0 reduction (9.8 M rows x 16 channel quads)
// then runs 2048 workgroups, ~8 per CU (512 left it latency-bound at 2 per CU), and the deep,
// wide-channel ones (config 5's 1/16-resolution BNs: 38400 rows x 1024 channels) 4x more than with
// the round-4 256-row slices.  Monotone in R: the callers' dscr scratch must be sized from
// colsum_slices() of their largest reduction.
#ifndef CAD_COLSLICE_ROWS
#define CAD_COLSLICE_ROWS 64
#endif
int colsum_slices(int64_t R) { return (int)std::max<int64_t>(1, std::min<int64_t>(2048, R / CAD_COLSLICE_ROWS)); }

void colsum(const float* x, int64_t ld, int coff, int64_t R, int C, double* part, hipStream_t st) {
    launch_colreduce<1>(OpSum{x, ld, coff}, R, C, part, st);
}
void colsum_bf16(const void* x, int64_t ld, int coff, int64_t R, int C, double* part, hipStream_t st) {
    launch_colreduce<1>(OpSumB16{static_cast<const float*>(x), ld, coff}, R, C, part, st);
}
void colsum_finalize(const double* part, int S, int C, float* dst, float scale, hipStream_t st) {
    launch_colfinal(part, S, C, nullptr, dst, scale, st);
}

// ------------------------------------------------------------------------------------------
// BatchNorm forward
// ------------------------------------------------------------------------------------------
// The slice sums of both columns of a channel (part[s][0][c], part[s][1][c]: k_colreduce<2>'s
// layout) in k_colfinal's order, then the batch statistics, running statistics and the apply
// coefficients (scale = gamma * invstd, shift = beta - mean * scale)
__global__ void k_bn_final(const double* part, int S, int C, int64_t count, const float* gamma, const float* beta,
                           float* rmean, float* rvar, float momentum, float eps, float* mean, float* invstd,
                           float* scale, float* shift) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    const int sy = threadIdx.y;
    double s0 = 0.0, s1 = 0.0;
    if (c < C)
#pragma unroll 4
        for (int i = sy; i < S; i += kFinalLanes) {
            s0 += part[(int64_t)i * 2 * C + c];
            s1 += part[(int64_t)i * 2 * C + C + c];
        }
    __shared__ double red[2][kFinalLanes][64];
    red[0][sy][threadIdx.x] = s0;
    red[1][sy][threadIdx.x] = s1;
    __syncthreads();
    if (sy != 0 || c >= C) return;
    s0 = s1 = 0.0;
    for (int y = 0; y < kFinalLanes; ++y) {
        s0 += red[0][y][threadIdx.x];
        s1 += red[1][y][threadIdx.x];
    }
    const double mu = s0 / (double)count;
    double var = s1 / (double)count - mu * mu;
    if (var < 0.0) var = 0.0;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    mean[c] = (float)mu;
    invstd[c] = is;
    const float sc = gamma[c] * is;
    scale[c] = sc;
    shift[c] = beta[c] - (float)mu * sc;
    if (rmean) {
        const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
}

void bn_fwd_finalize(const float* tile_part, int rows, int C, int64_t count, const float* gamma,
                     const float* beta, float* run_mean, float* run_var, float momentum, float eps,
                     double* scratch, float* mean, float* invstd, float* scale, float* shift,
                     hipStream_t st) {
    double* part = scratch + 2 * C;
    // tile_part: [rows][2][C] (S, M2) then [rows] counts (BnTilePartials); the variance below is
    // E[y^2] - mu^2 in fp64 over per-tile sums y^2 rebuilt from the shifted partials.  Slices of about
    // one tile row per thread (a few thousand tile rows: colsum_slices' 256-row slices left each thread
    // a serial chain of 16-64 loads, ~50 us per launch); at most colsum_slices(count) of them, which the
    // callers' scratch holds (it is sized for the BN backward's 2-output reduction over `count` rows)
    const int C4 = C >> 2, CX = std::min(C4, 64), RY = std::max(1, 256 / CX);
    const int S = (int)std::max<int64_t>(1, std::min<int64_t>(colsum_slices(count), cdiv(rows, RY)));
    launch_colreduce_slices<2>(OpBnTile{tile_part, tile_part + (int64_t)rows * 2 * C, C}, rows, C, S, cdiv(rows, S),
                               part, st);
    hipLaunchKernelGGL(k_bn_final, dim3(cdiv(C, 64)), dim3(64, kFinalLanes), 0, st, part, S, C, count, gamma, beta,
                       run_mean, run_var, momentum, eps, mean, invstd, scale, shift);
}

__global__ void k_bn_eval(const float* gamma, const float* beta, const float* rm, const float* rv, int C,
                          float eps, float* mean, float* invstd, float* scale, float* shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float is = 1.f / sqrtf(rv[c] + eps);
    mean[c] = rm[c];
    invstd[c] = is;
    scale[c] = gamma[c] * is;
    shift[c] = beta[c] - rm[c] * gamma[c] * is;
}
void bn_eval_coeffs(const float* gamma, const float* beta, const float* run_mean, const float* run_var,
                    int C, float eps, float* mean, float* invstd, float* scale, float* shift, hipStream_t st) {
    hipLaunchKernelGGL(k_bn_eval, dim3(cdiv(C, 64)), dim3(64), 0, st, gamma, beta, run_mean, run_var, C, eps,
                       mean, invstd, scale, shift);
}

// split-twin store of 4 channels [c, c+4) of row r (gemm_ps.hpp layout; c % 4 == 0): NP x 8 B
template <int NP>
__device__ __forceinline__ void split4_store(char* os, int64_t ldos, int oscoff, int64_t r, int c, float4 v) {
    const auto sp = split_np<NP>(v);
    const int cc = oscoff + c;
    char* d = os + r * ldos * 2 * NP + (int64_t)(cc >> 3) * 16 * NP + (cc & 7) * 2;
#pragma unroll
    for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(d + p * 16) = sp.p[p];
}

// BN passes in row-slice form: a thread owns one 4-channel group (its per-channel coefficients stay
// in registers) and walks the rows of its slice; a wavefront still reads whole contiguous row
// chunks.  (A flat grid-stride loop reloads every coefficient per element — 7 arrays in the
// backward — and ran issue-bound below the HBM rate.)
struct RowGrid {
    int CX, RY, S;
    int64_t rps;
};
inline RowGrid row_grid(int64_t M, int C) {
    RowGrid g;
    const int C4 = C >> 2;
    g.CX = std::min(C4, 64);
    g.RY = std::max(1, 256 / g.CX);
    g.S = (int)std::max<int64_t>(1, std::min<int64_t>(65535, cdiv(M, (int64_t)g.RY * 16)));
    g.rps = (M + g.S - 1) / g.S;
    return g;
}
// QX: also the MX-fp8 copy of the twin's (bf16-rounded) values for the next fp8 contraction (q / qs,
// ldq bytes per row): what k_mx8_quantize would write from the twin, without re-reading it
template <int NP, bool YB, bool QX = false>
__global__ __launch_bounds__(256) void k_bn_relu_fwd_rows(const float* __restrict__ y, int C,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, float* __restrict__ out,
                                                          int64_t ldo, int ocoff, int64_t M, int64_t rps,
                                                          char* __restrict__ os, int64_t ldos, int oscoff,
                                                          uint8_t* __restrict__ q = nullptr, uint8_t* __restrict__ qs = nullptr,
                                                          int64_t ldq = 0) {
    const int c4 = blockIdx.x * blockDim.x + threadIdx.x;
    if (c4 >= (C >> 2)) return;
    const int c = c4 * 4;
    const float4 s = *reinterpret_cast<const float4*>(scale + c);
    const float4 t = *reinterpret_cast<const float4*>(shift + c);
    const int64_t r1 = min(M, (int64_t)(blockIdx.y + 1) * rps);
    const int RY = blockDim.y;
    // four rows per pass of the loop, their loads issued together (memory-level parallelism)
    for (int64_t rb = (int64_t)blockIdx.y * rps + threadIdx.y; rb < r1; rb += 4 * RY) {
      float4 vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
          if (rb + u * RY < r1) vb[u] = load4<YB>(y, (rb + u * RY) * C + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t r = rb + u * RY;
        if (r >= r1) break;
        const float4 v = vb[u];
        float4 o;
        o.x = bn_relu1(v.x, s.x, t.x);
        o.y = bn_relu1(v.y, s.y, t.y);
        o.z = bn_relu1(v.z, s.z, t.z);
        o.w = bn_relu1(v.w, s.w, t.w);
        if (out) *reinterpret_cast<float4*>(out + r * ldo + ocoff + c) = o;
        if constexpr (NP > 0) split4_store<NP>(os, ldos, oscoff, r, c, o);
        if constexpr (QX) {
            const uint2 t = split_np<1>(o).p[0];   // the twin's values
            mx8_store_group(make_float4(__uint_as_float(t.x << 16), __uint_as_float(t.x & 0xFFFF0000u),
                                        __uint_as_float(t.y << 16), __uint_as_float(t.y & 0xFFFF0000u)),
                            q, qs, ldq, r, c);
        }
      }
    }
}
void bn_relu_fwd(const float* y, int C, const float* scale, const float* shift, float* out, int64_t ldo,
                 int ocoff, int64_t M, hipStream_t st, void* os, int64_t ldos, int oscoff, bool y_bf16, const Mx8* qx) {
    const int np = os ? split_planes() : 0;
    char* o = static_cast<char*>(os);
    const RowGrid g = row_grid(M, C);
    CAD_NO_ALIAS("bn_relu_fwd", {aview(out, M, ldo, ocoff, C, 4, "out"), aview(os, M, ldos, oscoff, C, 2, "out twin")},
                 {aview(y, M, C, 0, C, y_bf16 ? 2 : 4, "y")}, true);
    if (qx) {
        if (np != 1 || C % 32 || qx->ld % 128 || qx->coff || !qx->q || !qx->s)
            throw std::runtime_error("bn_relu_fwd: MX-fp8 copy layout");
        auto* q = static_cast<uint8_t*>(const_cast<void*>(qx->q));
        auto* qs = static_cast<uint8_t*>(const_cast<void*>(qx->s));
        auto goq = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(cdiv(C >> 2, g.CX), g.S), dim3(g.CX, g.RY), 0, st, y, C, scale, shift, out, ldo,
                               ocoff, M, g.rps, o, ldos, oscoff, q, qs, qx->ld);
        };
        y_bf16 ? goq(k_bn_relu_fwd_rows<1, true, true>) : goq(k_bn_relu_fwd_rows<1, false, true>);
        return;
    }
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(cdiv(C >> 2, g.CX), g.S), dim3(g.CX, g.RY), 0, st, y, C, scale, shift, out, ldo,
                           ocoff, M, g.rps, o, ldos, oscoff, nullptr, nullptr, 0);
    };
    if (np == 1) y_bf16 ? go(k_bn_relu_fwd_rows<1, true>) : go(k_bn_relu_fwd_rows<1, false>);
    else y_bf16 ? go(k_bn_relu_fwd_rows<0, true>) : go(k_bn_relu_fwd_rows<0, false>);
}

// ------------------------------------------------------------------------------------------
// BatchNorm + ReLU backward
// ------------------------------------------------------------------------------------------
__global__ void k_bn_bwd_coef(const double* tot, int C, int64_t M, const float* gamma, const float* invstd,
                              float* coef, float* dgamma, float* dbeta) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double sdz = tot[c], sdzx = tot[C + c];
    dgamma[c] = (float)sdzx;
    dbeta[c] = (float)sdz;
    const float k1 = gamma[c] * invstd[c];
    coef[c] = k1;
    coef[C + c] = (float)(k1 * sdz / (double)M);
    coef[2 * C + c] = (float)(k1 * sdzx / (double)M);
}
template <int NP, bool YB, bool HG, bool GB = false, bool PA = false>
__global__ __launch_bounds__(256) void k_bn_relu_bwd_rows(const float* __restrict__ g, int64_t ldg, int gcoff,
                                                          const float* __restrict__ y, int C,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ coef, float* __restrict__ dy,
                                                          int64_t M, int64_t rps, const float* __restrict__ gmul,
                                                          int64_t HW, char* __restrict__ os, bool relu, HeadGrad hg,
                                                          PoolAdd pa, FastDiv dHW) {
    const int c4 = blockIdx.x * blockDim.x + threadIdx.x;
    if (c4 >= (C >> 2)) return;
    const int c0 = c4 * 4;
    float sc[4], sh[4], mu[4], is[4], k0[4], k1[4], k2[4], hw[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        sc[e] = scale[c0 + e]; sh[e] = shift[c0 + e]; mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
        k0[e] = coef[c0 + e]; k1[e] = coef[C + c0 + e]; k2[e] = coef[2 * C + c0 + e];
        hw[e] = HG ? hg.w[c0 + e] : 0.f;
    }
    const int64_t r0 = (int64_t)blockIdx.y * rps, r1 = min(M, r0 + rps);
    // FiLM gamma: loaded once when the block's rows lie in one sample (uniform test), else per row
    float4 gm = make_float4(1.f, 1.f, 1.f, 1.f);
    bool gm_row = false;
    if (gmul && r0 < r1) {
        const uint32_t s0 = fdiv(dHW, (uint32_t)r0), s1 = fdiv(dHW, (uint32_t)(r1 - 1));
        gm_row = s0 != s1;
        if (!gm_row) gm = *reinterpret_cast<const float4*>(gmul + (int64_t)s0 * C + c0);
    }
    const int RY = blockDim.y;
    // U rows per pass of the loop: their g / y loads issued together (one row per iteration left the
    // pass latency-bound, 0.90 of wave-cycles parked; round 6: -6 % on the plain form, +18 % on the
    // head-gradient form, which loads y only); rows keep their per-thread order
    constexpr int U = HG ? 1 : 4;
    for (int64_t rb = r0 + threadIdx.y; rb < r1; rb += U * RY) {
      float4 gb[U], yb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = rb + u * RY;
        if (r >= r1) break;
        if constexpr (!HG && !PA) gb[u] = load4<GB>(g, r * ldg + gcoff + c0);
        yb[u] = load4<YB>(y, r * C + c0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = rb + u * RY;
        if (r >= r1) break;
        float4 gv;
        if constexpr (HG) {
            const float s = hg.sig[r];
            const float dp = hg.dpred[r] * hg.md * ((1.f - s) * s);
            gv = make_float4(dp * hw[0], dp * hw[1], dp * hw[2], dp * hw[3]);
        } else {
            if constexpr (PA) gv = pool_add(pa, C, r, c0, load4<GB>(g, r * ldg + gcoff + c0));
            else gv = gb[u];
            if (gmul) {
                const float4 m = gm_row ? *reinterpret_cast<const float4*>(gmul + (int64_t)fdiv(dHW, (uint32_t)r) * C + c0)
                                        : gm;
                gv.x *= m.x; gv.y *= m.y; gv.z *= m.z; gv.w *= m.w;
            }
        }
        const float4 yv = yb[u];
        const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, ya[4] = {yv.x, yv.y, yv.z, yv.w};
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float z = __fmaf_rn(ya[e], sc[e], sh[e]);
            const float dz = (!relu || z > 0.f) ? ga[e] : 0.f;
            const float xh = (ya[e] - mu[e]) * is[e];
            o[e] = __fsub_rn(__fmaf_rn(k0[e], dz, -k1[e]), __fmul_rn(k2[e], xh));
        }
        const float4 ov = make_float4(o[0], o[1], o[2], o[3]);
        if (dy) *reinterpret_cast<float4*>(dy + r * C + c0) = ov;
        if constexpr (NP > 0) split4_store<NP>(os, C, 0, r, c0, ov);
      }
    }
}
// k_bn_relu_bwd_rows<NP, YB, false, GB, true> walked over pooled pixels (OpBnBwdPoolQ's order): the
// same per-element arithmetic and outputs
template <int NP, bool YB, bool GB>
__global__ __launch_bounds__(256) void k_bn_relu_bwd_poolq(const float* __restrict__ g, int64_t ldg, int gcoff,
                                                           const float* __restrict__ y, int C,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ coef, float* __restrict__ dy,
                                                           int64_t Mo, int64_t rps, char* __restrict__ os, PoolAdd pa) {
    const int c4 = blockIdx.x * blockDim.x + threadIdx.x;
    if (c4 >= (C >> 2)) return;
    const int c0 = c4 * 4;
    float sc[4], sh[4], mu[4], is[4], k0[4], k1[4], k2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        sc[e] = scale[c0 + e]; sh[e] = shift[c0 + e]; mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
        k0[e] = coef[c0 + e]; k1[e] = coef[C + c0 + e]; k2[e] = coef[2 * C + c0 + e];
    }
    const int64_t o1 = min(Mo, (int64_t)(blockIdx.y + 1) * rps);
    for (int64_t op = (int64_t)blockIdx.y * rps + threadIdx.y; op < o1; op += blockDim.y) {
        const int64_t p00 = pool_window(pa, (uint32_t)op);
        const uchar4 a = *reinterpret_cast<const uchar4*>(pa.idx + op * C + c0);
        const float4 d = *reinterpret_cast<const float4*>(pa.d + op * C + c0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t r = p00 + (q >> 1) * pa.W + (q & 1);
            const float4 gv = pool_add_k(a, d, q, load4<GB>(g, r * ldg + gcoff + c0));
            const float4 yv = load4<YB>(y, r * C + c0);
            const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, ya[4] = {yv.x, yv.y, yv.z, yv.w};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float z = __fmaf_rn(ya[e], sc[e], sh[e]);
                const float dz = z > 0.f ? ga[e] : 0.f;
                const float xh = (ya[e] - mu[e]) * is[e];
                o[e] = __fsub_rn(__fmaf_rn(k0[e], dz, -k1[e]), __fmul_rn(k2[e], xh));
            }
            const float4 ov = make_float4(o[0], o[1], o[2], o[3]);
            if (dy) *reinterpret_cast<float4*>(dy + r * C + c0) = ov;
            if constexpr (NP > 0) split4_store<NP>(os, C, 0, r, c0, ov);
        }
    }
}
// FiLM sums from OpBnBwdFilm's sample-aligned slices: dgam[b][c] = sum over sample b's k slices
__global__ void k_film_from_parts(const double* __restrict__ part, int k, int C, int B, float* __restrict__ dgam,
                                  float* __restrict__ dbet) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * C) return;
    const int b = i / C, c = i - b * C;
    double g = 0.0, be = 0.0;
    for (int s = b * k; s < (b + 1) * k; ++s) {
        const double* p = part + (int64_t)s * 4 * C;
        g += p[2 * C + c];
        be += p[3 * C + c];
    }
    dgam[i] = (float)g;
    dbet[i] = (float)be;
}
void bn_relu_bwd(const float* g, int64_t ldg, int gcoff, const float* y, int C, const float* mean,
                 const float* invstd, const float* scale, const float* shift, const float* gamma,
                 int64_t M, double* scratch, float* coef, float* dgamma, float* dbeta, float* dy,
                 hipStream_t st, const float* gmul, int64_t HW, void* dy_split, bool relu, bool y_bf16,
                 const HeadGrad* head, bool g_bf16, const PoolAdd* pool, float* film_dgam, float* film_dbet,
                 const double* tile_part, int tiles) {
    double* tot = scratch;
    double* part = scratch + 2 * C;
    if (tile_part && (film_dgam || tiles <= 0)) throw std::runtime_error("bn_relu_bwd: tile partials");
    // the reduction pass reads g and y, then the apply pass rewrites each element it reads: dy may be
    // exactly g (in place), but no other overlap
    CAD_NO_ALIAS("bn_relu_bwd", {aview(dy, M, C, 0, C, 4, "dy"), aview(dy_split, M, C, 0, C, 2, "dy twin")},
                 {aview(head || pool ? nullptr : g, M, ldg, gcoff, C, g_bf16 ? 2 : 4, "g"),
                  aview(y, M, C, 0, C, y_bf16 ? 2 : 4, "y")}, true);
    if (gmul && (M >= ((int64_t)1 << 32) || HW < 1)) throw std::runtime_error("bn_relu_bwd: FiLM gradient layout");
    const FastDiv dHW = make_fastdiv(gmul ? (uint32_t)HW : 2u);
    if (film_dgam) {
        // a FiLM block's bn1: the BN sums and the FiLM affine's per-(sample, channel) sums in one pass,
        // k slices per sample (rows per slice dividing HW; >= 256 rows, <= 2048 slices in all)
        if (!gmul || !g || head || pool || !relu || M % HW) throw std::runtime_error("bn_relu_bwd: FiLM sums layout");
        const int B = (int)(M / HW);
        int k = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)64, HW / 256, (int64_t)(2048 / std::max(B, 1))}));
        while (HW % k) --k;
        const int S = B * k;
        part = scratch + 4 * C;
        if (y_bf16 && g_bf16)
            launch_colreduce_slices<4>(OpBnBwdFilm<true, true>{g, y, mean, invstd, scale, shift, gmul, ldg, gcoff, C, HW, dHW},
                                       M, C, S, HW / k, part, st);
        else if (y_bf16)
            launch_colreduce_slices<4>(OpBnBwdFilm<true, false>{g, y, mean, invstd, scale, shift, gmul, ldg, gcoff, C, HW, dHW},
                                       M, C, S, HW / k, part, st);
        else if (g_bf16)
            launch_colreduce_slices<4>(OpBnBwdFilm<false, true>{g, y, mean, invstd, scale, shift, gmul, ldg, gcoff, C, HW, dHW},
                                       M, C, S, HW / k, part, st);
        else
            launch_colreduce_slices<4>(OpBnBwdFilm<false, false>{g, y, mean, invstd, scale, shift, gmul, ldg, gcoff, C, HW, dHW},
                                       M, C, S, HW / k, part, st);
        launch_colfinal(part, S, 4 * C, tot, nullptr, 1.f, st);   // tot[0, 2C): the BN sums
        hipLaunchKernelGGL(k_film_from_parts, dim3(cdiv((int64_t)B * C, 256)), dim3(256), 0, st, part, k, C, B,
                           film_dgam, film_dbet);
    }
    const HeadGrad hg = head ? *head : HeadGrad{};
    PoolAdd pa = pool ? *pool : PoolAdd{};
    if (head && (g || gmul || g_bf16 || pool)) throw std::runtime_error("bn_relu_bwd: head gradient with an explicit gradient");
    if (pool && (M >= ((int64_t)1 << 32) || pa.H <= 0 || pa.W <= 0 || ((pa.H | pa.W) & 1) ||
                 M % ((int64_t)pa.H * pa.W) != 0))
        throw std::runtime_error("bn_relu_bwd: folded max-pool backward layout");
    if (pool) {
        pa.divW = make_fastdiv((uint32_t)pa.W);
        pa.divH = make_fastdiv((uint32_t)pa.H);
    }
    // the folded max-pool backward walked over pooled pixels (OpBnBwdPoolQ / k_bn_relu_bwd_poolq);
    // CAD_POOLQ=0 keeps the per-row walk (A/B)
    static const bool poolq_on = [] {
        const char* e = std::getenv("CAD_POOLQ");
        return !(e && e[0] == '0');
    }();
    const bool quad = pool && poolq_on && !gmul && relu && !tile_part;
    PoolAdd paq = pa;
    if (quad) {
        paq.divW = make_fastdiv((uint32_t)pa.W / 2);
        paq.divH = make_fastdiv((uint32_t)pa.H / 2);
    }
    // g source: 0 fp32, 1 head, 2 bf16, 3 fp32 + folded max-pool backward, 4 bf16 + folded max-pool backward
    const int gm = head ? 1 : (g_bf16 && pool) ? 4 : g_bf16 ? 2 : pool ? 3 : 0;
    using T = std::true_type;
    using F = std::false_type;
    auto with_mode = [&](auto fn) {
        switch (gm) {
            case 1: return fn(T{}, F{}, F{});
            case 2: return fn(F{}, T{}, F{});
            case 3: return fn(F{}, F{}, T{});
            case 4: return fn(F{}, T{}, T{});
            default: return fn(F{}, F{}, F{});
        }
    };
    if (tile_part) {   // tiles -> slices of about one tile row per thread (as bn_fwd_finalize) -> tot
        const int C2 = 2 * C, CX = std::min(C2 >> 2, 64), RY = std::max(1, 256 / CX);
        const int S = (int)std::max<int64_t>(1, std::min<int64_t>(colsum_slices(M), cdiv(tiles, RY)));
        launch_colreduce_slices<1>(OpSumD{tile_part, C2}, tiles, C2, S, cdiv(tiles, S), part, st);
        launch_colfinal(part, S, C2, tot, nullptr, 1.f, st);
    }
    const int S = (film_dgam || tile_part) ? 0 : quad ? (
        y_bf16 ? (g_bf16 ? launch_colreduce<2>(OpBnBwdPoolQ<true, true>{g, y, mean, invstd, scale, shift, ldg, gcoff, C, paq}, M / 4, C, part, st)
                         : launch_colreduce<2>(OpBnBwdPoolQ<true, false>{g, y, mean, invstd, scale, shift, ldg, gcoff, C, paq}, M / 4, C, part, st))
               : (g_bf16 ? launch_colreduce<2>(OpBnBwdPoolQ<false, true>{g, y, mean, invstd, scale, shift, ldg, gcoff, C, paq}, M / 4, C, part, st)
                         : launch_colreduce<2>(OpBnBwdPoolQ<false, false>{g, y, mean, invstd, scale, shift, ldg, gcoff, C, paq}, M / 4, C, part, st)))
        : with_mode([&](auto hgc, auto gbc, auto pac) {
        constexpr bool HG = decltype(hgc)::value, GB = decltype(gbc)::value, PA = decltype(pac)::value;
        return y_bf16 ? launch_colreduce<2>(OpBnBwd<true, HG, GB, PA>{g, y, mean, invstd, scale, shift, gmul, ldg, gcoff, C,
                                                                     HW, relu, hg, pa, dHW},
                                            M, C, part, st)
                      : launch_colreduce<2>(OpBnBwd<false, HG, GB, PA>{g, y, mean, invstd, scale, shift, gmul, ldg, gcoff,
                                                                      C, HW, relu, hg, pa, dHW},
                                            M, C, part, st);
    });
    if (!film_dgam && !tile_part) launch_colfinal(part, S, 2 * C, tot, nullptr, 1.f, st);
    hipLaunchKernelGGL(k_bn_bwd_coef, dim3(cdiv(C, 64)), dim3(64), 0, st, tot, C, M, gamma, invstd, coef, dgamma, dbeta);
    const int np = dy_split ? split_planes() : 0;
    char* os = static_cast<char*>(dy_split);
    if (quad) {
        const RowGrid rq = row_grid(M / 4, C);
        auto goq = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(cdiv(C >> 2, rq.CX), rq.S), dim3(rq.CX, rq.RY), 0, st, g, ldg, gcoff, y, C, mean,
                               invstd, scale, shift, coef, dy, M / 4, rq.rps, os, paq);
        };
        if (np == 1) {
            if (y_bf16) g_bf16 ? goq(k_bn_relu_bwd_poolq<1, true, true>) : goq(k_bn_relu_bwd_poolq<1, true, false>);
            else g_bf16 ? goq(k_bn_relu_bwd_poolq<1, false, true>) : goq(k_bn_relu_bwd_poolq<1, false, false>);
        } else {
            if (y_bf16) g_bf16 ? goq(k_bn_relu_bwd_poolq<0, true, true>) : goq(k_bn_relu_bwd_poolq<0, true, false>);
            else g_bf16 ? goq(k_bn_relu_bwd_poolq<0, false, true>) : goq(k_bn_relu_bwd_poolq<0, false, false>);
        }
        return;
    }
    const RowGrid rg = row_grid(M, C);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(cdiv(C >> 2, rg.CX), rg.S), dim3(rg.CX, rg.RY), 0, st, g, ldg, gcoff, y, C, mean,
                           invstd, scale, shift, coef, dy, M, rg.rps, gmul, HW, os, relu, hg, pa, dHW);
    };
    with_mode([&](auto hgc, auto gbc, auto pac) {
        constexpr bool HG = decltype(hgc)::value, GB = decltype(gbc)::value, PA = decltype(pac)::value;
        if (np == 1) y_bf16 ? go(k_bn_relu_bwd_rows<1, true, HG, GB, PA>) : go(k_bn_relu_bwd_rows<1, false, HG, GB, PA>);
        else y_bf16 ? go(k_bn_relu_bwd_rows<0, true, HG, GB, PA>) : go(k_bn_relu_bwd_rows<0, false, HG, GB, PA>);
        return 0;
    });
}

// ------------------------------------------------------------------------------------------
// MaxPool2d(2) (baseline_unet.h:55 / :62), argmax kept as uint8 in scan order 0..3
// ------------------------------------------------------------------------------------------
// XB: x holds bf16 values (the bf16 engine pools the encoder outputs' twin: bf16 rounding is
// monotone, so the pooled twin equals the one of the fp32 maximum; ties of the rounded values go to
// the first in scan order)
template <int NP, bool XB = false>
__global__ void k_maxpool_fwd(const float* __restrict__ x, int64_t ldx, int C, int B, int H, int W,
                              float* __restrict__ out, uint8_t* __restrict__ idx, int64_t n4, char* __restrict__ os) {
    const uint32_t C4 = (uint32_t)C >> 2, Ho = (uint32_t)H >> 1, Wo = (uint32_t)W >> 1;   // n4 < 2^31 (host)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)n4; i += gridDim.x * blockDim.x) {
        const uint32_t op = i / C4;
        const int c = (int)(i - op * C4) * 4;
        const int xo = (int)(op % Wo);
        const uint32_t t = op / Wo;
        const int yo = (int)(t % Ho);
        const int b = (int)(t / Ho);
        const int64_t p00 = ((int64_t)b * H + 2 * yo) * W + 2 * xo;
        const int64_t pp[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
        float best[4];
        uint8_t arg[4] = {0, 0, 0, 0};
        {
            const float4 v = load4<XB>(x, pp[0] * ldx + c);
            best[0] = v.x; best[1] = v.y; best[2] = v.z; best[3] = v.w;
        }
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            const float4 v = load4<XB>(x, pp[k] * ldx + c);
            const float va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (va[e] > best[e] || isnan(va[e])) { best[e] = va[e]; arg[e] = (uint8_t)k; }
        }
        const float4 o = make_float4(best[0], best[1], best[2], best[3]);
        if (out) *reinterpret_cast<float4*>(out + (int64_t)op * C + c) = o;   // nullptr: only the twin is read
        if constexpr (NP > 0) split4_store<NP>(os, C, 0, op, c, o);
        *reinterpret_cast<uchar4*>(idx + (int64_t)op * C + c) = make_uchar4(arg[0], arg[1], arg[2], arg[3]);
    }
}
// An encoder block's bn2 + ReLU and the MaxPool2d(2) of the level below in one pass (round 5): one
// thread per (pooled pixel, 4-channel group) applies the BN affine + ReLU to the four pixels of its
// window (k_bn_relu_fwd_rows' arithmetic), writes them — the fp32 skip half (`out`) and/or its bf16
// twin (NP = 1) — and pools the values the separate max-pool would have read back: the twin's bf16
// values on the bf16 engine (NP = 1: k_maxpool_fwd<1, true>), the fp32 ones otherwise,
// with its comparison (first in scan order wins ties, NaN propagates).  Saves re-reading the skip half.
template <int NP, bool YB>
__global__ __launch_bounds__(256) void k_bn_relu_pool_fwd(const float* __restrict__ y, int C,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, float* __restrict__ out,
                                                         int64_t ldo, char* __restrict__ os, int64_t ldos, int H,
                                                         int W, float* __restrict__ pout, uint8_t* __restrict__ idx,
                                                         char* __restrict__ pos, int64_t n4) {
    const uint32_t C4 = (uint32_t)C >> 2, Ho = (uint32_t)H >> 1, Wo = (uint32_t)W >> 1;   // n4 < 2^31 (host)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)n4; i += gridDim.x * blockDim.x) {
        const uint32_t op = i / C4;
        const int c = (int)(i - op * C4) * 4;
        const uint32_t xo = op % Wo, t = op / Wo;
        const uint32_t yo = t % Ho, b = t / Ho;
        const int64_t p00 = ((int64_t)b * H + 2 * yo) * W + 2 * xo;
        const float4 s = *reinterpret_cast<const float4*>(scale + c);
        const float4 sh = *reinterpret_cast<const float4*>(shift + c);
        float best[4];
        uint8_t arg[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t p = p00 + (k >> 1) * W + (k & 1);
            const float4 v = load4<YB>(y, p * C + c);
            float4 o;
            o.x = bn_relu1(v.x, s.x, sh.x);
            o.y = bn_relu1(v.y, s.y, sh.y);
            o.z = bn_relu1(v.z, s.z, sh.z);
            o.w = bn_relu1(v.w, s.w, sh.w);
            if (out) *reinterpret_cast<float4*>(out + p * ldo + c) = o;
            float va[4] = {o.x, o.y, o.z, o.w};
            if constexpr (NP == 1) {   // the twin, and the values the bf16 engine's max-pool reads from it
                const auto sp = split_np<1>(o);
                *reinterpret_cast<uint2*>(os + (p * ldos + c) * 2) = sp.p[0];
                va[0] = __uint_as_float(sp.p[0].x << 16);
                va[1] = __uint_as_float(sp.p[0].x & 0xffff0000u);
                va[2] = __uint_as_float(sp.p[0].y << 16);
                va[3] = __uint_as_float(sp.p[0].y & 0xffff0000u);
            }
            if (k == 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) best[e] = va[e];
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (va[e] > best[e] || isnan(va[e])) { best[e] = va[e]; arg[e] = (uint8_t)k; }
            }
        }
        const float4 o = make_float4(best[0], best[1], best[2], best[3]);
        if (pout) *reinterpret_cast<float4*>(pout + (int64_t)op * C + c) = o;
        if constexpr (NP == 1) {
            if (pos) split4_store<1>(pos, C, 0, op, c, o);
        }
        *reinterpret_cast<uchar4*>(idx + (int64_t)op * C + c) = make_uchar4(arg[0], arg[1], arg[2], arg[3]);
    }
}
void bn_relu_pool_fwd(const float* y, int C, const float* scale, const float* shift, float* out, int64_t ldo,
                      void* os, int64_t ldos, int B, int H, int W, bool y_bf16, float* pool, uint8_t* idx,
                      void* pool_split, hipStream_t st) {
    const int64_t n4 = (int64_t)B * (H / 2) * (W / 2) * C / 4;
    if (n4 >= ((int64_t)1 << 31)) throw std::runtime_error("bn_relu_pool_fwd: tensor too large for 32-bit indexing");
    if (H % 2 || W % 2 || C % 4 || !idx || (!out && !os)) throw std::runtime_error("bn_relu_pool_fwd: bad arguments");
    const int np = os ? split_planes() : 0;
    if (np != 0 && np != 1) throw std::runtime_error("bn_relu_pool_fwd: 1-plane twins only");
    if (pool_split && np != 1) throw std::runtime_error("bn_relu_pool_fwd: a pooled twin needs the block's twin");
    char* o = static_cast<char*>(os);
    char* po = static_cast<char*>(pool_split);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(ew_blocks(n4)), dim3(256), 0, st, y, C, scale, shift, out, ldo, o, ldos, H, W, pool,
                           idx, po, n4);
    };
    if (np == 1) y_bf16 ? go(k_bn_relu_pool_fwd<1, true>) : go(k_bn_relu_pool_fwd<1, false>);
    else y_bf16 ? go(k_bn_relu_pool_fwd<0, true>) : go(k_bn_relu_pool_fwd<0, false>);
}

void maxpool_fwd(const float* x, int64_t ldx, int C, int B, int H, int W, float* out, uint8_t* idx,
                 hipStream_t st, void* out_split, bool x_bf16) {
    const int64_t n4 = (int64_t)B * (H / 2) * (W / 2) * C / 4;
    if (n4 >= ((int64_t)1 << 31)) throw std::runtime_error("maxpool_fwd: tensor too large for 32-bit indexing");
    const int np = out_split ? split_planes() : 0;
    char* os = static_cast<char*>(out_split);
    if (x_bf16 && np != 1) throw std::runtime_error("maxpool_fwd: bf16 input needs the twin output");
    if (x_bf16)
        hipLaunchKernelGGL((k_maxpool_fwd<1, true>), dim3(ew_blocks(n4)), dim3(256), 0, st, x, ldx, C, B, H, W, out, idx,
                           n4, os);
    else if (np == 1)
        hipLaunchKernelGGL(k_maxpool_fwd<1>, dim3(ew_blocks(n4)), dim3(256), 0, st, x, ldx, C, B, H, W, out, idx, n4, os);
    else
        hipLaunchKernelGGL(k_maxpool_fwd<0>, dim3(ew_blocks(n4)), dim3(256), 0, st, x, ldx, C, B, H, W, out, idx, n4, os);
}
// gather form: one thread per (INPUT pixel, 4 channels) inside the pooled region, coalesced float4
// read-modify-write of dx; adds dout[parent] where this pixel is the recorded argmax
// one thread per pooled (pixel, 4-channel group): reads its argmax codes and gradient once and adds
// the gradient into the one input position each channel chose (every input element is owned by
// exactly one pooled element: no races, and the same single add per element as a gather).  32-bit
// index arithmetic (the host checks the range).
__global__ void k_maxpool_bwd_scatter(const float* __restrict__ dout, const uint8_t* __restrict__ idx, int C,
                                      int H, int W, float* __restrict__ dx, int64_t lddx, uint32_t n4) {
    const uint32_t C4 = (uint32_t)C >> 2, Ho = (uint32_t)H >> 1, Wo = (uint32_t)W >> 1;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
        const uint32_t op = i / C4;
        const int c = (int)(i - op * C4) * 4;
        const uint32_t xo = op % Wo, t = op / Wo;
        const uint32_t yo = t % Ho, b = t / Ho;
        const uchar4 a = *reinterpret_cast<const uchar4*>(idx + (int64_t)op * C + c);
        const float4 d = *reinterpret_cast<const float4*>(dout + (int64_t)op * C + c);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (a.x != k && a.y != k && a.z != k && a.w != k) continue;
            const int64_t px = ((int64_t)b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
            float* q = dx + px * lddx + c;
            float4 v = *reinterpret_cast<float4*>(q);
            if (a.x == k) v.x += d.x;
            if (a.y == k) v.y += d.y;
            if (a.z == k) v.z += d.z;
            if (a.w == k) v.w += d.w;
            *reinterpret_cast<float4*>(q) = v;
        }
    }
}
void maxpool_bwd(const float* dout, const uint8_t* idx, int C, int B, int H, int W, float* dx,
                 int64_t lddx, hipStream_t st) {
    const int64_t n4 = (int64_t)B * (H / 2) * (W / 2) * C / 4;
    if (n4 >= ((int64_t)1 << 31)) throw std::runtime_error("maxpool_bwd: tensor too large for 32-bit indexing");
    hipLaunchKernelGGL(k_maxpool_bwd_scatter, dim3(ew_blocks(n4)), dim3(256), 0, st, dout, idx, C, H, W, dx, lddx,
                       (uint32_t)n4);
}

// ------------------------------------------------------------------------------------------
// layout, head, repacks
// ------------------------------------------------------------------------------------------
__global__ void k_rgb_to_nhwc4(const float* __restrict__ rgb, float* __restrict__ out, int64_t HW, int64_t n) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = p / HW, yx = p - b * HW;
        const float* s = rgb + b * 3 * HW + yx;
        *reinterpret_cast<float4*>(out + p * 4) = make_float4(s[0], s[HW], s[2 * HW], 0.f);
    }
}
void rgb_to_nhwc4(const float* rgb, float* out, int B, int H, int W, hipStream_t st) {
    const int64_t n = (int64_t)B * H * W;
    hipLaunchKernelGGL(k_rgb_to_nhwc4, dim3(ew_blocks(n)), dim3(256), 0, st, rgb, out, (int64_t)H * W, n);
}
// NHWC8 (rgb + 5 zero channels): the row width of the pre-split (bf16 twin) conv loaders, 16-B pieces
__global__ void k_rgb_to_nhwc8(const float* __restrict__ rgb, float* __restrict__ out, int64_t HW, int64_t n) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = p / HW, yx = p - b * HW;
        const float* s = rgb + b * 3 * HW + yx;
        float4* o = reinterpret_cast<float4*>(out + p * 8);
        o[0] = make_float4(s[0], s[HW], s[2 * HW], 0.f);
        o[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
void rgb_to_nhwc8(const float* rgb, float* out, int B, int H, int W, hipStream_t st) {
    const int64_t n = (int64_t)B * H * W;
    hipLaunchKernelGGL(k_rgb_to_nhwc8, dim3(ew_blocks(n)), dim3(256), 0, st, rgb, out, (int64_t)H * W, n);
}

__global__ void k_head_fwd(const float* __restrict__ a, int C, const float* __restrict__ w,
                           const float* __restrict__ b, float md, float* __restrict__ sig,
                           float* __restrict__ pred, int64_t M) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < M; p += (int64_t)gridDim.x * blockDim.x) {
        const float* row = a + p * C;
        float z = 0.f;
        for (int c = 0; c < C; c += 4) {
            float4 v = *reinterpret_cast<const float4*>(row + c);
            z = __fadd_rn(z, head_dot4(v, make_float4(w[c], w[c + 1], w[c + 2], w[c + 3])));
        }
        z += b[0];
        const float s = 1.f / (1.f + expf(-z));
        sig[p] = s;
        pred[p] = s * md;
    }
}
// coalesced form: TPP = C/4 lanes share one pixel row (one float4 each), shuffle-reduced
template <int TPP>
__global__ __launch_bounds__(256) void k_head_fwd_coop(const float* __restrict__ a, int C, const float* __restrict__ w,
                                                       const float* __restrict__ b, float md, float* __restrict__ sig,
                                                       float* __restrict__ pred, int64_t M) {
    const int sub = threadIdx.x % TPP;
    const float4 wv = *reinterpret_cast<const float4*>(w + sub * 4);
    for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / TPP; p < M;
         p += (int64_t)gridDim.x * blockDim.x / TPP) {
        float4 v = *reinterpret_cast<const float4*>(a + p * C + sub * 4);
        float z = head_dot4(v, wv);
#pragma unroll
        for (int o = TPP / 2; o > 0; o >>= 1) z = __fadd_rn(z, __shfl_xor(z, o));
        if (sub == 0) {
            z += b[0];
            const float s = 1.f / (1.f + expf(-z));
            sig[p] = s;
            pred[p] = s * md;
        }
    }
}
void head_fwd(const float* a, int C, const float* w, const float* b, float max_depth, float* sig,
              float* pred, int64_t M, hipStream_t st) {
    const int blocks = std::max(1, std::min(8192, cdiv(M * (C / 4), 256)));
    switch (C / 4) {
        case 16: hipLaunchKernelGGL(k_head_fwd_coop<16>, dim3(blocks), dim3(256), 0, st, a, C, w, b, max_depth, sig, pred, M); return;
        case 32: hipLaunchKernelGGL(k_head_fwd_coop<32>, dim3(blocks), dim3(256), 0, st, a, C, w, b, max_depth, sig, pred, M); return;
        case 8: hipLaunchKernelGGL(k_head_fwd_coop<8>, dim3(blocks), dim3(256), 0, st, a, C, w, b, max_depth, sig, pred, M); return;
        case 4: hipLaunchKernelGGL(k_head_fwd_coop<4>, dim3(blocks), dim3(256), 0, st, a, C, w, b, max_depth, sig, pred, M); return;
        default:
            hipLaunchKernelGGL(k_head_fwd, dim3(ew_blocks(M)), dim3(256), 0, st, a, C, w, b, max_depth, sig, pred, M);
    }
}

__global__ void k_head_da(const float* __restrict__ w, int C, const float* __restrict__ dpred,
                          const float* __restrict__ sig, float md, float* __restrict__ da, int64_t n4) {
    const int C4 = C >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / C4;
        const int c = (int)(i - r * C4) * 4;
        const float s = sig[r];
        const float dp = dpred[r] * md * ((1.f - s) * s);
        *reinterpret_cast<float4*>(da + i * 4) = make_float4(dp * w[c], dp * w[c + 1], dp * w[c + 2], dp * w[c + 3]);
    }
}
void head_bwd(const float* a, int C, const float* w, const float* dpred, const float* sig,
              float max_depth, float* da, int64_t M, double* scratch, float* dw, float* db,
              hipStream_t st) {
    const int64_t n4 = M * C / 4;
    hipLaunchKernelGGL(k_head_da, dim3(ew_blocks(n4)), dim3(256), 0, st, w, C, dpred, sig, max_depth, da, n4);
    double* part = scratch + 2 * C;
    const int S = launch_colreduce<2>(OpHeadBwd{a, dpred, sig, max_depth, C}, M, C, part, st);
    // part[s][0][c] -> dw ; part[s][1][0] -> db
    launch_colfinal(part, S, 2 * C, scratch, nullptr, 1.f, st);
    hipLaunchKernelGGL(k_colfinal, dim3(cdiv(C, 64)), dim3(64, kFinalLanes), 0, st, scratch, 1, C, nullptr, dw, 1.f);
    hipLaunchKernelGGL(k_colfinal, dim3(1), dim3(64, kFinalLanes), 0, st, scratch + C, 1, 1, nullptr, db, 1.f);
}

// Level-0 fusion (decoder level 0's bn2 + ReLU + the depth head in one pass): the block's activation
// a = relu(y * scale + shift) only feeds the head, so it is reduced in registers and never stored.
// The row-slice grid puts a row's C/4 channel groups on adjacent lanes; they are reduced with the
// same xor butterfly as k_head_fwd_coop (for C/4 <= 2 that equals k_head_fwd's sequential sum), so
// sig / pred are bit-identical to bn_relu_fwd + head_fwd.
bool head_fusable(int C) {
    const int c4 = C / 4;
    return C % 4 == 0 && c4 >= 1 && c4 <= 32 && (c4 & (c4 - 1)) == 0;
}
template <bool YB, int TPP>
__global__ __launch_bounds__(256) void k_bn_relu_head_fwd_rows(const float* __restrict__ y, const float* __restrict__ scale,
                                                               const float* __restrict__ shift, const float* __restrict__ w,
                                                               const float* __restrict__ b, float md, float* __restrict__ sig,
                                                               float* __restrict__ pred, int64_t M, int64_t rps) {
    constexpr int C = 4 * TPP;
    const int c = threadIdx.x * 4;   // blockDim.x == TPP
    const float4 s = *reinterpret_cast<const float4*>(scale + c);
    const float4 t = *reinterpret_cast<const float4*>(shift + c);
    const float4 wv = *reinterpret_cast<const float4*>(w + c);
    const float bias = b[0];
    const int64_t r1 = min(M, (int64_t)(blockIdx.y + 1) * rps);
    for (int64_t r = (int64_t)blockIdx.y * rps + threadIdx.y; r < r1; r += blockDim.y) {
        const float4 v = load4<YB>(y, r * C + c);
        float4 a;
        a.x = bn_relu1(v.x, s.x, t.x);
        a.y = bn_relu1(v.y, s.y, t.y);
        a.z = bn_relu1(v.z, s.z, t.z);
        a.w = bn_relu1(v.w, s.w, t.w);
        float z = head_dot4(a, wv);
#pragma unroll
        for (int o = TPP / 2; o > 0; o >>= 1) z = __fadd_rn(z, __shfl_xor(z, o));
        if (threadIdx.x == 0) {
            z += bias;
            const float sg = 1.f / (1.f + expf(-z));
            sig[r] = sg;
            pred[r] = sg * md;
        }
    }
}
void bn_relu_head_fwd(const float* y, int C, const float* scale, const float* shift, const float* w, const float* b,
                      float max_depth, float* sig, float* pred, int64_t M, hipStream_t st, bool y_bf16) {
    if (!head_fusable(C)) throw std::runtime_error("bn_relu_head_fwd: C / 4 must be a power of two <= 32");
    const RowGrid g = row_grid(M, C);   // CX = C / 4: one row's channel groups on adjacent lanes
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(1, g.S), dim3(g.CX, g.RY), 0, st, y, scale, shift, w, b, max_depth, sig, pred, M,
                           g.rps);
    };
    auto pick = [&](auto yb) {
        constexpr bool YB = decltype(yb)::value;
        switch (C / 4) {
            case 1: go(k_bn_relu_head_fwd_rows<YB, 1>); break;
            case 2: go(k_bn_relu_head_fwd_rows<YB, 2>); break;
            case 4: go(k_bn_relu_head_fwd_rows<YB, 4>); break;
            case 8: go(k_bn_relu_head_fwd_rows<YB, 8>); break;
            case 16: go(k_bn_relu_head_fwd_rows<YB, 16>); break;
            default: go(k_bn_relu_head_fwd_rows<YB, 32>); break;
        }
    };
    y_bf16 ? pick(std::true_type{}) : pick(std::false_type{});
}
void head_bwd_y(const float* y, int C, const float* scale, const float* shift, const float* dpred, const float* sig,
                float max_depth, int64_t M, double* scratch, float* dw, float* db, hipStream_t st, bool y_bf16) {
    double* part = scratch + 2 * C;
    const int S = y_bf16 ? launch_colreduce<2>(OpHeadBwdY<true>{y, scale, shift, dpred, sig, max_depth, C}, M, C, part, st)
                         : launch_colreduce<2>(OpHeadBwdY<false>{y, scale, shift, dpred, sig, max_depth, C}, M, C, part, st);
    launch_colfinal(part, S, 2 * C, scratch, nullptr, 1.f, st);
    hipLaunchKernelGGL(k_colfinal, dim3(cdiv(C, 64)), dim3(64, kFinalLanes), 0, st, scratch, 1, C, nullptr, dw, 1.f);
    hipLaunchKernelGGL(k_colfinal, dim3(1), dim3(64, kFinalLanes), 0, st, scratch + C, 1, 1, nullptr, db, 1.f);
}

// computeDepthMetrics (tensorboard_trainer_enhanced.h:400-439): mask gt > 0
__global__ __launch_bounds__(256) void k_metrics(const float* __restrict__ pred, const float* __restrict__ gt,
                                                 int64_t HW, double* part, int nb) {
    const int b = blockIdx.y;
    double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < HW; i += (int64_t)nb * 256) {
        const float p = pred[b * HW + i], g = gt[b * HW + i];
        if (!(g > 0.f)) continue;
        const float ad = fabsf(p - g);
        const float ld = fabsf(logf(p + 1e-8f) - logf(g + 1e-8f));
        const float r = fmaxf(p / g, g / p);
        v[0] += 1.0; v[1] += ad / g; v[2] += (ad * ad) / g; v[3] += ad * ad; v[4] += ld * ld;
        v[5] += r < 1.25f; v[6] += r < 1.5625f; v[7] += r < 1.953125f;
    }
    __shared__ double red[4][8];
    for (int q = 0; q < 8; ++q) {
        double x = v[q];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][q] = x;
    }
    __syncthreads();
    if (threadIdx.x < 8)
        part[((int64_t)b * nb + blockIdx.x) * 8 + threadIdx.x] =
            red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}
int metrics_blocks(int64_t HW) { return std::max(1, std::min(64, cdiv(HW, 256))); }
void depth_metrics_partials(const float* pred, const float* gt, int B, int64_t HW, double* part, int nb,
                            hipStream_t st) {
    hipLaunchKernelGGL(k_metrics, dim3(nb, B), dim3(256), 0, st, pred, gt, HW, part, nb);
}

// conv3x3 dgrad weights: wd[ci][t][co] = w[co][8-t][ci]
__global__ void k_repack_conv_dgrad(const float* __restrict__ w, float* __restrict__ wd, int cout, int cin) {
    const int64_t n = (int64_t)cout * 9 * cin;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int co = (int)(i % cout);
        const int64_t t2 = i / cout;
        const int t = (int)(t2 % 9);
        const int ci = (int)(t2 / 9);
        wd[i] = w[((int64_t)co * 9 + (8 - t)) * cin + ci];
    }
}
void repack_conv_dgrad(const float* w, float* wd, int cout, int cin, hipStream_t st) {
    hipLaunchKernelGGL(k_repack_conv_dgrad, dim3(ew_blocks((int64_t)cout * 9 * cin)), dim3(256), 0, st, w, wd, cout, cin);
}
// convT forward weights: wf[q][co][ci] = wm[ci][q][co]
__global__ void k_repack_convT_fwd(const float* __restrict__ wm, float* __restrict__ wf, int cin, int cout) {
    const int64_t n = (int64_t)4 * cout * cin;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int ci = (int)(i % cin);
        const int64_t qc = i / cin;   // q*cout + co
        wf[i] = wm[(int64_t)ci * 4 * cout + qc];
    }
}
void repack_convT_fwd(const float* wm, float* wf, int cin, int cout, hipStream_t st) {
    hipLaunchKernelGGL(k_repack_convT_fwd, dim3(ew_blocks((int64_t)4 * cout * cin)), dim3(256), 0, st, wm, wf, cin, cout);
}

// one thread per 8 consecutive outputs; blocks are dealt to jobs in order (block-uniform job lookup)
__global__ __launch_bounds__(256) void k_weight_prep(WPrepList list) {
    int j = 0;
    while (j + 1 < list.njobs && (int)blockIdx.x >= list.job[j + 1].blk0) ++j;
    const WPrepJob& jb = list.job[j];
    const int64_t i = ((int64_t)(blockIdx.x - jb.blk0) * 256 + threadIdx.x) * 8;
    if (i >= jb.n) return;
    const int ne = (int)min<int64_t>(8, jb.n - i);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int64_t k = i + (e < ne ? e : 0);
        int64_t src;
        if (jb.kind == WPREP_SPLIT) {
            src = k;
        } else if (jb.kind == WPREP_DGRAD) {   // k = (ci*9 + t)*cout + co  <-  w[co][8 - t][ci]
            const int co = (int)(k % jb.cout);
            const int64_t t2 = k / jb.cout;
            const int t = (int)(t2 % 9), ci = (int)(t2 / 9);
            src = ((int64_t)co * 9 + (8 - t)) * jb.cin + ci;
        } else if (jb.kind == WPREP_CONVT) {   // k = qc*cin + ci  <-  wm[ci][qc]
            const int ci = (int)(k % jb.cin);
            src = (int64_t)ci * 4 * jb.cout + k / jb.cin;
        } else {   // WPREP_TRANSPOSE: k = kk*cout + co  <-  w[co][kk]
            const int co = (int)(k % jb.cout);
            src = (int64_t)co * jb.cin + k / jb.cout;
        }
        v[e] = jb.src[src];
    }
    if (jb.d32) {
        if (ne == 8) {
            *reinterpret_cast<float4*>(jb.d32 + i) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4*>(jb.d32 + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
        } else {
            for (int e = 0; e < ne; ++e) jb.d32[i + e] = v[e];
        }
    }
    if (jb.d16) {   // n % 8 == 0 (weight_prep)
        const auto sa = split_np<1>(make_float4(v[0], v[1], v[2], v[3]));
        const auto sb = split_np<1>(make_float4(v[4], v[5], v[6], v[7]));
        *reinterpret_cast<uint4*>(static_cast<char*>(jb.d16) + i * 2) = make_uint4(sa.p[0].x, sa.p[0].y, sb.p[0].x, sb.p[0].y);
    }
}
void weight_prep(WPrepList& list, hipStream_t st) {
    if (list.njobs <= 0) return;
    if (list.njobs > kWPrepMaxJobs) throw std::runtime_error("weight_prep: too many jobs");
    int blocks = 0;
    for (int j = 0; j < list.njobs; ++j) {
        WPrepJob& jb = list.job[j];
        if (jb.d16 && jb.n % 8) throw std::runtime_error("weight_prep: bf16 twin size not a multiple of 8");
        jb.blk0 = blocks;
        blocks += (int)cdiv(cdiv(jb.n, 8), (int64_t)256);
    }
    hipLaunchKernelGGL(k_weight_prep, dim3(blocks), dim3(256), 0, st, list);
}

}  // namespace cad
