// Camera conditioning of the config-3 models.
//
//   a14 normalizeCameraIntrinsics (intrinsics_unet.h:252-268): [fx/W, fy/H, 2cx/W - 1, 2cy/H - 1]
//   a15 (no reference code): cam4 = [K00, K11, K02, K12]
//   a16 FiLMLayerImpl::forward (film_layer.h:82-108):
//         h1 = relu(BN1d(fc1(c))) [128], h2 = relu(BN1d(fc2(h1))) [256]  (BN1d only when B > 1)
//         gamma = fc_gamma(h2), beta = fc_beta(h2) [C];   out = gamma * F + beta  (per sample, channel)
//   a17 FiLMDoubleConv: conv1 -> BN -> ReLU -> FiLM -> conv2 -> BN -> ReLU (intrinsics_unet.h:38-52)
//   a19 RayEnhancedConv enc1: cat(rgb, rays) -> the same block (geometry_aware_network.h:47-64)
//
// The FiLM MLP is a few hundred kFLOP per sample: each piece is a small deterministic kernel
// (no atomics; batch statistics reduced in a fixed order, fp64).  The per-pixel affine is a
// memory-bound elementwise pass; its backward reduces Σ dA·r and Σ dA per (sample, channel) with
// the same two-level slice scheme as the BN reductions.
#include <algorithm>

#include "gemm_s3.hpp"   // split_np (the bf16 twin of the modulated activations)
#include "ew_load.hpp"
#include "kernels.hpp"

namespace cad {
namespace {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline int ew_blocks(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(n, 256)), 8192); }
constexpr int H1 = kFilmH1, H2 = kFilmH2;
}  // namespace

// ------------------------------------------------------------------------------------------
// a15 + a14
// ------------------------------------------------------------------------------------------
__global__ void k_cam_from_K(const float* __restrict__ K, int B, float* __restrict__ cam4) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float* k = K + b * 9;
    cam4[b * 4 + 0] = k[0];
    cam4[b * 4 + 1] = k[4];
    cam4[b * 4 + 2] = k[2];
    cam4[b * 4 + 3] = k[5];
}
void camera_from_K(const float* K, int B, float* cam4, hipStream_t st) {
    hipLaunchKernelGGL(k_cam_from_K, dim3(cdiv(B, 64)), dim3(64), 0, st, K, B, cam4);
}

__global__ void k_cam_normalize(const float* __restrict__ cam4, int B, int H, int W, float* __restrict__ camn) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float w = (float)W, h = (float)H;
    camn[b * 4 + 0] = cam4[b * 4 + 0] / w;
    camn[b * 4 + 1] = cam4[b * 4 + 1] / h;
    camn[b * 4 + 2] = (cam4[b * 4 + 2] / w) * 2.0f - 1.0f;
    camn[b * 4 + 3] = (cam4[b * 4 + 3] / h) * 2.0f - 1.0f;
}
void camera_normalize(const float* cam4, int B, int H, int W, float* camn, hipStream_t st) {
    hipLaunchKernelGGL(k_cam_normalize, dim3(cdiv(B, 64)), dim3(64), 0, st, cam4, B, H, W, camn);
}

// ------------------------------------------------------------------------------------------
// a19 input: NHWC8 [r, g, b, ray_x, ray_y, ray_z, 0, 0], rays computed in place from cam4 (a18
// formula of ray_direction_computer.cpp:47-55), so the (B,3,H,W) ray tensor is never materialised.
// ------------------------------------------------------------------------------------------
__global__ void k_rgb_rays_to_nhwc8(const float* __restrict__ rgb, const float* __restrict__ cam4, int H, int W,
                                    float* __restrict__ out, int64_t n) {
    const int64_t HW = (int64_t)H * W;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = p / HW, yx = p - b * HW;
        const int u = (int)(yx % W), v = (int)(yx / W);
        const float* c = cam4 + b * 4;
        const float fx_inv = 1.0f / c[0], fy_inv = 1.0f / c[1];
        const float x = ((float)u - c[2]) * fx_inv;
        const float y = ((float)v - c[3]) * fy_inv;
        const float z = 1.0f;
        // (x*x + y*y) + 1 with one rounding per operation, as the fp32 reference evaluates it (no FMA
        // contraction: a contracted norm moves a ray by an fp32 ulp, which flips its bf16 rounding)
        const float nrm = sqrtf(__fadd_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)), z));
        const float* s = rgb + b * 3 * HW + yx;
        float4* o = reinterpret_cast<float4*>(out + p * 8);
        o[0] = make_float4(s[0], s[HW], s[2 * HW], x / nrm);
        o[1] = make_float4(y / nrm, z / nrm, 0.f, 0.f);
    }
}
void rgb_rays_to_nhwc8(const float* rgb, const float* cam4, int B, int H, int W, float* out, hipStream_t st) {
    const int64_t n = (int64_t)B * H * W;
    hipLaunchKernelGGL(k_rgb_rays_to_nhwc8, dim3(ew_blocks(n)), dim3(256), 0, st, rgb, cam4, H, W, out, n);
}

// ------------------------------------------------------------------------------------------
// a16 FiLM MLP forward
// ------------------------------------------------------------------------------------------
// one BatchNorm1d(+ReLU) feature column j over the batch, z[b] given in `zx` (overwritten by xhat)
__device__ void bn1d_relu_col(float* zx, float* h, int ldz, int j, int B, bool bn, bool train, const float* g,
                              const float* be, float* rm, float* rv, float* is_out) {
    if (!bn) {   // film_layer.h:85,91: BatchNorm1d skipped when the batch has one sample
        for (int b = 0; b < B; ++b) {
            const float z = zx[b * ldz + j];
            zx[b * ldz + j] = z;
            h[b * ldz + j] = fmaxf(z, 0.f);
        }
        is_out[j] = 1.f;
        return;
    }
    float mean, is;
    if (train) {
        double s = 0.0, s2 = 0.0;
#pragma unroll 8
        for (int b = 0; b < B; ++b) {
            const double z = zx[b * ldz + j];
            s += z;
            s2 += z * z;
        }
        const double mu = s / B;
        double var = s2 / B - mu * mu;
        if (var < 0.0) var = 0.0;
        mean = (float)mu;
        is = (float)(1.0 / sqrt(var + 1e-5));
        rm[j] = 0.9f * rm[j] + 0.1f * mean;
        rv[j] = 0.9f * rv[j] + 0.1f * (float)(var * B / (B - 1));
    } else {
        mean = rm[j];
        is = 1.f / sqrtf(rv[j] + 1e-5f);
    }
    is_out[j] = is;
#pragma unroll 8
    for (int b = 0; b < B; ++b) {
        const float xh = (zx[b * ldz + j] - mean) * is;
        zx[b * ldz + j] = xh;
        h[b * ldz + j] = fmaxf(xh * g[j] + be[j], 0.f);
    }
}

// fc1 (4 -> 128) + BN1d + ReLU: one thread per feature column, the batch in a loop
__global__ __launch_bounds__(H1) void k_film_l1_fwd(FilmLayer L, const float* __restrict__ camn, int B, int train) {
    const int j = threadIdx.x;
    for (int b = 0; b < B; ++b) {
        float z = L.b1[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) z += camn[b * 4 + k] * L.w1[j * 4 + k];
        L.xh1[b * H1 + j] = z;
    }
    bn1d_relu_col(L.xh1, L.h1, H1, j, B, B > 1, train, L.g1, L.be1, L.rm1, L.rv1, L.is1);
}

// Y[b][o] = bias[o] + sum_k X[b][k] W[o][k] (nn.Linear, W row-major [O][K]): one thread per output
// (b, o), o fastest — X[b] is a wavefront-wide broadcast, the weight rows stream through L1/L2 in
// 16-B pieces — summed bias first, then k in order (the arithmetic of the sequential form exactly).
// blockIdx.y selects one of two (W, bias, Y) sets (the gamma / beta heads in one launch).
template <int K>
__global__ __launch_bounds__(256) void k_film_linear(const float* __restrict__ X, const float* __restrict__ W0,
                                                     const float* __restrict__ b0, float* __restrict__ Y0,
                                                     const float* __restrict__ W1, const float* __restrict__ b1,
                                                     float* __restrict__ Y1, int B, int O) {
    static_assert(K % 4 == 0, "K");
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)B * O) return;
    const int b = (int)(t / O), o = (int)(t - (int64_t)b * O);
    const float* W = (blockIdx.y ? W1 : W0) + (int64_t)o * K;
    const float* x = X + (int64_t)b * K;
    float z = (blockIdx.y ? b1 : b0)[o];
#pragma unroll 8
    for (int k = 0; k < K; k += 4) {
        const float4 w = *reinterpret_cast<const float4*>(W + k);
        const float4 v = *reinterpret_cast<const float4*>(x + k);
        z += v.x * w.x;
        z += v.y * w.y;
        z += v.z * w.z;
        z += v.w * w.w;
    }
    (blockIdx.y ? Y1 : Y0)[t] = z;
}

// BN1d + ReLU over the fc2 outputs (already in xh2): one thread per feature column
__global__ __launch_bounds__(H2) void k_film_l2_bn(FilmLayer L, int B, int train) {
    bn1d_relu_col(L.xh2, L.h2, H2, threadIdx.x, B, B > 1, train, L.g2, L.be2, L.rm2, L.rv2, L.is2);
}

// the list forms: blockIdx.x (l1 / l2 BN) or blockIdx.z (the Linears) selects the layer
__global__ __launch_bounds__(H1) void k_film_l1_fwd_all(FilmList list, const float* __restrict__ camn, int B, int train) {
    const FilmLayer& L = list.l[blockIdx.x];
    const int j = threadIdx.x;
    for (int b = 0; b < B; ++b) {
        float z = L.b1[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) z += camn[b * 4 + k] * L.w1[j * 4 + k];
        L.xh1[b * H1 + j] = z;
    }
    bn1d_relu_col(L.xh1, L.h1, H1, j, B, B > 1, train, L.g1, L.be1, L.rm1, L.rv1, L.is1);
}
__global__ __launch_bounds__(H2) void k_film_l2_bn_all(FilmList list, int B, int train) {
    const FilmLayer& L = list.l[blockIdx.x];
    bn1d_relu_col(L.xh2, L.h2, H2, threadIdx.x, B, B > 1, train, L.g2, L.be2, L.rm2, L.rv2, L.is2);
}
// HEADS = false: fc2 (h1 -> xh2, O = H2); true: the gamma / beta heads (h2 -> gam, bet; O = C, blockIdx.y)
template <int K, bool HEADS>
__global__ __launch_bounds__(256) void k_film_linear_all(FilmList list, int B) {
    const FilmLayer& L = list.l[blockIdx.z];
    const int O = HEADS ? L.C : H2;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)B * O) return;
    const int b = (int)(t / O), o = (int)(t - (int64_t)b * O);
    const float* X = HEADS ? L.h2 : L.h1;
    const float* W = (HEADS ? (blockIdx.y ? L.wb : L.wg) : L.w2) + (int64_t)o * K;
    const float* x = X + (int64_t)b * K;
    float z = (HEADS ? (blockIdx.y ? L.bb : L.bg) : L.b2)[o];
#pragma unroll 8
    for (int k = 0; k < K; k += 4) {   // (k_film_linear's order)
        const float4 w = *reinterpret_cast<const float4*>(W + k);
        const float4 v = *reinterpret_cast<const float4*>(x + k);
        z += v.x * w.x;
        z += v.y * w.y;
        z += v.z * w.z;
        z += v.w * w.w;
    }
    (HEADS ? (blockIdx.y ? L.bet : L.gam) : L.xh2)[t] = z;
}
void film_mlp_fwd_all(const FilmList& list, const float* camn, int B, bool train, hipStream_t st) {
    if (list.n <= 0) return;
    if (list.n > kFilmMaxLayers) throw std::runtime_error("film_mlp_fwd_all: too many layers");
    int cmax = 0;
    for (int i = 0; i < list.n; ++i) cmax = std::max(cmax, list.l[i].C);
    hipLaunchKernelGGL(k_film_l1_fwd_all, dim3(list.n), dim3(H1), 0, st, list, camn, B, (int)train);
    hipLaunchKernelGGL((k_film_linear_all<H1, false>), dim3(cdiv((int64_t)B * H2, 256), 1, list.n), dim3(256), 0, st, list,
                       B);
    hipLaunchKernelGGL(k_film_l2_bn_all, dim3(list.n), dim3(H2), 0, st, list, B, (int)train);
    hipLaunchKernelGGL((k_film_linear_all<H2, true>), dim3(cdiv((int64_t)B * cmax, 256), 2, list.n), dim3(256), 0, st, list,
                       B);
}

void film_mlp_fwd(const FilmLayer& L, const float* camn, int B, bool train, hipStream_t st) {
    hipLaunchKernelGGL(k_film_l1_fwd, dim3(1), dim3(H1), 0, st, L, camn, B, (int)train);
    hipLaunchKernelGGL(k_film_linear<H1>, dim3(cdiv((int64_t)B * H2, 256), 1), dim3(256), 0, st, (const float*)L.h1,
                       (const float*)L.w2, (const float*)L.b2, L.xh2, (const float*)nullptr, (const float*)nullptr,
                       (float*)nullptr, B, H2);
    hipLaunchKernelGGL(k_film_l2_bn, dim3(1), dim3(H2), 0, st, L, B, (int)train);
    hipLaunchKernelGGL(k_film_linear<H2>, dim3(cdiv((int64_t)B * L.C, 256), 2), dim3(256), 0, st, (const float*)L.h2,
                       (const float*)L.wg, (const float*)L.bg, L.gam, (const float*)L.wb, (const float*)L.bb, L.bet,
                       B, L.C);
}

// ------------------------------------------------------------------------------------------
// a16/a17 affine: a1 = gamma[b,c] * relu(y1 * scale[c] + shift[c]) + beta[b,c]
// ------------------------------------------------------------------------------------------
// row-slice form (as the BN passes, nn_kernels.hip): a thread owns one 4-channel group, keeps its BN
// scale / shift in registers and re-reads gamma / beta only when its rows cross into the next sample
// os: the bf16 twin (pre-split operand of conv2 and its weight gradient, rows of C); out (fp32) may be
// null when only the twin has readers
template <bool YB, bool TW>
__global__ __launch_bounds__(256) void k_film_apply(const float* __restrict__ y, int C, const float* __restrict__ scale,
                                                    const float* __restrict__ shift, const float* __restrict__ gam,
                                                    const float* __restrict__ bet, FastDiv dHW, float* __restrict__ out,
                                                    char* __restrict__ os, int64_t M, int64_t rps) {
    const int c4 = blockIdx.x * blockDim.x + threadIdx.x;
    if (c4 >= (C >> 2)) return;
    const int c = c4 * 4;
    const float4 s = *reinterpret_cast<const float4*>(scale + c);
    const float4 t = *reinterpret_cast<const float4*>(shift + c);
    int64_t cur = -1;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f), b = g;
    const int64_t r1 = min(M, (int64_t)(blockIdx.y + 1) * rps);
    for (int64_t r = (int64_t)blockIdx.y * rps + threadIdx.y; r < r1; r += blockDim.y) {
        const int64_t smp = fdiv(dHW, (uint32_t)r);   // (r / HW: a 64-bit division per row)
        if (smp != cur) {
            cur = smp;
            g = *reinterpret_cast<const float4*>(gam + smp * C + c);
            b = *reinterpret_cast<const float4*>(bet + smp * C + c);
        }
        const float4 v = load4<YB>(y, r * C + c);
        float4 o;
        o.x = g.x * fmaxf(v.x * s.x + t.x, 0.f) + b.x;
        o.y = g.y * fmaxf(v.y * s.y + t.y, 0.f) + b.y;
        o.z = g.z * fmaxf(v.z * s.z + t.z, 0.f) + b.z;
        o.w = g.w * fmaxf(v.w * s.w + t.w, 0.f) + b.w;
        if (out) *reinterpret_cast<float4*>(out + r * C + c) = o;
        if constexpr (TW) *reinterpret_cast<uint2*>(os + (r * C + c) * 2) = split_np<1>(o).p[0];
    }
}
void film_apply(const float* y, int C, const float* scale, const float* shift, const float* gam, const float* bet,
                int B, int64_t HW, float* out, hipStream_t st, bool y_bf16, void* os) {
    const int64_t M = (int64_t)B * HW;
    if (M >= ((int64_t)1 << 32) || HW < 1) throw std::runtime_error("film_apply: layout");
    const FastDiv dHW = make_fastdiv((uint32_t)HW);
    const int C4 = C >> 2, CX = std::min(C4, 64), RY = std::max(1, 256 / CX);
    const int S = (int)std::max<int64_t>(1, std::min<int64_t>(65535, cdiv(M, (int64_t)RY * 16)));
    const int64_t rps = (M + S - 1) / S;
    char* o = static_cast<char*>(os);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(cdiv(C4, CX), S), dim3(CX, RY), 0, st, y, C, scale, shift, gam, bet, dHW, out, o,
                           M, rps);
    };
    if (os) y_bf16 ? go(k_film_apply<true, true>) : go(k_film_apply<false, true>);
    else y_bf16 ? go(k_film_apply<true, false>) : go(k_film_apply<false, false>);
}

// ------------------------------------------------------------------------------------------
// affine backward reductions: dgam[b,c] = Σ_hw dA·relu(y·sc+sh), dbet[b,c] = Σ_hw dA
// part[b][s][2][C] (double), slices of each sample's HW rows; then a fixed-order sum over s.
// ------------------------------------------------------------------------------------------
int film_reduce_slices(int64_t HW) { return (int)std::max<int64_t>(1, std::min<int64_t>(64, HW / 1024)); }

template <bool YB, bool GB = false>   // GB: dA holds bf16 values
__global__ __launch_bounds__(256) void k_film_reduce(const float* __restrict__ dA, const float* __restrict__ y,
                                                     int C, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, int64_t HW, int64_t rps,
                                                     double* __restrict__ part) {
    const int CX = blockDim.x, RY = blockDim.y;
    const int C4 = C >> 2;
    const int c4 = blockIdx.x * CX + threadIdx.x;
    const int S = gridDim.y;
    const int b = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.y * rps, r1 = min(HW, r0 + rps);
    double ag[4] = {0, 0, 0, 0}, ab[4] = {0, 0, 0, 0};
    if (c4 < C4) {
        const float4 s = *reinterpret_cast<const float4*>(scale + c4 * 4);
        const float4 t = *reinterpret_cast<const float4*>(shift + c4 * 4);
        for (int64_t r = r0 + threadIdx.y; r < r1; r += RY) {
            const int64_t off = ((int64_t)b * HW + r) * C + c4 * 4;
            const float4 d = load4<GB>(dA, off);
            const float4 v = load4<YB>(y, off);
            ag[0] += (double)d.x * fmaxf(v.x * s.x + t.x, 0.f);
            ag[1] += (double)d.y * fmaxf(v.y * s.y + t.y, 0.f);
            ag[2] += (double)d.z * fmaxf(v.z * s.z + t.z, 0.f);
            ag[3] += (double)d.w * fmaxf(v.w * s.w + t.w, 0.f);
            ab[0] += d.x; ab[1] += d.y; ab[2] += d.z; ab[3] += d.w;
        }
    }
    extern __shared__ double red[];   // [RY][CX][8]
    double* mine = red + ((int64_t)threadIdx.y * CX + threadIdx.x) * 8;
    for (int e = 0; e < 4; ++e) { mine[e] = ag[e]; mine[4 + e] = ab[e]; }
    __syncthreads();
    if (threadIdx.y == 0 && c4 < C4) {
        for (int yy = 1; yy < RY; ++yy) {
            const double* o = red + ((int64_t)yy * CX + threadIdx.x) * 8;
            for (int e = 0; e < 4; ++e) { ag[e] += o[e]; ab[e] += o[4 + e]; }
        }
        double* p = part + (((int64_t)b * S + blockIdx.y) * 2) * C + c4 * 4;
        for (int e = 0; e < 4; ++e) { p[e] = ag[e]; p[C + e] = ab[e]; }
    }
}
__global__ void k_film_reduce_final(const double* __restrict__ part, int S, int C, int B, float* __restrict__ dgam,
                                    float* __restrict__ dbet) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * C) return;
    const int b = i / C, c = i - b * C;
    double g = 0.0, be = 0.0;
    for (int s = 0; s < S; ++s) {
        const double* p = part + (((int64_t)b * S + s) * 2) * C;
        g += p[c];
        be += p[C + c];
    }
    dgam[i] = (float)g;
    dbet[i] = (float)be;
}
void film_affine_bwd(const float* dA, const float* y, int C, const float* scale, const float* shift, int B, int64_t HW,
                     double* scratch, float* dgam, float* dbet, hipStream_t st, bool y_bf16, bool dA_bf16) {
    const int C4 = C >> 2;
    const int CX = std::min(C4, 64);
    const int RY = std::max(1, 256 / CX);
    const int S = film_reduce_slices(HW);
    const int64_t rps = (HW + S - 1) / S;
    const size_t shm = (size_t)RY * CX * 8 * sizeof(double);
    if (y_bf16 && dA_bf16)
        hipLaunchKernelGGL((k_film_reduce<true, true>), dim3(cdiv(C4, CX), S, B), dim3(CX, RY), shm, st, dA, y, C, scale,
                           shift, HW, rps, scratch);
    else if (dA_bf16)
        hipLaunchKernelGGL((k_film_reduce<false, true>), dim3(cdiv(C4, CX), S, B), dim3(CX, RY), shm, st, dA, y, C, scale,
                           shift, HW, rps, scratch);
    else if (y_bf16)
        hipLaunchKernelGGL(k_film_reduce<true>, dim3(cdiv(C4, CX), S, B), dim3(CX, RY), shm, st, dA, y, C, scale, shift, HW,
                           rps, scratch);
    else
        hipLaunchKernelGGL(k_film_reduce<false>, dim3(cdiv(C4, CX), S, B), dim3(CX, RY), shm, st, dA, y, C, scale, shift,
                           HW, rps, scratch);
    hipLaunchKernelGGL(k_film_reduce_final, dim3(cdiv((int64_t)B * C, 256)), dim3(256), 0, st, scratch, S, C, B, dgam,
                       dbet);
}
int64_t film_reduce_doubles(int B, int64_t HW, int C) { return (int64_t)B * film_reduce_slices(HW) * 2 * C; }

// ------------------------------------------------------------------------------------------
// a16 FiLM MLP backward (train mode)
// ------------------------------------------------------------------------------------------
// heads: dW[o][k] = Σ_b d[b][o] h2[b][k], db[o] = Σ_b d[b][o]; column k == H2 is the bias
// dh2[b][k] = Σ_c dgam[b][c] Wg[c][k] + Σ_c dbet[b][c] Wb[c][k], summed in that order: one thread per
// (b, k), k fastest (coalesced weight rows, dgam / dbet broadcast); loads run 8 terms ahead of the
// dependent FMA chain

// BatchNorm1d(+ReLU) backward for feature column j: in: dh (grad of h = relu(n)), out: dz (grad of
// the Linear output) into dh's slot; writes the BN affine grads
__device__ void bn1d_relu_bwd_col(float* dh, const float* h, const float* xh, int ldz, int j, int B, bool bn,
                                  const float* g, const float* is, float* dg, float* dbe) {
    if (!bn) {
        for (int b = 0; b < B; ++b) dh[b * ldz + j] = h[b * ldz + j] > 0.f ? dh[b * ldz + j] : 0.f;
        dg[j] = 0.f;
        dbe[j] = 0.f;
        return;
    }
    double s = 0.0, sx = 0.0;
#pragma unroll 8
    for (int b = 0; b < B; ++b) {
        const float dn = h[b * ldz + j] > 0.f ? dh[b * ldz + j] : 0.f;
        dh[b * ldz + j] = dn;
        s += dn;
        sx += (double)dn * xh[b * ldz + j];
    }
    dg[j] = (float)sx;
    dbe[j] = (float)s;
    const float k1 = g[j] * is[j];
    const float k2 = (float)(k1 * s / B), k3 = (float)(k1 * sx / B);
#pragma unroll 8
    for (int b = 0; b < B; ++b) dh[b * ldz + j] = k1 * dh[b * ldz + j] - k2 - k3 * xh[b * ldz + j];
}

// layer 2: dh2 -> dz2 (in place) through BN1d + ReLU, fc2 bias gradient
__global__ __launch_bounds__(H2) void k_film_l2_bwd(FilmLayer L, int B) {
    const int j = threadIdx.x;
    bn1d_relu_bwd_col(L.dh2, L.h2, L.xh2, H2, j, B, B > 1, L.g2, L.is2, L.gg2, L.gbe2);
    float db = 0.f;
    for (int b = 0; b < B; ++b) db += L.dh2[b * H2 + j];
    L.gb2[j] = db;
}

// fc2 weight gradient gw2[j][k] = Σ_b dz2[b][j] h1[b][k]: one thread per weight (k fastest)

// layer 1: dh1[b][j] = Σ_jj dz2[b][jj] W2[jj][j], one thread per (b, j) (j fastest: coalesced weight
// rows, dz2 broadcast), loads 8 terms ahead of the dependent FMA chain (jj ascending)
// then BN1d + ReLU backward and the fc1 gradients per column
__global__ __launch_bounds__(H1) void k_film_l1_bwd(FilmLayer L, const float* __restrict__ camn, int B) {
    const int j = threadIdx.x;
    bn1d_relu_bwd_col(L.dh1, L.h1, L.xh1, H1, j, B, B > 1, L.g1, L.is1, L.gg1, L.gbe1);
    float db = 0.f;
    float dw[4] = {0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; ++b) {
        const float d = L.dh1[b * H1 + j];
        db += d;
#pragma unroll
        for (int k = 0; k < 4; ++k) dw[k] += d * camn[b * 4 + k];
    }
    L.gb1[j] = db;
#pragma unroll
    for (int k = 0; k < 4; ++k) L.gw1[j * 4 + k] = dw[k];
}

// two independent steps in one launch: blocks [0, nb0) run the first kernel's body, the rest the
// second's (each thread's work and order exactly the separate kernels')
template <void (*A)(const FilmLayer&, int, int), void (*Bf)(const FilmLayer&, int, int)>
__global__ __launch_bounds__(256) void k_film_pair(FilmLayer L, int B, int nb0) {
    if ((int)blockIdx.x < nb0) A(L, B, blockIdx.x * 256 + threadIdx.x);
    else Bf(L, B, ((int)blockIdx.x - nb0) * 256 + threadIdx.x);
}
__device__ void film_head_bwd_w_at(const FilmLayer& L, int B, int t) {
    const int C = L.C;
    if (t >= 2 * C * (H2 + 1)) return;
    const int o = t / (H2 + 1), k = t - o * (H2 + 1);
    const bool isg = o < C;
    const int c = isg ? o : o - C;
    const float* d = isg ? L.dgam : L.dbet;
    float acc = 0.f;
    if (k < H2)
        for (int b = 0; b < B; ++b) acc += d[b * C + c] * L.h2[b * H2 + k];
    else
        for (int b = 0; b < B; ++b) acc += d[b * C + c];
    if (k < H2) (isg ? L.gwg : L.gwb)[(int64_t)c * H2 + k] = acc;
    else (isg ? L.gbg : L.gbb)[c] = acc;
}
__device__ void film_dh2_at(const FilmLayer& L, int B, int t) {
    if (t >= B * H2) return;
    const int b = t / H2, k = t - b * H2;
    const int C = L.C;
    float acc = 0.f;
    for (int pass = 0; pass < 2; ++pass) {
        const float* d = (pass ? L.dbet : L.dgam) + (int64_t)b * C;
        const float* w = (pass ? L.wb : L.wg) + k;
        int c = 0;
        for (; c + 8 <= C; c += 8) {
            float dv[8], wv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { dv[u] = d[c + u]; wv[u] = w[(int64_t)(c + u) * H2]; }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += dv[u] * wv[u];
        }
        for (; c < C; ++c) acc += d[c] * w[(int64_t)c * H2];
    }
    L.dh2[t] = acc;
}
__device__ void film_gw2_at(const FilmLayer& L, int B, int t) {
    if (t >= H2 * H1) return;
    const int j = t / H1, k = t - j * H1;
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += L.dh2[b * H2 + j] * L.h1[b * H1 + k];
    L.gw2[t] = acc;
}
__device__ void film_dh1_at(const FilmLayer& L, int B, int t) {
    if (t >= B * H1) return;
    const int b = t / H1, j = t - b * H1;
    const float* d = L.dh2 + (int64_t)b * H2;
    const float* w = L.w2 + j;
    float acc = 0.f;
    for (int jj = 0; jj < H2; jj += 8) {
        float dv[8], wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { dv[u] = d[jj + u]; wv[u] = w[(jj + u) * H1]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += dv[u] * wv[u];
    }
    L.dh1[t] = acc;
}

// six steps in four launches: {heads' weight gradients, dh2} -> layer-2 BN backward -> {fc2 weight
// gradient, dh1} -> layer-1 BN backward and fc1 gradients
void film_mlp_bwd(const FilmLayer& L, const float* camn, int B, hipStream_t st) {
    const int nb_w = cdiv((int64_t)2 * L.C * (H2 + 1), 256), nb_dh2 = cdiv((int64_t)B * H2, 256);
    hipLaunchKernelGGL((k_film_pair<film_head_bwd_w_at, film_dh2_at>), dim3(nb_w + nb_dh2), dim3(256), 0, st, L, B, nb_w);
    hipLaunchKernelGGL(k_film_l2_bwd, dim3(1), dim3(H2), 0, st, L, B);
    const int nb_gw2 = cdiv(H2 * H1, 256), nb_dh1 = cdiv((int64_t)B * H1, 256);
    hipLaunchKernelGGL((k_film_pair<film_gw2_at, film_dh1_at>), dim3(nb_gw2 + nb_dh1), dim3(256), 0, st, L, B, nb_gw2);
    hipLaunchKernelGGL(k_film_l1_bwd, dim3(1), dim3(H1), 0, st, L, camn, B);
}

}  // namespace cad
