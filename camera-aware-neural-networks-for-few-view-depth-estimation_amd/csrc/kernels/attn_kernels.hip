// Geometry-aware family: CBAM attention and the Perspective Correction Layer.
//
//   CBAMImpl::forward (spatial_attention.h:142-191):
//     att[b,c] = σ(fc2(relu(fc1(avgpool_hw x))) + fc2(relu(fc1(maxpool_hw x))))     ChannelAttention :55-75
//     x1 = x ⊙ att;  sa[p] = σ(conv7x7([mean_c x1, max_c x1]))                      SpatialAttention :100-117
//     out = x1 ⊙ sa
//   PerspectiveCorrectionLayerImpl::forward (pcl_layer.h:76-111) + buildAffineMatrix (:148-178):
//     h = relu(loc_fc2(relu(loc_fc1([avgpool_hw u, cam])))), t = fc_transform(h) (6)
//     θ = [[t0 cos t4, −sin t4 + t5, t2], [sin t4, t1 cos t4, t3]]
//     out = grid_sample(u, affine_grid(θ, align_corners=false), bilinear, zeros, align_corners=false)
//
// Everything is NHWC fp32 ([B·H·W][C] rows).  The per-pixel passes are HBM-bound elementwise/row
// reductions (one wavefront per pixel row for the channel reductions, channels on the lanes so a row
// is one coalesced read); the per-(sample, channel) reductions over H·W use the two-level slice scheme
// of the BN reductions (fp64 partials, fixed-order final sum: deterministic).  The MLPs are a few
// kFLOP per sample: one workgroup per sample.  The only non-deterministic step is grid_sample's input
// gradient, a scatter (hardware fp32 atomics, like the reference's CUDA kernel); the reference's CPU
// path adds serially, so that gradient agrees to rounding, not bit for bit.
#include <algorithm>

#include "kernels.hpp"

namespace cad {
namespace {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline int ew_blocks(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(n, 256)), 16384); }
__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + __expf(-z)); }

// (value, index) max with the first occurrence winning ties (ATen's CPU max / adaptive_max_pool2d)
__device__ __forceinline__ void amax_merge(float& v, int64_t& i, float ov, int64_t oi) {
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}
__device__ __forceinline__ void wave_amax(float& v, int& i) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const float ov = __shfl_xor(v, m);
        const int oi = __shfl_xor(i, m);
        if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
    }
}

// at::linspace(-1, 1, n)[idx] * (n - 1) / n  (affine_grid's base coordinate, align_corners = false)
__device__ __forceinline__ float grid_base(int idx, int n) {
    if (n <= 1) return 0.f;
    const float step = 2.0f / (float)(n - 1);
    const int half = n / 2;
    const float v = idx < half ? -1.0f + step * (float)idx : 1.0f - step * (float)(n - idx - 1);
    return (v * (float)(n - 1)) / (float)n;
}
}  // namespace

int chan_pool_slices(int64_t HW) { return (int)std::max<int64_t>(1, std::min<int64_t>(64, HW / 256)); }
int64_t attn_scratch_doubles(int B, int64_t HW, int C) {
    const int S = chan_pool_slices(HW);
    return std::max<int64_t>((int64_t)B * S * 3 * C, (int64_t)256 * 98 + (int64_t)B * 64 * 8) + 64;
}

// ------------------------------------------------------------------------------------------
// input pack: NHWC8 [r g b rx ry rz 0 0] from NCHW rgb and NCHW rays (cat(rgb, rays), :47-51)
// ------------------------------------------------------------------------------------------
__global__ void k_pack_rgb_rays(const float* __restrict__ rgb, const float* __restrict__ rays, int64_t HW,
                                float* __restrict__ out, int64_t n) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = p / HW, yx = p - b * HW;
        const float* s = rgb + b * 3 * HW + yx;
        const float* r = rays + b * 3 * HW + yx;
        float4* o = reinterpret_cast<float4*>(out + p * 8);
        o[0] = make_float4(s[0], s[HW], s[2 * HW], r[0]);
        o[1] = make_float4(r[HW], r[2 * HW], 0.f, 0.f);
    }
}
void pack_rgb_rays(const float* rgb, const float* rays, int B, int H, int W, float* out, hipStream_t st) {
    const int64_t n = (int64_t)B * H * W;
    hipLaunchKernelGGL(k_pack_rgb_rays, dim3(ew_blocks(n)), dim3(256), 0, st, rgb, rays, (int64_t)H * W, out, n);
}

// ------------------------------------------------------------------------------------------
// per-(sample, channel) mean / max+argmax over H·W (AdaptiveAvgPool2d(1), AdaptiveMaxPool2d(1))
// part[b][s][3][C] = {Σ, max, argmax} of slice s; block (CX channels, RY row lanes)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_chan_pool(const float* __restrict__ x, int64_t ldx, int xcoff, int C,
                                                   int64_t HW, int64_t rps, int want_max, double* __restrict__ part) {
    const int CX = blockDim.x, RY = blockDim.y;
    const int c = blockIdx.x * CX + threadIdx.x;
    const int S = gridDim.y, s = blockIdx.y, b = blockIdx.z;
    const int64_t r0 = (int64_t)s * rps, r1 = min(HW, r0 + rps);
    double sum = 0.0;
    float mx = -INFINITY;
    int64_t mi = HW;   // "none": loses every tie against a real index
    if (c < C) {
        for (int64_t r = r0 + threadIdx.y; r < r1; r += RY) {
            const float v = x[((int64_t)b * HW + r) * ldx + xcoff + c];
            sum += v;
            if (want_max && v > mx) { mx = v; mi = r; }
        }
    }
    extern __shared__ double red[];   // [RY][CX][3]
    double* mine = red + ((int64_t)threadIdx.y * CX + threadIdx.x) * 3;
    mine[0] = sum; mine[1] = mx; mine[2] = (double)mi;
    __syncthreads();
    if (threadIdx.y == 0 && c < C) {
        for (int yy = 1; yy < RY; ++yy) {
            const double* o = red + ((int64_t)yy * CX + threadIdx.x) * 3;
            sum += o[0];
            amax_merge(mx, mi, (float)o[1], (int64_t)o[2]);
        }
        double* p = part + (((int64_t)b * S + s) * 3) * C + c;
        p[0] = sum; p[C] = mx; p[2 * C] = (double)mi;
    }
}
__global__ void k_chan_pool_final(const double* __restrict__ part, int S, int C, int B, int64_t HW,
                                  float* __restrict__ avg, float* __restrict__ mx, int* __restrict__ amax) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * C) return;
    const int b = i / C, c = i - b * C;
    double sum = 0.0;
    float m = -INFINITY;
    int64_t mi = HW;
    for (int s = 0; s < S; ++s) {
        const double* p = part + (((int64_t)b * S + s) * 3) * C + c;
        sum += p[0];
        amax_merge(m, mi, (float)p[C], (int64_t)p[2 * C]);
    }
    avg[i] = (float)(sum / (double)HW);
    if (mx) { mx[i] = m; amax[i] = (int)mi; }
}
void chan_pool(const float* x, int64_t ldx, int xcoff, int C, int B, int64_t HW, double* part, float* avg, float* mx,
               int* amax, hipStream_t st) {
    const int CX = std::min(C, 64), RY = std::max(1, 256 / CX);
    const int S = chan_pool_slices(HW);
    const int64_t rps = (HW + S - 1) / S;
    const size_t shm = (size_t)RY * CX * 3 * sizeof(double);
    hipLaunchKernelGGL(k_chan_pool, dim3(cdiv(C, CX), S, B), dim3(CX, RY), shm, st, x, ldx, xcoff, C, HW, rps,
                       (int)(mx != nullptr), part);
    hipLaunchKernelGGL(k_chan_pool_final, dim3(cdiv((int64_t)B * C, 256)), dim3(256), 0, st, part, S, C, B, HW, avg,
                       mx, amax);
}

// ------------------------------------------------------------------------------------------
// CBAM forward
// ------------------------------------------------------------------------------------------
// ChannelAttention MLP, one workgroup per sample: ha/hm = relu(fc1(avg/max)), att = σ(fc2(ha) + fc2(hm))
__global__ __launch_bounds__(256) void k_cbam_mlp_fwd(Cbam A) {
    const int b = blockIdx.x, C = A.C, Cr = A.Cr;
    const float* va = A.avg + (int64_t)b * C;
    const float* vm = A.mx + (int64_t)b * C;
    for (int j = threadIdx.x; j < 2 * Cr; j += blockDim.x) {
        const int jj = j < Cr ? j : j - Cr;
        const float* v = j < Cr ? va : vm;
        const float* w = A.w1 + (int64_t)jj * C;
        float z = 0.f;
        for (int c = 0; c < C; ++c) z += w[c] * v[c];
        z += A.b1[jj];
        (j < Cr ? A.ha : A.hm)[(int64_t)b * Cr + jj] = fmaxf(z, 0.f);
    }
    __syncthreads();
    const float* ha = A.ha + (int64_t)b * Cr;
    const float* hm = A.hm + (int64_t)b * Cr;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float* w = A.w2 + (int64_t)c * Cr;
        float oa = 0.f, om = 0.f;
        for (int j = 0; j < Cr; ++j) { oa += w[j] * ha[j]; om += w[j] * hm[j]; }
        oa += A.b2[c];
        om += A.b2[c];
        A.att[(int64_t)b * C + c] = sigm(oa + om);
    }
}

// one wavefront per pixel: s[p] = {mean_c x·att, max_c x·att}, sidx[p] = first argmax channel
__global__ __launch_bounds__(256) void k_cbam_spool(Cbam A, const float* __restrict__ x, int64_t HW, int64_t M) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= M) return;
    const int C = A.C;
    const float* xr = x + p * C;
    const float* at = A.att + (p / HW) * C;
    float sum = 0.f, mx = -INFINITY;
    int mi = INT32_MAX;
    for (int c = lane; c < C; c += 64) {
        const float v = xr[c] * at[c];
        sum += v;
        if (v > mx) { mx = v; mi = c; }
    }
    sum = wave_sum(sum);
    wave_amax(mx, mi);
    if (lane == 0) {
        A.s[p * 2 + 0] = sum / (float)C;
        A.s[p * 2 + 1] = mx;
        A.sidx[p] = mi;
    }
}

// SpatialAttention conv (2 -> 1, 7x7, pad 3, no bias) + sigmoid; one thread per pixel
__global__ void k_cbam_sconv(Cbam A, int H, int W, int64_t M) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= M) return;
    const int64_t HW = (int64_t)H * W, b = p / HW, yx = p - b * HW;
    const int y = (int)(yx / W), xx = (int)(yx - (int64_t)y * W);
    float z = 0.f;
    for (int ch = 0; ch < 2; ++ch)
        for (int ky = 0; ky < 7; ++ky) {
            const int yy = y + ky - 3;
            if (yy < 0 || yy >= H) continue;
            for (int kx = 0; kx < 7; ++kx) {
                const int xs = xx + kx - 3;
                if (xs < 0 || xs >= W) continue;
                z += A.wsp[(ch * 7 + ky) * 7 + kx] * A.s[((b * H + yy) * W + xs) * 2 + ch];
            }
        }
    A.sa[p] = sigm(z);
}

// out = (x·att)·sa
__global__ void k_cbam_out(Cbam A, const float* __restrict__ x, int64_t HW, float* __restrict__ out, int64_t ldo,
                           int ocoff, int64_t n) {
    const int C = A.C;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int c = (int)(i - p * C);
        out[p * ldo + ocoff + c] = (x[i] * A.att[(p / HW) * C + c]) * A.sa[p];
    }
}

void cbam_fwd(const Cbam& A, const float* x, int B, int H, int W, float* out, int64_t ldo, int ocoff, double* scratch,
              hipStream_t st) {
    const int64_t HW = (int64_t)H * W, M = (int64_t)B * HW;
    chan_pool(x, A.C, 0, A.C, B, HW, scratch, A.avg, A.mx, A.amax, st);
    hipLaunchKernelGGL(k_cbam_mlp_fwd, dim3(B), dim3(256), 0, st, A);
    hipLaunchKernelGGL(k_cbam_spool, dim3(cdiv(M, 4)), dim3(256), 0, st, A, x, HW, M);
    hipLaunchKernelGGL(k_cbam_sconv, dim3(cdiv(M, 256)), dim3(256), 0, st, A, H, W, M);
    hipLaunchKernelGGL(k_cbam_out, dim3(ew_blocks(M * A.C)), dim3(256), 0, st, A, x, HW, out, ldo, ocoff, M * A.C);
}

// ------------------------------------------------------------------------------------------
// CBAM backward
// ------------------------------------------------------------------------------------------
// one wavefront per pixel: dlog[p] = σ'(.)·Σ_c g·x1
__global__ __launch_bounds__(256) void k_cbam_bwd_sa(Cbam A, const float* __restrict__ x, const float* __restrict__ g,
                                                     int64_t ldg, int gcoff, int64_t HW, int64_t M) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= M) return;
    const int C = A.C;
    const float* xr = x + p * C;
    const float* gr = g + p * ldg + gcoff;
    const float* at = A.att + (p / HW) * C;
    float acc = 0.f;
    for (int c = lane; c < C; c += 64) acc += gr[c] * (xr[c] * at[c]);
    acc = wave_sum(acc);
    if (lane == 0) {
        const float s = A.sa[p];
        A.dlog[p] = acc * (1.f - s) * s;
    }
}
// spatial conv input gradient (gather over the 49 taps): ds[q][ch]
__global__ void k_cbam_sconv_bwd_in(Cbam A, int H, int W, int64_t M) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= M) return;
    const int64_t HW = (int64_t)H * W, b = q / HW, yx = q - b * HW;
    const int y = (int)(yx / W), xx = (int)(yx - (int64_t)y * W);
    float d0 = 0.f, d1 = 0.f;
    for (int ky = 0; ky < 7; ++ky) {
        const int py = y - (ky - 3);
        if (py < 0 || py >= H) continue;
        for (int kx = 0; kx < 7; ++kx) {
            const int px = xx - (kx - 3);
            if (px < 0 || px >= W) continue;
            const float dl = A.dlog[(b * H + py) * W + px];
            d0 += A.wsp[ky * 7 + kx] * dl;
            d1 += A.wsp[49 + ky * 7 + kx] * dl;
        }
    }
    A.ds[q * 2 + 0] = d0;
    A.ds[q * 2 + 1] = d1;
}
// spatial conv weight gradient: part[s][t] = Σ_{p in slice s} dlog[p]·s[p + off(t)][ch(t)]
__global__ __launch_bounds__(256) void k_cbam_sconv_wgrad(Cbam A, int H, int W, int64_t M, int64_t pps,
                                                          double* __restrict__ part) {
    const int t = blockIdx.x, ch = t / 49, ky = (t % 49) / 7, kx = t % 7;
    const int64_t HW = (int64_t)H * W;
    const int64_t p0 = (int64_t)blockIdx.y * pps, p1 = min(M, p0 + pps);
    double acc = 0.0;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const int64_t b = p / HW, yx = p - b * HW;
        const int y = (int)(yx / W) + ky - 3, xx = (int)(yx % W) + kx - 3;
        if (y < 0 || y >= H || xx < 0 || xx >= W) continue;
        acc += (double)A.dlog[p] * A.s[((b * H + y) * W + xx) * 2 + ch];
    }
    __shared__ double red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int m = 128; m >= 1; m >>= 1) {
        if ((int)threadIdx.x < m) red[threadIdx.x] += red[threadIdx.x + m];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[(int64_t)blockIdx.y * 98 + t] = red[0];
}
__global__ void k_cbam_sconv_wgrad_final(Cbam A, const double* __restrict__ part, int S) {
    const int t = threadIdx.x;
    if (t >= 98) return;
    double acc = 0.0;
    for (int s = 0; s < S; ++s) acc += part[(int64_t)s * 98 + t];
    A.gwsp[t] = (float)acc;
}
// dx1[p][c] = g·sa + ds_mean/C + [c == sidx] ds_max
__device__ __forceinline__ float cbam_dx1(const Cbam& A, const float* g, int64_t ldg, int gcoff, int64_t p, int c) {
    float d = g[p * ldg + gcoff + c] * A.sa[p] + A.ds[p * 2] / (float)A.C;
    if (A.sidx[p] == c) d += A.ds[p * 2 + 1];
    return d;
}
// datt partials: part[b][s][c] = Σ_{rows of slice s} dx1·x
__global__ __launch_bounds__(256) void k_cbam_datt(Cbam A, const float* __restrict__ x, const float* __restrict__ g,
                                                   int64_t ldg, int gcoff, int64_t HW, int64_t rps,
                                                   double* __restrict__ part) {
    const int CX = blockDim.x, RY = blockDim.y, C = A.C;
    const int c = blockIdx.x * CX + threadIdx.x;
    const int S = gridDim.y, s = blockIdx.y, b = blockIdx.z;
    const int64_t r0 = (int64_t)s * rps, r1 = min(HW, r0 + rps);
    double acc = 0.0;
    if (c < C)
        for (int64_t r = r0 + threadIdx.y; r < r1; r += RY) {
            const int64_t p = (int64_t)b * HW + r;
            acc += (double)cbam_dx1(A, g, ldg, gcoff, p, c) * x[p * C + c];
        }
    extern __shared__ double red[];   // [RY][CX]
    red[threadIdx.y * CX + threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.y == 0 && c < C) {
        for (int yy = 1; yy < RY; ++yy) acc += red[yy * CX + threadIdx.x];
        part[((int64_t)b * S + s) * C + c] = acc;
    }
}
// one workgroup per sample: datt -> dlogit (do), hidden grads, pooled-vector grads
__global__ __launch_bounds__(256) void k_cbam_mlp_bwd(Cbam A, const double* __restrict__ part, int S) {
    const int b = blockIdx.x, C = A.C, Cr = A.Cr;
    float* dO = A.dO + (int64_t)b * C;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        double acc = 0.0;
        for (int s = 0; s < S; ++s) acc += part[((int64_t)b * S + s) * C + c];
        const float a = A.att[(int64_t)b * C + c];
        dO[c] = (float)acc * (1.f - a) * a;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 2 * Cr; j += blockDim.x) {
        const int jj = j < Cr ? j : j - Cr;
        const float h = (j < Cr ? A.ha : A.hm)[(int64_t)b * Cr + jj];
        float acc = 0.f;
        for (int c = 0; c < C; ++c) acc += A.w2[(int64_t)c * Cr + jj] * dO[c];
        (j < Cr ? A.dha : A.dhm)[(int64_t)b * Cr + jj] = h > 0.f ? acc : 0.f;
    }
    __syncthreads();
    const float* dha = A.dha + (int64_t)b * Cr;
    const float* dhm = A.dhm + (int64_t)b * Cr;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float da = 0.f, dm = 0.f;
        for (int j = 0; j < Cr; ++j) {
            const float w = A.w1[(int64_t)j * C + c];
            da += w * dha[j];
            dm += w * dhm[j];
        }
        A.dva[(int64_t)b * C + c] = da;
        A.dvm[(int64_t)b * C + c] = dm;
    }
}
// shared-MLP weight gradients over the batch (both branches)
__global__ void k_cbam_mlp_wgrad(Cbam A, int B) {
    const int C = A.C, Cr = A.Cr;
    const int64_t n2 = (int64_t)C * Cr, n1 = (int64_t)Cr * C;
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n2) {   // fc2.weight [C][Cr]
        const int c = (int)(t / Cr), j = (int)(t - (int64_t)c * Cr);
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += A.dO[(int64_t)b * C + c] * A.ha[(int64_t)b * Cr + j];
        for (int b = 0; b < B; ++b) acc += A.dO[(int64_t)b * C + c] * A.hm[(int64_t)b * Cr + j];
        A.gw2[t] = acc;
        return;
    }
    t -= n2;
    if (t < C) {   // fc2.bias
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += A.dO[(int64_t)b * C + t];
        A.gb2[t] = acc + acc;
        return;
    }
    t -= C;
    if (t < n1) {   // fc1.weight [Cr][C]
        const int j = (int)(t / C), c = (int)(t - (int64_t)j * C);
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += A.dha[(int64_t)b * Cr + j] * A.avg[(int64_t)b * C + c];
        for (int b = 0; b < B; ++b) acc += A.dhm[(int64_t)b * Cr + j] * A.mx[(int64_t)b * C + c];
        A.gw1[t] = acc;
        return;
    }
    t -= n1;
    if (t < Cr) {   // fc1.bias
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += A.dha[(int64_t)b * Cr + t];
        for (int b = 0; b < B; ++b) acc += A.dhm[(int64_t)b * Cr + t];
        A.gb1[t] = acc;
    }
}
// dx = dx1·att + dva/HW + [p == argmax] dvm
__global__ void k_cbam_dx(Cbam A, const float* __restrict__ g, int64_t ldg, int gcoff, int64_t HW,
                          float* __restrict__ dx, int64_t n) {
    const int C = A.C;
    const float inv = 1.0f / (float)HW;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int c = (int)(i - p * C);
        const int64_t b = p / HW, bc = b * C + c;
        float d = cbam_dx1(A, g, ldg, gcoff, p, c) * A.att[bc] + A.dva[bc] * inv;
        if ((int64_t)A.amax[bc] == p - b * HW) d += A.dvm[bc];
        dx[i] = d;
    }
}

void cbam_bwd(const Cbam& A, const float* x, const float* g, int64_t ldg, int gcoff, int B, int H, int W, float* dx,
              double* scratch, hipStream_t st) {
    const int64_t HW = (int64_t)H * W, M = (int64_t)B * HW;
    hipLaunchKernelGGL(k_cbam_bwd_sa, dim3(cdiv(M, 4)), dim3(256), 0, st, A, x, g, ldg, gcoff, HW, M);
    hipLaunchKernelGGL(k_cbam_sconv_bwd_in, dim3(cdiv(M, 256)), dim3(256), 0, st, A, H, W, M);
    const int SW = (int)std::max<int64_t>(1, std::min<int64_t>(256, M / 4096));
    hipLaunchKernelGGL(k_cbam_sconv_wgrad, dim3(98, SW), dim3(256), 0, st, A, H, W, M, (M + SW - 1) / SW, scratch);
    hipLaunchKernelGGL(k_cbam_sconv_wgrad_final, dim3(1), dim3(128), 0, st, A, scratch, SW);
    const int C = A.C, CX = std::min(C, 64), RY = std::max(1, 256 / CX);
    const int S = chan_pool_slices(HW);
    const int64_t rps = (HW + S - 1) / S;
    hipLaunchKernelGGL(k_cbam_datt, dim3(cdiv(C, CX), S, B), dim3(CX, RY), (size_t)RY * CX * sizeof(double), st, A, x,
                       g, ldg, gcoff, HW, rps, scratch);
    hipLaunchKernelGGL(k_cbam_mlp_bwd, dim3(B), dim3(256), 0, st, A, scratch, S);
    const int64_t nw = 2 * (int64_t)C * A.Cr + C + A.Cr;
    hipLaunchKernelGGL(k_cbam_mlp_wgrad, dim3(cdiv(nw, 256)), dim3(256), 0, st, A, B);
    hipLaunchKernelGGL(k_cbam_dx, dim3(ew_blocks(M * C)), dim3(256), 0, st, A, g, ldg, gcoff, HW, dx, M * C);
}

// ------------------------------------------------------------------------------------------
// PCL forward
// ------------------------------------------------------------------------------------------
// localization MLP + affine matrix, one workgroup (128 threads) per sample
__global__ __launch_bounds__(128) void k_pcl_mlp_fwd(Pcl P, const float* __restrict__ camn) {
    const int b = blockIdx.x, C = P.C, K1 = C + 4, j = threadIdx.x;
    __shared__ float h1[kPclHidden], h2[kPclHidden];
    const float* pooled = P.pooled + (int64_t)b * C;
    {
        const float* w = P.w1 + (int64_t)j * K1;
        float z = 0.f;
        for (int k = 0; k < C; ++k) z += w[k] * pooled[k];
        for (int k = 0; k < 4; ++k) z += w[C + k] * camn[b * 4 + k];
        z += P.b1[j];
        h1[j] = fmaxf(z, 0.f);
        P.h1[b * kPclHidden + j] = h1[j];
    }
    __syncthreads();
    {
        const float* w = P.w2 + (int64_t)j * kPclHidden;
        float z = 0.f;
        for (int k = 0; k < kPclHidden; ++k) z += w[k] * h1[k];
        z += P.b2[j];
        h2[j] = fmaxf(z, 0.f);
        P.h2[b * kPclHidden + j] = h2[j];
    }
    __syncthreads();
    if (j < 6) {
        const float* w = P.w3 + j * kPclHidden;
        float z = 0.f;
        for (int k = 0; k < kPclHidden; ++k) z += w[k] * h2[k];
        P.tp[b * 6 + j] = z + P.b3[j];
    }
    __syncthreads();
    if (j == 0) {   // buildAffineMatrix (pcl_layer.h:148-178)
        const float* t = P.tp + b * 6;
        const float cr = cosf(t[4]), sr = sinf(t[4]);
        float* th = P.theta + b * 6;
        th[0] = t[0] * cr; th[1] = -sr + t[5]; th[2] = t[2];
        th[3] = sr;        th[4] = t[1] * cr;  th[5] = t[3];
    }
}

// sampling position of output pixel (i, j) of sample b, in input pixel units (unnormalised)
struct GsPos {
    float ix, iy;
};
__device__ __forceinline__ GsPos gs_pos(const float* th, int i, int j, int H, int W) {
    const float x = grid_base(j, W), y = grid_base(i, H);
    const float gx = x * th[0] + y * th[1] + th[2];
    const float gy = x * th[3] + y * th[4] + th[5];
    GsPos q;
    q.ix = (gx + 1.f) * ((float)W * 0.5f) - 0.5f;
    q.iy = (gy + 1.f) * ((float)H * 0.5f) - 0.5f;
    return q;
}

__global__ void k_grid_sample_fwd(Pcl P, const float* __restrict__ u, int H, int W, float* __restrict__ out,
                                  int64_t ldo, int ocoff, int64_t n) {
    const int C = P.C;
    const int64_t HW = (int64_t)H * W;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = e / C;
        const int c = (int)(e - p * C);
        const int64_t b = p / HW, yx = p - b * HW;
        const int i = (int)(yx / W), j = (int)(yx - (int64_t)i * W);
        const GsPos q = gs_pos(P.theta + b * 6, i, j, H, W);
        const float xw = floorf(q.ix), yn = floorf(q.iy);
        const float w = q.ix - xw, e_ = 1.f - w, nn = q.iy - yn, s = 1.f - nn;
        const int x0 = (int)xw, y0 = (int)yn;
        const float* ub = u + b * HW * C + c;
        auto at = [&](int yy, int xx) -> float {
            return (yy >= 0 && yy < H && xx >= 0 && xx < W) ? ub[((int64_t)yy * W + xx) * C] : 0.f;
        };
        const float v = at(y0, x0) * (s * e_) + at(y0, x0 + 1) * (s * w) + at(y0 + 1, x0) * (nn * e_) +
                        at(y0 + 1, x0 + 1) * (nn * w);
        out[p * ldo + ocoff + c] = v;
    }
}

void pcl_fwd(const Pcl& P, const float* u, const float* camn, int B, int H, int W, float* out, int64_t ldo, int ocoff,
             double* scratch, hipStream_t st) {
    const int64_t HW = (int64_t)H * W, n = (int64_t)B * HW * P.C;
    chan_pool(u, P.C, 0, P.C, B, HW, scratch, P.pooled, nullptr, nullptr, st);
    hipLaunchKernelGGL(k_pcl_mlp_fwd, dim3(B), dim3(kPclHidden), 0, st, P, camn);
    hipLaunchKernelGGL(k_grid_sample_fwd, dim3(ew_blocks(n)), dim3(256), 0, st, P, u, H, W, out, ldo, ocoff, n);
}

// ------------------------------------------------------------------------------------------
// PCL backward
// ------------------------------------------------------------------------------------------
// The input gradient is GATHERED: each input pixel sums, in a fixed row-major order, the bilinear
// weights of the output pixels whose sampling cell touches it, so the backward is deterministic run
// to run (a scatter with fp32 atomics is not).  Those output pixels lie in the preimage of the 2x2
// input cell under the sample's affine map: ix = a j + b i + c0, iy = d j + e i + f0 in pixel units,
// a = th0, b = th1 W/H, d = th3 H/W, e = th4.  A near-singular map (a preimage box of more than
// kGsGatherMax output pixels per input pixel) keeps the atomic scatter for that sample.
constexpr int kGsGatherMax = 1024;
struct GsFoot {
    float inv00, inv01, inv10, inv11, c0, f0;   // (j, i) = inv * ((ix, iy) - (c0, f0))
    int hj, hi;                                 // half extents of the preimage box (+2 guard)
    bool gather;
};
__device__ __forceinline__ GsFoot gs_foot(const float* th, int H, int W) {
    GsFoot f;
    const float a = th[0], bb = th[1] * (float)W / (float)H, d = th[3] * (float)H / (float)W, e = th[4];
    const float det = a * e - bb * d;
    const GsPos o = gs_pos(th, 0, 0, H, W);
    f.c0 = o.ix;
    f.f0 = o.iy;
    f.gather = false;
    f.hj = f.hi = 0;
    f.inv00 = f.inv01 = f.inv10 = f.inv11 = 0.f;
    if (!(fabsf(det) > 1e-6f)) return f;
    f.inv00 = e / det;
    f.inv01 = -bb / det;
    f.inv10 = -d / det;
    f.inv11 = a / det;
    const float ej = fabsf(f.inv00) + fabsf(f.inv01), ei = fabsf(f.inv10) + fabsf(f.inv11);
    if (!(ej < 4096.f && ei < 4096.f)) return f;
    f.hj = (int)ceilf(ej) + 2;
    f.hi = (int)ceilf(ei) + 2;
    f.gather = (int64_t)(2 * f.hj + 1) * (2 * f.hi + 1) <= kGsGatherMax;
    return f;
}

// one wavefront per input pixel of a gather-mode sample, lanes over channels
__global__ __launch_bounds__(256) void k_grid_sample_bwd_gather(Pcl P, const float* __restrict__ g, int64_t ldg,
                                                                int gcoff, int H, int W, float* __restrict__ du,
                                                                int64_t M) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= M) return;
    const int C = P.C;
    const int64_t HW = (int64_t)H * W, b = p / HW, yx = p - b * HW;
    const int yy = (int)(yx / W), xx = (int)(yx - (int64_t)yy * W);
    const float* th = P.theta + b * 6;
    const GsFoot f = gs_foot(th, H, W);
    if (!f.gather) return;
    const float rx = (float)xx - f.c0, ry = (float)yy - f.f0;
    const int cj = (int)floorf(f.inv00 * rx + f.inv01 * ry), ci = (int)floorf(f.inv10 * rx + f.inv11 * ry);
    const int j0 = max(0, cj - f.hj), j1 = min(W - 1, cj + f.hj + 1);
    const int i0 = max(0, ci - f.hi), i1 = min(H - 1, ci + f.hi + 1);
    for (int c0 = 0; c0 < C; c0 += 64) {
        const int c = c0 + lane;
        float acc = 0.f;
        for (int i = i0; i <= i1; ++i)
            for (int j = j0; j <= j1; ++j) {
                const GsPos q = gs_pos(th, i, j, H, W);
                const float xw = floorf(q.ix), yn = floorf(q.iy);
                const int x0 = (int)xw, y0 = (int)yn;
                const int dx = xx - x0, dy = yy - y0;   // 0/1: which corner of (i, j)'s cell this pixel is
                if ((unsigned)dx > 1u || (unsigned)dy > 1u) continue;
                const float w = q.ix - xw, e_ = 1.f - w, nn = q.iy - yn, s = 1.f - nn;
                const float wt = (dy ? nn : s) * (dx ? w : e_);
                if (c < C) acc += wt * g[(b * HW + (int64_t)i * W + j) * ldg + gcoff + c];
            }
        if (c < C) du[p * C + c] = acc;
    }
}

// one wavefront per output pixel: grid gradient reduced over the channels -> dgrid[p] (d gx, d gy);
// the input gradient scattered with fp32 atomics (du zeroed first) only for near-singular samples
__global__ __launch_bounds__(256) void k_grid_sample_bwd(Pcl P, const float* __restrict__ u,
                                                         const float* __restrict__ g, int64_t ldg, int gcoff, int H,
                                                         int W, float* __restrict__ du, int64_t M) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= M) return;
    const int C = P.C;
    const int64_t HW = (int64_t)H * W, b = p / HW, yx = p - b * HW;
    const int i = (int)(yx / W), j = (int)(yx - (int64_t)i * W);
    const bool scatter = !gs_foot(P.theta + b * 6, H, W).gather;
    const GsPos q = gs_pos(P.theta + b * 6, i, j, H, W);
    const float xw = floorf(q.ix), yn = floorf(q.iy);
    const float w = q.ix - xw, e_ = 1.f - w, nn = q.iy - yn, s = 1.f - nn;
    const int x0 = (int)xw, y0 = (int)yn;
    const bool in_nw = y0 >= 0 && y0 < H && x0 >= 0 && x0 < W;
    const bool in_ne = y0 >= 0 && y0 < H && x0 + 1 >= 0 && x0 + 1 < W;
    const bool in_sw = y0 + 1 >= 0 && y0 + 1 < H && x0 >= 0 && x0 < W;
    const bool in_se = y0 + 1 >= 0 && y0 + 1 < H && x0 + 1 >= 0 && x0 + 1 < W;
    const int64_t base = b * HW;
    const int64_t o_nw = (base + (int64_t)y0 * W + x0) * C, o_ne = o_nw + C;
    const int64_t o_sw = o_nw + (int64_t)W * C, o_se = o_sw + C;
    const float* gr = g + p * ldg + gcoff;
    float gx = 0.f, gy = 0.f;
    for (int c = lane; c < C; c += 64) {
        const float go = gr[c];
        const float vnw = in_nw ? u[o_nw + c] : 0.f, vne = in_ne ? u[o_ne + c] : 0.f;
        const float vsw = in_sw ? u[o_sw + c] : 0.f, vse = in_se ? u[o_se + c] : 0.f;
        gx += ((vne - vnw) * s + (vse - vsw) * nn) * go;
        gy += ((vsw - vnw) * e_ + (vse - vne) * w) * go;
        if (!scatter) continue;
        if (in_nw) unsafeAtomicAdd(du + o_nw + c, (s * e_) * go);
        if (in_ne) unsafeAtomicAdd(du + o_ne + c, (s * w) * go);
        if (in_sw) unsafeAtomicAdd(du + o_sw + c, (nn * e_) * go);
        if (in_se) unsafeAtomicAdd(du + o_se + c, (nn * w) * go);
    }
    gx = wave_sum(gx);
    gy = wave_sum(gy);
    if (lane == 0) {
        P.dgrid[p * 2 + 0] = gx * ((float)W * 0.5f);
        P.dgrid[p * 2 + 1] = gy * ((float)H * 0.5f);
    }
}
// affine_grid backward: part[b][s][6] = Σ_{pixels of slice s} dgrid[p][r]·(x, y, 1)[k]
__global__ __launch_bounds__(256) void k_pcl_dtheta(Pcl P, int H, int W, int64_t pps, double* __restrict__ part) {
    const int b = blockIdx.y, S = gridDim.x, s = blockIdx.x;
    const int64_t HW = (int64_t)H * W;
    const int64_t p0 = (int64_t)s * pps, p1 = min(HW, p0 + pps);
    double a[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t r = p0 + threadIdx.x; r < p1; r += blockDim.x) {
        const int i = (int)(r / W), j = (int)(r - (int64_t)i * W);
        const float x = grid_base(j, W), y = grid_base(i, H);
        const float* d = P.dgrid + ((int64_t)b * HW + r) * 2;
        a[0] += (double)d[0] * x; a[1] += (double)d[0] * y; a[2] += d[0];
        a[3] += (double)d[1] * x; a[4] += (double)d[1] * y; a[5] += d[1];
    }
    __shared__ double red[6][256];
    for (int k = 0; k < 6; ++k) red[k][threadIdx.x] = a[k];
    __syncthreads();
    for (int m = 128; m >= 1; m >>= 1) {
        if ((int)threadIdx.x < m)
            for (int k = 0; k < 6; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + m];
        __syncthreads();
    }
    if (threadIdx.x < 6) part[((int64_t)b * S + s) * 6 + threadIdx.x] = red[threadIdx.x][0];
}
// one workgroup per sample: dθ -> d(transform params) -> localization MLP -> d pooled
__global__ __launch_bounds__(128) void k_pcl_mlp_bwd(Pcl P, const double* __restrict__ part, int S) {
    const int b = blockIdx.x, C = P.C, K1 = C + 4, j = threadIdx.x;
    __shared__ float dtp[6], dh2[kPclHidden], dh1[kPclHidden];
    if (j == 0) {
        double d[6] = {0, 0, 0, 0, 0, 0};
        for (int s = 0; s < S; ++s)
            for (int k = 0; k < 6; ++k) d[k] += part[((int64_t)b * S + s) * 6 + k];
        const float* t = P.tp + b * 6;
        const float cr = cosf(t[4]), sr = sinf(t[4]);
        const float d00 = (float)d[0], d01 = (float)d[1], d02 = (float)d[2];
        const float d10 = (float)d[3], d11 = (float)d[4], d12 = (float)d[5];
        dtp[0] = d00 * cr;
        dtp[1] = d11 * cr;
        dtp[2] = d02;
        dtp[3] = d12;
        dtp[4] = -d00 * t[0] * sr - d01 * cr + d10 * cr - d11 * t[1] * sr;
        dtp[5] = d01;
        for (int k = 0; k < 6; ++k) P.dtp[b * 6 + k] = dtp[k];
    }
    __syncthreads();
    {
        float acc = 0.f;
        for (int i = 0; i < 6; ++i) acc += P.w3[i * kPclHidden + j] * dtp[i];
        dh2[j] = P.h2[b * kPclHidden + j] > 0.f ? acc : 0.f;
        P.dh2[b * kPclHidden + j] = dh2[j];
    }
    __syncthreads();
    {
        float acc = 0.f;
        for (int i = 0; i < kPclHidden; ++i) acc += P.w2[i * kPclHidden + j] * dh2[i];
        dh1[j] = P.h1[b * kPclHidden + j] > 0.f ? acc : 0.f;
        P.dh1[b * kPclHidden + j] = dh1[j];
    }
    __syncthreads();
    for (int c = j; c < C; c += blockDim.x) {
        float acc = 0.f;
        for (int i = 0; i < kPclHidden; ++i) acc += P.w1[(int64_t)i * K1 + c] * dh1[i];
        P.dpooled[(int64_t)b * C + c] = acc;
    }
}
// localization MLP weight gradients over the batch
__global__ void k_pcl_wgrad(Pcl P, const float* __restrict__ camn, int B) {
    const int C = P.C, K1 = C + 4, Hd = kPclHidden;
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 6 * Hd) {   // fc_transform.weight [6][128]
        const int i = (int)(t / Hd), k = (int)(t % Hd);
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += P.dtp[b * 6 + i] * P.h2[b * Hd + k];
        P.gw3[t] = acc;
        return;
    }
    t -= 6 * Hd;
    if (t < 6) {
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += P.dtp[b * 6 + t];
        P.gb3[t] = acc;
        return;
    }
    t -= 6;
    if (t < Hd * Hd) {   // loc_fc2.weight
        const int i = (int)(t / Hd), k = (int)(t % Hd);
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += P.dh2[b * Hd + i] * P.h1[b * Hd + k];
        P.gw2[t] = acc;
        return;
    }
    t -= Hd * Hd;
    if (t < Hd) {
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += P.dh2[b * Hd + t];
        P.gb2[t] = acc;
        return;
    }
    t -= Hd;
    if (t < (int64_t)Hd * K1) {   // loc_fc1.weight [128][C + 4]
        const int i = (int)(t / K1), k = (int)(t % K1);
        float acc = 0.f;
        for (int b = 0; b < B; ++b)
            acc += P.dh1[b * Hd + i] * (k < C ? P.pooled[(int64_t)b * C + k] : camn[b * 4 + (k - C)]);
        P.gw1[t] = acc;
        return;
    }
    t -= (int64_t)Hd * K1;
    if (t < Hd) {
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += P.dh1[b * Hd + t];
        P.gb1[t] = acc;
    }
}
// du[p][c] += dpooled[b][c] / HW   (adaptive_avg_pool2d backward)
__global__ void k_pcl_pool_bwd(Pcl P, int64_t HW, float* __restrict__ du, int64_t n) {
    const int C = P.C;
    const float inv = 1.0f / (float)HW;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int c = (int)(i - p * C);
        du[i] += P.dpooled[(p / HW) * C + c] * inv;
    }
}

void pcl_bwd(const Pcl& P, const float* u, const float* camn, const float* g, int64_t ldg, int gcoff, int B, int H,
             int W, float* du, double* scratch, hipStream_t st) {
    const int64_t HW = (int64_t)H * W, M = (int64_t)B * HW, n = M * P.C;
    (void)hipMemsetAsync(du, 0, sizeof(float) * n, st);
    hipLaunchKernelGGL(k_grid_sample_bwd, dim3(cdiv(M, 4)), dim3(256), 0, st, P, u, g, ldg, gcoff, H, W, du, M);
    hipLaunchKernelGGL(k_grid_sample_bwd_gather, dim3(cdiv(M, 4)), dim3(256), 0, st, P, g, ldg, gcoff, H, W, du, M);
    const int S = (int)std::max<int64_t>(1, std::min<int64_t>(64, HW / 2048));
    hipLaunchKernelGGL(k_pcl_dtheta, dim3(S, B), dim3(256), 0, st, P, H, W, (HW + S - 1) / S, scratch);
    hipLaunchKernelGGL(k_pcl_mlp_bwd, dim3(B), dim3(kPclHidden), 0, st, P, scratch, S);
    const int64_t nw = 6 * kPclHidden + 6 + kPclHidden * kPclHidden + kPclHidden + (int64_t)kPclHidden * (P.C + 4) +
                       kPclHidden;
    hipLaunchKernelGGL(k_pcl_wgrad, dim3(cdiv(nw, 256)), dim3(256), 0, st, P, camn, B);
    hipLaunchKernelGGL(k_pcl_pool_bwd, dim3(ew_blocks(n)), dim3(256), 0, st, P, HW, du, n);
}

}  // namespace cad
