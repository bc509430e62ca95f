// Fused depth-loss forward + analytic backward.
// Replaces CombinedDepthLoss::forwardWithIntrinsics (src/loss/depth_loss.h:416-433) and its autograd
// backward with 7 small kernels: wavefront/LDS reductions into fixed-order fp64 partials (no
// atomics, bitwise-reproducible), one pooled pyramid, one elementwise dL/dpred pass.
//
// Semantics reproduced (file:line in /root/reference/src/loss/depth_loss.h):
//   SI      :33-64   mask gt>eps (global over batch) or the caller's valid_mask; d = log(clamp p) - log(clamp g);
//                    L = sum d^2/n - lam (sum d)^2/n^2; n == 0 -> 0 and no gradient.
//   grad    :95-166  4 scales, avg_pool2d(k=2^s) then log(clamp), forward differences, L1 means,
//                    mask IGNORED (invalid gt contributes log(1e-6)), /num_scales.
//   smooth  :189-234 per-sample mean normalisation, |dI| averaged over the 3 channels, exp(-|dI|).
//   reproj  :268-331 integer pixel grid, eps added to fx/fy and inside the sqrt, mean over the same mask.
// clamp(x, eps, 1000) passes gradient where eps <= x <= 1000; |x|' = sgn(x) with sgn(0) = 0.
#include <algorithm>

#include "kernels.hpp"

namespace cad {
namespace {
constexpr float kEps = 1e-6f;
constexpr float kLam = 0.5f;
constexpr int kScales = 4;
constexpr int kTPB = 256;
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ float clampf(float x) { return fminf(fmaxf(x, kEps), 1000.f); }
__device__ __forceinline__ float clampgrad(float x) { return (x >= kEps && x <= 1000.f) ? 1.f : 0.f; }
__device__ __forceinline__ float sgnf(float x) { return (float)((x > 0.f) - (x < 0.f)); }

// block-wide sum of NV doubles, result valid in thread 0
template <int NV>
__device__ void block_sum(double (&v)[NV], double* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        double x = v[i];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        v[i] = x;
    }
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) red[wv * NV + i] = v[i];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            double s = 0.0;
            for (int w = 0; w < kTPB / 64; ++w) s += red[w * NV + i];
            v[i] = s;
        }
}

struct Geo {
    int B, H, W;
    int Hs[kScales], Ws[kScales];
    int64_t off[kScales];   // pyramid offsets (scale s >= 1) in floats, per array
    int64_t pyr_n;          // floats per pyramid array
};

// scalar slots (double) in dsc
enum { S_N = 0, S_SD, S_SD2, S_SE, S_GX0, S_GY0 = S_GX0 + kScales, S_SMX = S_GY0 + kScales, S_SMY,
       S_PB /* B per-sample sum(pred) */ };
// per-sample tail after S_PB: [B] sum pred, [B] S_b (sum gn*p)

// pass A: SI + reproj sums (global) and per-sample sum(pred)
__global__ __launch_bounds__(kTPB) void k_passA(const float* __restrict__ pred, const float* __restrict__ gt,
                                                const float* __restrict__ K, const uint8_t* __restrict__ mask, Geo g,
                                                double* partA, int nb) {
    __shared__ double red[4 * 5];
    const int b = blockIdx.y;
    const int64_t HW = (int64_t)g.H * g.W;
    const float* kk = K + b * 9;
    const float fx = kk[0], cx = kk[2], fy = kk[4], cy = kk[5];
    double v[5] = {0, 0, 0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < HW; i += (int64_t)nb * kTPB) {
        const float p = pred[b * HW + i], t = gt[b * HW + i];
        v[4] += p;
        if (mask ? mask[b * HW + i] != 0 : t > kEps) {
            const float d = logf(clampf(p)) - logf(clampf(t));
            v[0] += 1.0;
            v[1] += d;
            v[2] += (double)d * d;
            const int u = (int)(i % g.W), vv = (int)(i / g.W);
            const float gu = (float)u - cx, gv = (float)vv - cy;
            const float dX = (gu * p) / (fx + kEps) - (gu * t) / (fx + kEps);
            const float dY = (gv * p) / (fy + kEps) - (gv * t) / (fy + kEps);
            const float dZ = p - t;
            v[3] += sqrtf(dX * dX + dY * dY + dZ * dZ + kEps);
        }
    }
    block_sum<5>(v, red);
    if (threadIdx.x == 0)
        for (int i = 0; i < 5; ++i) partA[((int64_t)b * nb + blockIdx.x) * 5 + i] = v[i];
}

// pyramid scale s (1..3): avg_pool2d(k) of pred and gt; stores avgP, logP, logG
__global__ void k_pyramid(const float* __restrict__ pred, const float* __restrict__ gt, Geo g, int s,
                          float* __restrict__ avgP, float* __restrict__ logP, float* __restrict__ logG) {
    const int k = 1 << s, Hs = g.Hs[s], Ws = g.Ws[s];
    const int64_t n = (int64_t)g.B * Hs * Ws;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(i % Ws);
        const int64_t t = i / Ws;
        const int r = (int)(t % Hs), b = (int)(t / Hs);
        const int64_t base = ((int64_t)b * g.H + r * k) * g.W + j * k;
        float sp = 0.f, sg = 0.f;
        for (int y = 0; y < k; ++y)
            for (int x = 0; x < k; ++x) {
                sp += pred[base + (int64_t)y * g.W + x];
                sg += gt[base + (int64_t)y * g.W + x];
            }
        const float ap = sp / (float)(k * k), ag = sg / (float)(k * k);
        avgP[g.off[s] + i] = ap;
        logP[g.off[s] + i] = logf(clampf(ap));
        logG[g.off[s] + i] = logf(clampf(ag));
    }
}

__device__ __forceinline__ float lp_at(const float* pred, const float* logP, const Geo& g, int s, int64_t i) {
    return s == 0 ? logf(clampf(pred[i])) : logP[g.off[s] + i];
}

// gradient-matching sums for all scales: |dx| and |dy| per scale
__global__ __launch_bounds__(kTPB) void k_gradsum(const float* __restrict__ pred, const float* __restrict__ gt,
                                                  const float* __restrict__ logP, const float* __restrict__ logG,
                                                  Geo g, double* partG, int64_t total) {
    __shared__ double red[4 * 2 * kScales];
    double v[2 * kScales];
#pragma unroll
    for (int i = 0; i < 2 * kScales; ++i) v[i] = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * kTPB) {
        int s = 0;
        int64_t li = i;
        while (s < kScales - 1 && li >= (int64_t)g.B * g.Hs[s] * g.Ws[s]) { li -= (int64_t)g.B * g.Hs[s] * g.Ws[s]; ++s; }
        const int Hs = g.Hs[s], Ws = g.Ws[s];
        const int j = (int)(li % Ws), r = (int)((li / Ws) % Hs);
        const float p0 = lp_at(pred, logP, g, s, li);
        const float g0 = s == 0 ? logf(clampf(gt[li])) : logG[g.off[s] + li];
        float ax = 0.f, ay = 0.f;
        if (j + 1 < Ws) {
            const float p1 = lp_at(pred, logP, g, s, li + 1);
            const float g1 = s == 0 ? logf(clampf(gt[li + 1])) : logG[g.off[s] + li + 1];
            ax = fabsf((p1 - p0) - (g1 - g0));
        }
        if (r + 1 < Hs) {
            const float p1 = lp_at(pred, logP, g, s, li + Ws);
            const float g1 = s == 0 ? logf(clampf(gt[li + Ws])) : logG[g.off[s] + li + Ws];
            ay = fabsf((p1 - p0) - (g1 - g0));
        }
#pragma unroll
        for (int q = 0; q < kScales; ++q)
            if (q == s) { v[2 * q] += ax; v[2 * q + 1] += ay; }
    }
    block_sum<2 * kScales>(v, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < 2 * kScales; ++q) partG[(int64_t)blockIdx.x * 2 * kScales + q] = v[q];
}

// single block: reduce pass-A and gradsum partials into dsc
__global__ __launch_bounds__(kTPB) void k_reduce1(const double* partA, int nb, const double* partG, int ng,
                                                  Geo g, double* dsc) {
    __shared__ double red[4 * 8];
    double v[4];
    for (int q = 0; q < 4; ++q) v[q] = 0.0;
    for (int i = threadIdx.x; i < g.B * nb; i += kTPB)
        for (int q = 0; q < 4; ++q) v[q] += partA[(int64_t)i * 5 + q];
    block_sum<4>(v, red);
    if (threadIdx.x == 0) { dsc[S_N] = v[0]; dsc[S_SD] = v[1]; dsc[S_SD2] = v[2]; dsc[S_SE] = v[3]; }
    double w[2 * kScales];
    for (int q = 0; q < 2 * kScales; ++q) w[q] = 0.0;
    for (int i = threadIdx.x; i < ng; i += kTPB)
        for (int q = 0; q < 2 * kScales; ++q) w[q] += partG[(int64_t)i * 2 * kScales + q];
    block_sum<2 * kScales>(w, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < kScales; ++q) { dsc[S_GX0 + q] = w[2 * q]; dsc[S_GY0 + q] = w[2 * q + 1]; }
    // per-sample sum(pred)
    for (int b = 0; b < g.B; ++b) {
        double u[1] = {0.0};
        for (int i = threadIdx.x; i < nb; i += kTPB) u[0] += partA[((int64_t)b * nb + i) * 5 + 4];
        block_sum<1>(u, red);
        if (threadIdx.x == 0) dsc[S_PB + b] = u[0];
    }
}

struct SmoothCtx {
    float inv_nx, inv_ny;
};

__device__ __forceinline__ float edge_wx(const float* img, int64_t HW, int64_t i) {   // between i, i+1
    const float d0 = fabsf(img[i + 1] - img[i]);
    const float d1 = fabsf(img[HW + i + 1] - img[HW + i]);
    const float d2 = fabsf(img[2 * HW + i + 1] - img[2 * HW + i]);
    return expf(-((d0 + d1 + d2) / 3.f));
}
__device__ __forceinline__ float edge_wy(const float* img, int64_t HW, int64_t i, int W) {   // i, i+W
    const float d0 = fabsf(img[i + W] - img[i]);
    const float d1 = fabsf(img[HW + i + W] - img[HW + i]);
    const float d2 = fabsf(img[2 * HW + i + W] - img[2 * HW + i]);
    return expf(-((d0 + d1 + d2) / 3.f));
}

// dL_smooth/dn at pixel i of sample plane (pp = pred plane, img = rgb of the sample).  n = p / denom
// by true division, as the reference computes it (depth_loss.h:193): the sign of a difference of
// neighbouring n must come out as the reference's, and a rounded reciprocal can merge neighbours
// that differ by an ulp (sign 0 instead of +-1).
__device__ __forceinline__ float smooth_gn(const float* pp, const float* img, int64_t HW, int W, int H,
                                           int x, int y, int64_t i, float denom, const SmoothCtx& c) {
    const float n0 = pp[i] / denom;
    float gx = 0.f, gy = 0.f;
    if (x > 0) gx += sgnf(n0 - pp[i - 1] / denom) * edge_wx(img, HW, i - 1);
    if (x + 1 < W) gx -= sgnf(pp[i + 1] / denom - n0) * edge_wx(img, HW, i);
    if (y > 0) gy += sgnf(n0 - pp[i - W] / denom) * edge_wy(img, HW, i - W, W);
    if (y + 1 < H) gy -= sgnf(pp[i + W] / denom - n0) * edge_wy(img, HW, i, W);
    return gx * c.inv_nx + gy * c.inv_ny;
}

// smoothness forward sums (global) and per-sample coupling S_b = sum gn * p
__global__ __launch_bounds__(kTPB) void k_smooth(const float* __restrict__ pred, const float* __restrict__ rgb,
                                                 Geo g, const double* dsc, double* partS, int nb, SmoothCtx c) {
    __shared__ double red[4 * 3];
    const int b = blockIdx.y;
    const int64_t HW = (int64_t)g.H * g.W;
    const float* pp = pred + b * HW;
    const float* img = rgb + (int64_t)b * 3 * HW;
    const float mean = (float)(dsc[S_PB + b] / (double)HW);
    const float denom = mean + kEps;
    double v[3] = {0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < HW; i += (int64_t)nb * kTPB) {
        const int x = (int)(i % g.W), y = (int)(i / g.W);
        const float n0 = pp[i] / denom;
        if (x + 1 < g.W) v[0] += fabsf(pp[i + 1] / denom - n0) * edge_wx(img, HW, i);
        if (y + 1 < g.H) v[1] += fabsf(pp[i + g.W] / denom - n0) * edge_wy(img, HW, i, g.W);
        v[2] += (double)smooth_gn(pp, img, HW, g.W, g.H, x, y, i, denom, c) * pp[i];
    }
    block_sum<3>(v, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < 3; ++q) partS[((int64_t)b * nb + blockIdx.x) * 3 + q] = v[q];
}

// single block: smooth sums, S_b, final scalar losses
__global__ __launch_bounds__(kTPB) void k_reduce2(const double* partS, int nb, Geo g, double* dsc, float w0,
                                                  float w1, float w2, float w3, float* out5) {
    __shared__ double red[4 * 2];
    double v[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < g.B * nb; i += kTPB) { v[0] += partS[(int64_t)i * 3]; v[1] += partS[(int64_t)i * 3 + 1]; }
    block_sum<2>(v, red);
    if (threadIdx.x == 0) { dsc[S_SMX] = v[0]; dsc[S_SMY] = v[1]; }
    for (int b = 0; b < g.B; ++b) {
        double u[1] = {0.0};
        for (int i = threadIdx.x; i < nb; i += kTPB) u[0] += partS[((int64_t)b * nb + i) * 3 + 2];
        block_sum<1>(u, red);
        if (threadIdx.x == 0) dsc[S_PB + g.B + b] = u[0];
    }
    if (threadIdx.x == 0) {
        const double n = dsc[S_N];
        const double si = n > 0 ? dsc[S_SD2] / n - kLam * dsc[S_SD] * dsc[S_SD] / (n * n) : 0.0;
        const double rp = n > 0 ? dsc[S_SE] / n : 0.0;
        double gr = 0.0;
        for (int s = 0; s < kScales; ++s) {
            const double nx = (double)g.B * g.Hs[s] * (g.Ws[s] - 1), ny = (double)g.B * (g.Hs[s] - 1) * g.Ws[s];
            gr += dsc[S_GX0 + s] / nx + dsc[S_GY0 + s] / ny;
        }
        gr /= kScales;
        const double nx = (double)g.B * g.H * (g.W - 1), ny = (double)g.B * (g.H - 1) * g.W;
        const double sm = dsc[S_SMX] / nx + dsc[S_SMY] / ny;
        const float fsi = (float)si, fgr = (float)gr, fsm = (float)sm, frp = (float)rp;
        out5[0] = w0 * fsi + w1 * fgr + w2 * fsm + w3 * frp;
        out5[1] = fsi; out5[2] = fgr; out5[3] = fsm; out5[4] = frp;
    }
}

// dL/dP_s at pooled pixel li of scale s (sign terms of both neighbours), before the 1/4 factor
__device__ float dgrad_scale(const float* pred, const float* gt, const float* logP, const float* logG,
                             const Geo& g, int s, int64_t li, int r, int j) {
    const int Hs = g.Hs[s], Ws = g.Ws[s];
    auto P = [&](int64_t q) { return s == 0 ? logf(clampf(pred[q])) : logP[g.off[s] + q]; };
    auto G = [&](int64_t q) { return s == 0 ? logf(clampf(gt[q])) : logG[g.off[s] + q]; };
    const float p0 = P(li), g0 = G(li);
    float ax = 0.f, ay = 0.f;
    if (j > 0) ax += sgnf((p0 - P(li - 1)) - (g0 - G(li - 1)));
    if (j + 1 < Ws) ax -= sgnf((P(li + 1) - p0) - (G(li + 1) - g0));
    if (r > 0) ay += sgnf((p0 - P(li - Ws)) - (g0 - G(li - Ws)));
    if (r + 1 < Hs) ay -= sgnf((P(li + Ws) - p0) - (G(li + Ws) - g0));
    const float nx = (float)g.B * Hs * (Ws - 1), ny = (float)g.B * (Hs - 1) * Ws;
    return ax / nx + ay / ny;
}

__global__ void k_dpred(const float* __restrict__ pred, const float* __restrict__ gt, const float* __restrict__ rgb,
                        const float* __restrict__ K, const uint8_t* __restrict__ mask, const float* __restrict__ avgP,
                        const float* __restrict__ logP,
                        const float* __restrict__ logG, Geo g, const double* dsc, float w0, float w1, float w2,
                        float w3, SmoothCtx c, float* __restrict__ dpred) {
    const int64_t HW = (int64_t)g.H * g.W, n = (int64_t)g.B * HW;
    const double cnt = dsc[S_N];
    const float inv_n = cnt > 0 ? (float)(1.0 / cnt) : 0.f;
    const float sd_term = cnt > 0 ? (float)(2.0 * kLam * dsc[S_SD] / (cnt * cnt)) : 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / HW);
        const int64_t pi = i - (int64_t)b * HW;
        const int x = (int)(pi % g.W), y = (int)(pi / g.W);
        const float p = pred[i], t = gt[i];
        float grad = 0.f;
        if ((mask ? mask[i] != 0 : t > kEps) && cnt > 0) {
            // SI
            const float d = logf(clampf(p)) - logf(clampf(t));
            const float dd = 2.f * d * inv_n - sd_term;
            grad += w0 * (dd / clampf(p)) * clampgrad(p);
            // reprojection
            const float* kk = K + b * 9;
            const float fx = kk[0], cx = kk[2], fy = kk[4], cy = kk[5];
            const float gu = (float)x - cx, gv = (float)y - cy;
            const float a = gu / (fx + kEps), bb = gv / (fy + kEps);
            const float dX = (gu * p) / (fx + kEps) - (gu * t) / (fx + kEps);
            const float dY = (gv * p) / (fy + kEps) - (gv * t) / (fy + kEps);
            const float dZ = p - t;
            const float e = sqrtf(dX * dX + dY * dY + dZ * dZ + kEps);
            grad += w3 * inv_n * (dX * a + dY * bb + dZ) / e;
        }
        // gradient matching, every scale whose pooled cell covers this pixel
        float gg = 0.f;
        {
            const float dP = dgrad_scale(pred, gt, logP, logG, g, 0, i, y, x);
            gg += dP * clampgrad(p) / clampf(p);
        }
        for (int s = 1; s < kScales; ++s) {
            const int r = y >> s, j = x >> s;
            if (r >= g.Hs[s] || j >= g.Ws[s]) continue;
            const int64_t li = ((int64_t)b * g.Hs[s] + r) * g.Ws[s] + j;
            const float ap = avgP[g.off[s] + li];
            const float dP = dgrad_scale(pred, gt, logP, logG, g, s, li, r, j);
            gg += (dP * clampgrad(ap) / clampf(ap)) / (float)(1 << (2 * s));
        }
        grad += w1 * gg / (float)kScales;
        // smoothness
        {
            const float mean = (float)(dsc[S_PB + b] / (double)HW);
            const float denom = mean + kEps;
            const float gn = smooth_gn(pred + (int64_t)b * HW, rgb + (int64_t)b * 3 * HW, HW, g.W, g.H, x, y, pi,
                                       denom, c);
            const float Sb = (float)dsc[S_PB + g.B + b];
            grad += w2 * (gn / denom - Sb / (denom * denom * (float)HW));
        }
        dpred[i] = grad;
    }
}

Geo make_geo(int B, int H, int W) {
    Geo g{};
    g.B = B; g.H = H; g.W = W;
    int64_t off = 0;
    for (int s = 0; s < kScales; ++s) {
        g.Hs[s] = H >> s;
        g.Ws[s] = W >> s;
        g.off[s] = s == 0 ? 0 : off;
        if (s > 0) off += (int64_t)B * g.Hs[s] * g.Ws[s];
    }
    g.pyr_n = off;
    return g;
}
int nb_per_sample(int B, int64_t HW) {
    return std::max(1, std::min(cdiv(1024, B), cdiv(HW, kTPB)));
}
int ng_blocks(int64_t total) { return std::max(1, std::min(1024, cdiv(total, kTPB))); }
}  // namespace

int64_t loss_workspace_floats(int B, int H, int W) { return 3 * make_geo(B, H, W).pyr_n + 64; }
int64_t loss_part_doubles(int B, int H, int W) {
    const int nb = nb_per_sample(B, (int64_t)H * W);
    return (int64_t)B * nb * 5 + 1024 * 2 * kScales + (int64_t)B * nb * 3 + S_PB + 2 * B + 64;
}

void loss_fwd_bwd(const float* pred, const float* gt, const float* rgb, const float* K, const uint8_t* mask, int B,
                  int H, int W, const float w[4], float* out5, float* dpred, LossWorkspace ws, hipStream_t st) {
    Geo g = make_geo(B, H, W);
    const int64_t HW = (int64_t)H * W;
    const int nb = nb_per_sample(B, HW);
    int64_t total = 0;
    for (int s = 0; s < kScales; ++s) total += (int64_t)B * g.Hs[s] * g.Ws[s];
    const int ng = ng_blocks(total);
    double* dsc = ws.part;
    double* partA = dsc + S_PB + 2 * B + 16;
    double* partG = partA + (int64_t)B * nb * 5;
    double* partS = partG + (int64_t)ng * 2 * kScales;
    float* avgP = ws.pyr;
    float* logP = avgP + g.pyr_n;
    float* logG = logP + g.pyr_n;
    SmoothCtx c;
    c.inv_nx = 1.f / ((float)B * H * (W - 1));
    c.inv_ny = 1.f / ((float)B * (H - 1) * W);

    hipLaunchKernelGGL(k_passA, dim3(nb, B), dim3(kTPB), 0, st, pred, gt, K, mask, g, partA, nb);
    for (int s = 1; s < kScales; ++s) {
        const int64_t n = (int64_t)B * g.Hs[s] * g.Ws[s];
        if (n > 0)
            hipLaunchKernelGGL(k_pyramid, dim3(std::max(1, std::min(4096, cdiv(n, 256)))), dim3(256), 0, st, pred, gt, g, s,
                               avgP, logP, logG);
    }
    hipLaunchKernelGGL(k_gradsum, dim3(ng), dim3(kTPB), 0, st, pred, gt, logP, logG, g, partG, total);
    hipLaunchKernelGGL(k_reduce1, dim3(1), dim3(kTPB), 0, st, partA, nb, partG, ng, g, dsc);
    hipLaunchKernelGGL(k_smooth, dim3(nb, B), dim3(kTPB), 0, st, pred, rgb, g, dsc, partS, nb, c);
    hipLaunchKernelGGL(k_reduce2, dim3(1), dim3(kTPB), 0, st, partS, nb, g, dsc, w[0], w[1], w[2], w[3], out5);
    const int64_t n = (int64_t)B * HW;
    hipLaunchKernelGGL(k_dpred, dim3(std::max(1, std::min(8192, cdiv(n, 256)))), dim3(256), 0, st, pred, gt, rgb, K,
                       mask, avgP, logP, logG, g, dsc, w[0], w[1], w[2], w[3], c, dpred);
}

}  // namespace cad
