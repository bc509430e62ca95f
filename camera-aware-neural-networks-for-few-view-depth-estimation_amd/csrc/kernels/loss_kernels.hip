// Fused depth-loss forward + analytic backward.
// Replaces CombinedDepthLoss::forwardWithIntrinsics (src/loss/depth_loss.h:416-433) and its autograd
// backward with two fused passes over the depth map and two single-block reductions: pass A (SI /
// reprojection sums, per-sample sum(pred), the scale-0 logs and the smoothness edge weights), the
// pooled pyramid (one launch for scales 1-3), reduction 1, pass B (smoothness sums and S_b, the
// gradient-matching sums of every scale, dL/dpred), reduction 2 (the five losses), and, when the
// smoothness weight is non-zero, the per-sample S_b coupling subtracted from dL/dpred.  Partials are
// fp64 in a fixed order (no atomics, bitwise-reproducible); index math is 32-bit (multiply-shift
// division: B*H*W < 2^31, checked).
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
    int cells;              // pooled cells of one sample over scales 1..3
    FastDiv dW;             // / W
    FastDiv dWs[kScales];   // / Ws[s]
    FastDiv dHs[kScales];   // / Hs[s]
};

// scalar slots (double) in dsc
enum { S_N = 0, S_SD, S_SD2, S_SE, S_GX0, S_GY0 = S_GX0 + kScales, S_SMX = S_GY0 + kScales, S_SMY,
       S_PB /* B per-sample sum(pred) */ };
// per-sample tail after S_PB: [B] sum pred, [B] S_b (sum gn*p)
constexpr int kPA = 5;                  // pass-A partials per block: n, sum d, sum d^2, sum e, sum pred
constexpr int kPB = 3 + 2 * kScales;    // pass-B partials: smooth x, smooth y, S_b, |dx| / |dy| per scale

__device__ __forceinline__ float edge_w(const float* img, int64_t HW, int64_t i, int64_t step) {   // between i, i+step
    const float d0 = fabsf(img[i + step] - img[i]);
    const float d1 = fabsf(img[HW + i + step] - img[HW + i]);
    const float d2 = fabsf(img[2 * HW + i + step] - img[2 * HW + i]);
    return expf(-((d0 + d1 + d2) / 3.f));
}

// Pass A, per (sample, chunk): SI + reprojection sums over the mask, per-sample sum(pred); and, per
// pixel, the scale-0 logs log(clamp p), log(clamp g) and the smoothness edge weights of its right and
// lower edges (0 past the border) — each computed once here and read by pass B's stencils (the
// previous kernels evaluated every log up to 10x and every edge weight up to 10x per pixel)
__global__ __launch_bounds__(kTPB) void k_lossA(const float* __restrict__ pred, const float* __restrict__ gt,
                                                const float* __restrict__ rgb, const float* __restrict__ K,
                                                const uint8_t* __restrict__ mask, Geo g, float* __restrict__ lp0,
                                                float* __restrict__ lg0, float* __restrict__ wx, float* __restrict__ wy,
                                                double* partA, int nb) {
    __shared__ double red[4 * kPA];
    const int b = blockIdx.y;
    const int HW = g.H * g.W;
    const float* kk = K + b * 9;
    const float fx = kk[0], cx = kk[2], fy = kk[4], cy = kk[5];
    const float* img = rgb + (int64_t)b * 3 * HW;
    const int64_t o = (int64_t)b * HW;
    double v[kPA] = {0, 0, 0, 0, 0};
    for (int i = blockIdx.x * kTPB + threadIdx.x; i < HW; i += nb * kTPB) {
        const float p = pred[o + i], t = gt[o + i];
        const int y = (int)fdiv(g.dW, (uint32_t)i), x = i - y * g.W;
        const float lp = logf(clampf(p)), lg = logf(clampf(t));
        lp0[o + i] = lp;
        lg0[o + i] = lg;
        wx[o + i] = x + 1 < g.W ? edge_w(img, HW, i, 1) : 0.f;
        wy[o + i] = y + 1 < g.H ? edge_w(img, HW, i, g.W) : 0.f;
        v[4] += p;
        if (mask ? mask[o + i] != 0 : t > kEps) {
            const float d = lp - lg;
            v[0] += 1.0;
            v[1] += d;
            v[2] += (double)d * d;
            const float gu = (float)x - cx, gv = (float)y - cy;
            const float dX = (gu * p) / (fx + kEps) - (gu * t) / (fx + kEps);
            const float dY = (gv * p) / (fy + kEps) - (gv * t) / (fy + kEps);
            const float dZ = p - t;
            v[3] += sqrtf(dX * dX + dY * dY + dZ * dZ + kEps);
        }
    }
    block_sum<kPA>(v, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < kPA; ++q) partA[((int64_t)b * nb + blockIdx.x) * kPA + q] = v[q];
}

// pyramid, scales 1..3 in one launch: avg_pool2d(k = 2^s) of pred and gt -> avgP, logP, logG
__global__ void k_lossPyr(const float* __restrict__ pred, const float* __restrict__ gt, Geo g, int total,
                          float* __restrict__ avgP, float* __restrict__ logP, float* __restrict__ logG) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        int s = 1, li = i;
        while (s < kScales - 1 && li >= g.B * g.Hs[s] * g.Ws[s]) { li -= g.B * g.Hs[s] * g.Ws[s]; ++s; }
        const int k = 1 << s, Hs = g.Hs[s], Ws = g.Ws[s];
        const int t = (int)fdiv(g.dWs[s], (uint32_t)li), j = li - t * Ws;
        const int b = (int)fdiv(g.dHs[s], (uint32_t)t), r = t - b * Hs;
        const int64_t base = ((int64_t)b * g.H + r * k) * g.W + j * k;
        float sp = 0.f, sg = 0.f;
        for (int yy = 0; yy < k; ++yy)
            for (int xx = 0; xx < k; ++xx) {
                sp += pred[base + (int64_t)yy * g.W + xx];
                sg += gt[base + (int64_t)yy * g.W + xx];
            }
        const float ap = sp / (float)(k * k), ag = sg / (float)(k * k);
        avgP[g.off[s] + li] = ap;
        logP[g.off[s] + li] = logf(clampf(ap));
        logG[g.off[s] + li] = logf(clampf(ag));
    }
}

// single block: pass-A partials -> dsc (SI / reprojection sums, per-sample sum(pred))
__global__ __launch_bounds__(kTPB) void k_lossR1(const double* partA, int nb, Geo g, double* dsc) {
    __shared__ double red[4 * 4];
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < g.B * nb; i += kTPB)
        for (int q = 0; q < 4; ++q) v[q] += partA[(int64_t)i * kPA + q];
    block_sum<4>(v, red);
    if (threadIdx.x == 0) { dsc[S_N] = v[0]; dsc[S_SD] = v[1]; dsc[S_SD2] = v[2]; dsc[S_SE] = v[3]; }
    for (int b = 0; b < g.B; ++b) {
        double u[1] = {0.0};
        for (int i = threadIdx.x; i < nb; i += kTPB) u[0] += partA[((int64_t)b * nb + i) * kPA + 4];
        block_sum<1>(u, red);
        if (threadIdx.x == 0) dsc[S_PB + b] = u[0];
    }
}

struct SmoothCtx {
    float inv_nx, inv_ny;
};

// dL_smooth/dn at pixel i of the sample plane (pp = pred plane, wx / wy its edge weights).  n = p /
// denom by true division, as the reference computes it (depth_loss.h:193): the sign of a difference of
// neighbouring n must come out as the reference's, and a rounded reciprocal can merge neighbours that
// differ by an ulp (sign 0 instead of +-1).
__device__ __forceinline__ float smooth_gn(const float* pp, const float* wxp, const float* wyp, int W, int H, int x,
                                           int y, int i, float denom, const SmoothCtx& c) {
    const float n0 = pp[i] / denom;
    float gx = 0.f, gy = 0.f;
    if (x > 0) gx += sgnf(n0 - pp[i - 1] / denom) * wxp[i - 1];
    if (x + 1 < W) gx -= sgnf(pp[i + 1] / denom - n0) * wxp[i];
    if (y > 0) gy += sgnf(n0 - pp[i - W] / denom) * wyp[i - W];
    if (y + 1 < H) gy -= sgnf(pp[i + W] / denom - n0) * wyp[i];
    return gx * c.inv_nx + gy * c.inv_ny;
}

// dL/dP_s at pooled pixel li of scale s >= 1 (sign terms of both neighbours), before the 1/4^s factor
__device__ float dgrad_pyr(const float* logP, const float* logG, const Geo& g, int s, int64_t li, int r, int j) {
    const int Hs = g.Hs[s], Ws = g.Ws[s];
    const float* P = logP + g.off[s];
    const float* G = logG + g.off[s];
    const float p0 = P[li], g0 = G[li];
    float ax = 0.f, ay = 0.f;
    if (j > 0) ax += sgnf((p0 - P[li - 1]) - (g0 - G[li - 1]));
    if (j + 1 < Ws) ax -= sgnf((P[li + 1] - p0) - (G[li + 1] - g0));
    if (r > 0) ay += sgnf((p0 - P[li - Ws]) - (g0 - G[li - Ws]));
    if (r + 1 < Hs) ay -= sgnf((P[li + Ws] - p0) - (G[li + Ws] - g0));
    const float nx = (float)g.B * Hs * (Ws - 1), ny = (float)g.B * (Hs - 1) * Ws;
    return ax / nx + ay / ny;
}

// Pass B, per (sample, chunk), after pass A's sums: the smoothness sums and S_b = sum gn p, the
// gradient-matching |dx| / |dy| sums of every scale, and dL/dpred of every term but the smoothness
// term's per-sample coupling -w2 S_b / (denom^2 HW), which k_lossC subtracts once S_b is reduced.
__global__ __launch_bounds__(kTPB) void k_lossB(const float* __restrict__ pred, const float* __restrict__ gt,
                                                const float* __restrict__ K, const uint8_t* __restrict__ mask,
                                                const float* __restrict__ lp0, const float* __restrict__ lg0,
                                                const float* __restrict__ wx, const float* __restrict__ wy,
                                                const float* __restrict__ avgP, const float* __restrict__ logP,
                                                const float* __restrict__ logG, Geo g, const double* dsc, float w0,
                                                float w1, float w2, float w3, SmoothCtx c, float* __restrict__ dpred,
                                                double* partB, int nb) {
    __shared__ double red[4 * kPB];
    const int b = blockIdx.y;
    const int HW = g.H * g.W, W = g.W;
    const int64_t o = (int64_t)b * HW;
    const float* pp = pred + o;
    const float* lp = lp0 + o;
    const float* lg = lg0 + o;
    const float* wxp = wx + o;
    const float* wyp = wy + o;
    const float mean = (float)(dsc[S_PB + b] / (double)HW);
    const float denom = mean + kEps;
    const double cnt = dsc[S_N];
    const float inv_n = cnt > 0 ? (float)(1.0 / cnt) : 0.f;
    const float sd_term = cnt > 0 ? (float)(2.0 * kLam * dsc[S_SD] / (cnt * cnt)) : 0.f;
    const float* kk = K + b * 9;
    const float fx = kk[0], cx = kk[2], fy = kk[4], cy = kk[5];
    const float nx0 = (float)g.B * g.H * (W - 1), ny0 = (float)g.B * (g.H - 1) * W;
    double v[kPB];
#pragma unroll
    for (int q = 0; q < kPB; ++q) v[q] = 0.0;
    for (int i = blockIdx.x * kTPB + threadIdx.x; i < HW; i += nb * kTPB) {
        const int y = (int)fdiv(g.dW, (uint32_t)i), x = i - y * W;
        const float p = pp[i], t = gt[o + i];
        // smoothness: forward sums and gn
        const float n0 = p / denom;
        if (x + 1 < W) v[0] += fabsf(pp[i + 1] / denom - n0) * wxp[i];
        if (y + 1 < g.H) v[1] += fabsf(pp[i + W] / denom - n0) * wyp[i];
        const float gn = smooth_gn(pp, wxp, wyp, W, g.H, x, y, i, denom, c);
        v[2] += (double)gn * p;
        // gradient matching at scale 0: sums and the sign terms of both neighbours
        const float p0 = lp[i], g0 = lg[i];
        float ax = 0.f, ay = 0.f;
        if (x > 0) ax += sgnf((p0 - lp[i - 1]) - (g0 - lg[i - 1]));
        if (x + 1 < W) {
            const float dx = (lp[i + 1] - p0) - (lg[i + 1] - g0);
            v[3] += fabsf(dx);
            ax -= sgnf(dx);
        }
        if (y > 0) ay += sgnf((p0 - lp[i - W]) - (g0 - lg[i - W]));
        if (y + 1 < g.H) {
            const float dy = (lp[i + W] - p0) - (lg[i + W] - g0);
            v[4] += fabsf(dy);
            ay -= sgnf(dy);
        }
        // dL/dpred
        float grad = 0.f;
        if ((mask ? mask[o + i] != 0 : t > kEps) && cnt > 0) {
            // SI
            const float d = p0 - g0;
            const float dd = 2.f * d * inv_n - sd_term;
            grad += w0 * (dd / clampf(p)) * clampgrad(p);
            // reprojection
            const float gu = (float)x - cx, gv = (float)y - cy;
            const float a = gu / (fx + kEps), bb = gv / (fy + kEps);
            const float dX = (gu * p) / (fx + kEps) - (gu * t) / (fx + kEps);
            const float dY = (gv * p) / (fy + kEps) - (gv * t) / (fy + kEps);
            const float dZ = p - t;
            const float e = sqrtf(dX * dX + dY * dY + dZ * dZ + kEps);
            grad += w3 * inv_n * (dX * a + dY * bb + dZ) / e;
        }
        float gg = (ax / nx0 + ay / ny0) * clampgrad(p) / clampf(p);
        for (int s = 1; s < kScales; ++s) {
            const int r = y >> s, j = x >> s;
            if (r >= g.Hs[s] || j >= g.Ws[s]) continue;
            const int64_t li = ((int64_t)b * g.Hs[s] + r) * g.Ws[s] + j;
            const float ap = avgP[g.off[s] + li];
            const float dP = dgrad_pyr(logP, logG, g, s, li, r, j);
            gg += (dP * clampgrad(ap) / clampf(ap)) / (float)(1 << (2 * s));
        }
        grad += w1 * gg / (float)kScales;
        dpred[o + i] = grad + w2 * (gn / denom);
    }
    // gradient-matching sums at scales 1..3 over this sample's pooled cells
    for (int ci = blockIdx.x * kTPB + threadIdx.x; ci < g.cells; ci += nb * kTPB) {
        int s = 1, li = ci;
        while (s < kScales - 1 && li >= g.Hs[s] * g.Ws[s]) { li -= g.Hs[s] * g.Ws[s]; ++s; }
        const int Ws = g.Ws[s];
        const int r = (int)fdiv(g.dWs[s], (uint32_t)li), j = li - r * Ws;
        const int64_t q = (int64_t)b * g.Hs[s] * Ws + li;
        const float* P = logP + g.off[s];
        const float* G = logG + g.off[s];
        const float p0 = P[q], g0 = G[q];
        float ax = 0.f, ay = 0.f;
        if (j + 1 < Ws) ax = fabsf((P[q + 1] - p0) - (G[q + 1] - g0));
        if (r + 1 < g.Hs[s]) ay = fabsf((P[q + Ws] - p0) - (G[q + Ws] - g0));
#pragma unroll
        for (int u = 1; u < kScales; ++u)
            if (u == s) { v[3 + 2 * u] += ax; v[4 + 2 * u] += ay; }
    }
    block_sum<kPB>(v, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < kPB; ++q) partB[((int64_t)b * nb + blockIdx.x) * kPB + q] = v[q];
}

// single block: pass-B partials -> smoothness sums, S_b, gradient-matching sums, the five losses
__global__ __launch_bounds__(kTPB) void k_lossR2(const double* partB, int nb, Geo g, double* dsc, float w0, float w1,
                                                 float w2, float w3, float* out5) {
    __shared__ double red[4 * (2 + 2 * kScales)];
    double v[2 + 2 * kScales];
#pragma unroll
    for (int q = 0; q < 2 + 2 * kScales; ++q) v[q] = 0.0;
    for (int i = threadIdx.x; i < g.B * nb; i += kTPB) {
        const double* pr = partB + (int64_t)i * kPB;
        v[0] += pr[0];
        v[1] += pr[1];
#pragma unroll
        for (int q = 0; q < 2 * kScales; ++q) v[2 + q] += pr[3 + q];
    }
    block_sum<2 + 2 * kScales>(v, red);
    if (threadIdx.x == 0) {
        dsc[S_SMX] = v[0];
        dsc[S_SMY] = v[1];
        for (int s = 0; s < kScales; ++s) { dsc[S_GX0 + s] = v[2 + 2 * s]; dsc[S_GY0 + s] = v[3 + 2 * s]; }
    }
    for (int b = 0; b < g.B; ++b) {
        double u[1] = {0.0};
        for (int i = threadIdx.x; i < nb; i += kTPB) u[0] += partB[((int64_t)b * nb + i) * kPB + 2];
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

// the smoothness term's per-sample coupling: dpred -= w2 S_b / (denom^2 HW) (w2 != 0 only)
__global__ void k_lossC(Geo g, const double* dsc, float w2, float* __restrict__ dpred) {
    const int b = blockIdx.y;
    const int HW = g.H * g.W;
    const float mean = (float)(dsc[S_PB + b] / (double)HW);
    const float denom = mean + kEps;
    const float Sb = (float)dsc[S_PB + g.B + b];
    const float cb = w2 * (Sb / (denom * denom * (float)HW));
    float* d = dpred + (int64_t)b * HW;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += gridDim.x * blockDim.x) d[i] -= cb;
}

Geo make_geo(int B, int H, int W) {
    Geo g{};
    g.B = B; g.H = H; g.W = W;
    int64_t off = 0;
    for (int s = 0; s < kScales; ++s) {
        g.Hs[s] = H >> s;
        g.Ws[s] = W >> s;
        g.off[s] = s == 0 ? 0 : off;
        if (s > 0) {
            off += (int64_t)B * g.Hs[s] * g.Ws[s];
            g.cells += g.Hs[s] * g.Ws[s];
        }
        g.dWs[s] = make_fastdiv((uint32_t)std::max(1, g.Ws[s]));
        g.dHs[s] = make_fastdiv((uint32_t)std::max(1, g.Hs[s]));
    }
    g.dW = make_fastdiv((uint32_t)W);
    g.pyr_n = off;
    return g;
}
int nb_per_sample(int B, int64_t HW) {
    return std::max(1, std::min(cdiv(2048, B), cdiv(HW, kTPB)));
}
}  // namespace

int64_t loss_workspace_floats(int B, int H, int W) {
    // pyramid (avgP, logP, logG for scales 1..3), then scale-0 logs and edge weights (lp, lg, wx, wy)
    return 3 * make_geo(B, H, W).pyr_n + 4 * (int64_t)B * H * W + 64;
}
int64_t loss_part_doubles(int B, int H, int W) {
    const int nb = nb_per_sample(B, (int64_t)H * W);
    return (int64_t)B * nb * (kPA + kPB) + S_PB + 2 * B + 64;
}

void loss_fwd_bwd(const float* pred, const float* gt, const float* rgb, const float* K, const uint8_t* mask, int B,
                  int H, int W, const float w[4], float* out5, float* dpred, LossWorkspace ws, hipStream_t st) {
    if ((int64_t)B * H * W >= ((int64_t)1 << 31) || H < 2 || W < 2)
        throw std::runtime_error("loss: B*H*W must stay below 2^31 and H, W >= 2");
    Geo g = make_geo(B, H, W);
    const int64_t HW = (int64_t)H * W, n = (int64_t)B * HW;
    const int nb = nb_per_sample(B, HW);
    double* dsc = ws.part;
    double* partA = dsc + S_PB + 2 * B + 16;
    double* partB = partA + (int64_t)B * nb * kPA;
    float* avgP = ws.pyr;
    float* logP = avgP + g.pyr_n;
    float* logG = logP + g.pyr_n;
    float* lp0 = logG + g.pyr_n;
    float* lg0 = lp0 + n;
    float* wx = lg0 + n;
    float* wy = wx + n;
    SmoothCtx c;
    c.inv_nx = 1.f / ((float)B * H * (W - 1));
    c.inv_ny = 1.f / ((float)B * (H - 1) * W);
    CAD_NO_ALIAS("loss_fwd_bwd", {aview(dpred, n, 1, 0, 1, 4, "dpred"), aview(ws.pyr, 1, 1, 0, 3 * g.pyr_n + 4 * n, 4, "workspace")},
                 {aview(pred, n, 1, 0, 1, 4, "pred"), aview(gt, n, 1, 0, 1, 4, "gt"), aview(rgb, 3 * n, 1, 0, 1, 4, "rgb"),
                  aview(mask, n, 1, 0, 1, 1, "mask")});

    hipLaunchKernelGGL(k_lossA, dim3(nb, B), dim3(kTPB), 0, st, pred, gt, rgb, K, mask, g, lp0, lg0, wx, wy, partA, nb);
    const int64_t total = g.pyr_n;
    if (total > 0)
        hipLaunchKernelGGL(k_lossPyr, dim3(std::max(1, std::min(8192, cdiv(total, 256)))), dim3(256), 0, st, pred, gt, g,
                           (int)total, avgP, logP, logG);
    hipLaunchKernelGGL(k_lossR1, dim3(1), dim3(kTPB), 0, st, partA, nb, g, dsc);
    hipLaunchKernelGGL(k_lossB, dim3(nb, B), dim3(kTPB), 0, st, pred, gt, K, mask, lp0, lg0, wx, wy, avgP, logP, logG, g,
                       dsc, w[0], w[1], w[2], w[3], c, dpred, partB, nb);
    hipLaunchKernelGGL(k_lossR2, dim3(1), dim3(kTPB), 0, st, partB, nb, g, dsc, w[0], w[1], w[2], w[3], out5);
    if (w[2] != 0.f)
        hipLaunchKernelGGL(k_lossC, dim3(std::max(1, std::min(256, cdiv(HW, 256 * 4))), B), dim3(256), 0, st, g, dsc, w[2],
                           dpred);
}

}  // namespace cad
