// Fused depth-loss forward + analytic backward.
// Replaces CombinedDepthLoss::forwardWithIntrinsics (src/loss/depth_loss.h:416-433) and its autograd
// backward with two fused passes over the depth map: pass A (SI / reprojection sums, per-sample
// sum(pred), the scale-0 logs and the smoothness edge weights), the pooled pyramid (scales 1-3 from
// one read of each 8x8 block), the pyramid's gradient terms per pooled cell, reduction 1, pass B
// (smoothness sums and S_b, the gradient-matching sums of every scale, dL/dpred; each wave walks 64
// columns down a band of rows so that every n = p / denom is divided once, not five times),
// and reduction 2 (the five losses; when the smoothness weight is non-zero, also the per-sample S_b
// coupling subtracted from dL/dpred).  Partials are fp64 in a fixed order (no atomics,
// bitwise-reproducible); index math is 32-bit (multiply-shift division: B*H*W < 2^31, checked).
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
        const int y = (int)fdiv(g.dW, (uint32_t)i), x = i - y * g.W;
        // all loads up front, neighbours at clamped addresses (branch-guarded loads wait one by one)
        const bool hR = x + 1 < g.W, hD = y + 1 < g.H;
        const int iR = hR ? i + 1 : i, iD = hD ? i + g.W : i;
        const float p = pred[o + i], t = gt[o + i];
        float c0[3], cr[3], cd[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            c0[ch] = img[ch * HW + i];
            cr[ch] = img[ch * HW + iR];
            cd[ch] = img[ch * HW + iD];
        }
        const bool valid = mask ? mask[o + i] != 0 : t > kEps;
        const float lp = logf(clampf(p)), lg = logf(clampf(t));
        lp0[o + i] = lp;
        lg0[o + i] = lg;
        // exp(-mean |dI|) over the 3 channels, between i and its right / lower neighbour (0 past the border)
        wx[o + i] = hR ? expf(-((fabsf(cr[0] - c0[0]) + fabsf(cr[1] - c0[1]) + fabsf(cr[2] - c0[2])) / 3.f)) : 0.f;
        wy[o + i] = hD ? expf(-((fabsf(cd[0] - c0[0]) + fabsf(cd[1] - c0[1]) + fabsf(cd[2] - c0[2])) / 3.f)) : 0.f;
        v[4] += p;
        if (valid) {
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

// pyramid, scales 1..3 in one launch: avg_pool2d(k = 2^s) of pred and gt -> avgP, logP, logG.  One
// thread per 8 x 8 block of the depth map (4 x 4 scale-1 cells, 2 x 2 scale-2, one scale-3 cell) reads
// each pixel once; every window still sums its k x k pixels in row-major order (avg_pool2d's sum)
__global__ __launch_bounds__(256) void k_lossPyr(const float* __restrict__ pred, const float* __restrict__ gt, Geo g, int nby, int nbx,
                          int total, float* __restrict__ avgP, float* __restrict__ logP, float* __restrict__ logG) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const int q = t / nbx, bx = t - q * nbx;
        const int b = q / nby, by = q - b * nby;
        float sp1[16], sg1[16], sp2[4], sg2[4], sp3 = 0.f, sg3 = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) sp1[k] = sg1[k] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) sp2[k] = sg2[k] = 0.f;
        const float* pb = pred + (int64_t)b * g.H * g.W;
        const float* gb = gt + (int64_t)b * g.H * g.W;
        // whole 8-pixel rows as two 16-byte loads each when they lie inside the scale-1 grid
        const bool vec = (g.W & 3) == 0 && 8 * bx + 8 <= 2 * g.Ws[1];
#pragma unroll
        for (int yy = 0; yy < 8; ++yy) {
            const int r1 = 4 * by + (yy >> 1);
            if (r1 >= g.Hs[1]) break;
            const int64_t row = (int64_t)(8 * by + yy) * g.W + 8 * bx;
            float vp[8], vg[8];
            if (vec) {
                const float4 p0 = *reinterpret_cast<const float4*>(pb + row), p1 = *reinterpret_cast<const float4*>(pb + row + 4);
                const float4 q0 = *reinterpret_cast<const float4*>(gb + row), q1 = *reinterpret_cast<const float4*>(gb + row + 4);
                vp[0] = p0.x; vp[1] = p0.y; vp[2] = p0.z; vp[3] = p0.w; vp[4] = p1.x; vp[5] = p1.y; vp[6] = p1.z; vp[7] = p1.w;
                vg[0] = q0.x; vg[1] = q0.y; vg[2] = q0.z; vg[3] = q0.w; vg[4] = q1.x; vg[5] = q1.y; vg[6] = q1.z; vg[7] = q1.w;
            } else {
#pragma unroll
                for (int xx = 0; xx < 8; ++xx) {
                    const bool in = 4 * bx + (xx >> 1) < g.Ws[1];
                    vp[xx] = in ? pb[row + xx] : 0.f;
                    vg[xx] = in ? gb[row + xx] : 0.f;
                }
            }
#pragma unroll
            for (int xx = 0; xx < 8; ++xx) {
                if (4 * bx + (xx >> 1) < g.Ws[1]) {   // (row-major order inside every window)
                    const int k1 = (yy >> 1) * 4 + (xx >> 1), k2 = (yy >> 2) * 2 + (xx >> 2);
                    sp1[k1] += vp[xx]; sg1[k1] += vg[xx];
                    sp2[k2] += vp[xx]; sg2[k2] += vg[xx];
                    sp3 += vp[xx]; sg3 += vg[xx];
                }
            }
        }
        auto put = [&](int s, int r, int j, float sp, float sg) {
            if (r >= g.Hs[s] || j >= g.Ws[s]) return;
            const float kk = (float)(1 << (2 * s));
            const float ap = sp / kk, ag = sg / kk;
            const int64_t li = g.off[s] + ((int64_t)b * g.Hs[s] + r) * g.Ws[s] + j;
            avgP[li] = ap;
            logP[li] = logf(clampf(ap));
            logG[li] = logf(clampf(ag));
        };
#pragma unroll
        for (int k = 0; k < 16; ++k) put(1, 4 * by + (k >> 2), 4 * bx + (k & 3), sp1[k], sg1[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) put(2, 2 * by + (k >> 1), 2 * bx + (k & 1), sp2[k], sg2[k]);
        put(3, by, bx, sp3, sg3);
    }
}

// pass-A partials -> dsc: block 0 the SI / reprojection sums, block 1 + b sample b's sum(pred)
__global__ __launch_bounds__(kTPB) void k_lossR1(const double* partA, int nb, Geo g, double* dsc) {
    __shared__ double red[4 * 4];
    if (blockIdx.x == 0) {
        double v[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = threadIdx.x; i < g.B * nb; i += kTPB)
            for (int q = 0; q < 4; ++q) v[q] += partA[(int64_t)i * kPA + q];
        block_sum<4>(v, red);
        if (threadIdx.x == 0) { dsc[S_N] = v[0]; dsc[S_SD] = v[1]; dsc[S_SD2] = v[2]; dsc[S_SE] = v[3]; }
    } else {
        const int b = blockIdx.x - 1;
        double u[1] = {0.0};
        for (int i = threadIdx.x; i < nb; i += kTPB) u[0] += partA[((int64_t)b * nb + i) * kPA + 4];
        block_sum<1>(u, red);
        if (threadIdx.x == 0) dsc[S_PB + b] = u[0];
    }
}

struct SmoothCtx {
    float inv_nx, inv_ny;
};

// dL/dP_s at pooled pixel li of scale s >= 1 (sign terms of both neighbours), before the 1/4^s factor
__device__ float dgrad_pyr(const float* logP, const float* logG, const Geo& g, int s, int64_t li, int r, int j) {
    const int Hs = g.Hs[s], Ws = g.Ws[s];
    const float* P = logP + g.off[s];
    const float* G = logG + g.off[s];
    // neighbours loaded up front at clamped addresses
    const bool hL = j > 0, hR = j + 1 < Ws, hU = r > 0, hD = r + 1 < Hs;
    const int64_t iL = hL ? li - 1 : li, iR = hR ? li + 1 : li, iU = hU ? li - Ws : li, iD = hD ? li + Ws : li;
    const float p0 = P[li], g0 = G[li], pl = P[iL], gl = G[iL], pr = P[iR], gr = G[iR];
    const float pu = P[iU], gu = G[iU], pd = P[iD], gd = G[iD];
    float ax = 0.f, ay = 0.f;
    if (hL) ax += sgnf((p0 - pl) - (g0 - gl));
    if (hR) ax -= sgnf((pr - p0) - (gr - g0));
    if (hU) ay += sgnf((p0 - pu) - (g0 - gu));
    if (hD) ay -= sgnf((pd - p0) - (gd - g0));
    const float nx = (float)g.B * Hs * (Ws - 1), ny = (float)g.B * (Hs - 1) * Ws;
    return ax / nx + ay / ny;
}

// the pyramid's term of dL_grad/dpred per pooled cell, (dP clampgrad(ap) / clampf(ap)) / 4^s: the
// 4^s depth pixels under a cell add the same value (pass B reads it instead of re-deriving it)
__global__ void k_lossPyrG(const float* __restrict__ avgP, const float* __restrict__ logP,
                           const float* __restrict__ logG, Geo g, float* __restrict__ gP) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)g.pyr_n; i += gridDim.x * blockDim.x) {
        int s = 1, li = i;
        while (s < kScales - 1 && li >= g.B * g.Hs[s] * g.Ws[s]) { li -= g.B * g.Hs[s] * g.Ws[s]; ++s; }
        const int t = (int)fdiv(g.dWs[s], (uint32_t)li), j = li - t * g.Ws[s];
        const int r = t - (int)fdiv(g.dHs[s], (uint32_t)t) * g.Hs[s];
        const float ap = avgP[g.off[s] + li];
        const float dP = dgrad_pyr(logP, logG, g, s, li, r, j);
        gP[g.off[s] + li] = (dP * clampgrad(ap) / clampf(ap)) / (float)(1 << (2 * s));
    }
}

// Pass B, per (sample, chunk), after pass A's sums: the smoothness sums and S_b = sum gn p, the
// gradient-matching |dx| / |dy| sums of every scale, and dL/dpred of every term but the smoothness
// term's per-sample coupling -w2 S_b / (denom^2 HW), which reduction 2 subtracts once S_b is summed.
// Pixel walk: wave w of the sample takes 64 columns (cg) of a band of rpb rows and walks down it, so
// n = p / denom of the row below is the only division per pixel (the row above and this row come
// from the previous step, the left / right neighbours from lanes -+1; the wave's edge lanes divide
// their outside neighbour) — the same quotients as dividing each neighbour where it is used.
__global__ __launch_bounds__(kTPB) __attribute__((amdgpu_waves_per_eu(6))) void k_lossB(const float* __restrict__ pred, const float* __restrict__ gt,
                                                const float* __restrict__ K, const uint8_t* __restrict__ mask,
                                                const float* __restrict__ lp0, const float* __restrict__ lg0,
                                                const float* __restrict__ wx, const float* __restrict__ wy,
                                                const float* __restrict__ logP, const float* __restrict__ logG,
                                                const float* __restrict__ gP, Geo g, const double* dsc, float w0,
                                                float w1, float w2, float w3, SmoothCtx c, float* __restrict__ dpred,
                                                double* partB, int nb, int ncg, int rpb) {
    __shared__ double red[4 * kPB];
    const int b = blockIdx.y;
    const int HW = g.H * g.W, W = g.W, H = g.H;
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
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
    const int band = gw / ncg, cg = gw - band * ncg;
    const int x = cg * 64 + lane;
    const bool xin = x < W;
    const int xc = xin ? x : W - 1;   // lanes past the edge load column W - 1 and discard it
    const int ya = band * rpb, yb = min(H, ya + rpb);   // wave-uniform
    // the walk carries this row's p, log p, log g and the row above's log p, log g, wy, n from the
    // previous step; every load of a step is issued up front at clamped addresses (branch-guarded
    // loads each waited on their own: ~10 serialised memory latencies per pixel row)
    float nU = 0.f, n0 = 0.f, p = 0.f, p0 = 0.f, g0 = 0.f, pu = 0.f, gu_ = 0.f, wyu = 0.f;
    if (ya < yb) {
        const int i = ya * W + xc, iU = ya > 0 ? i - W : i;
        p = pp[i];
        p0 = lp[i];
        g0 = lg[i];
        pu = lp[iU];
        gu_ = lg[iU];
        wyu = wyp[iU];
        const float pU = pp[iU];
        n0 = p / denom;
        nU = ya > 0 ? pU / denom : 0.f;
    }
    const float gu = (float)x - cx, a = gu / (fx + kEps);   // (the lane's column is fixed)
    for (int y = ya; y < yb; ++y) {
        const int i = y * W + xc;
        const bool hL = xc > 0, hR = xc + 1 < W, hU = y > 0, hD = y + 1 < H;
        const int iL = hL ? i - 1 : i, iR = hR ? i + 1 : i, iD = hD ? i + W : i;
        const float pD = pp[iD], pE = pp[lane == 0 ? iL : iR];
        const float t = gt[o + i];
        const float wxi = wxp[i], wxl = wxp[iL], wyi = wyp[i];
        const float pl = lp[iL], pr = lp[iR], pd = lp[iD];
        const float gl = lg[iL], gr = lg[iR], gd = lg[iD];
        const bool valid = mask ? mask[o + i] != 0 : t > kEps;
        float gps[kScales];
#pragma unroll
        for (int s = 1; s < kScales; ++s) {
            const int r = y >> s, j = xc >> s;
            const bool in = r < g.Hs[s] && j < g.Ws[s];
            gps[s] = gP[g.off[s] + (in ? ((int64_t)b * g.Hs[s] + r) * g.Ws[s] + j : 0)];
            if (!in) gps[s] = 0.f;
        }
        const float nD = hD ? pD / denom : 0.f;
        float nL = __shfl_up(n0, 1), nR = __shfl_down(n0, 1);
        if (lane == 0 || lane == 63) {
            const float ev = pE / denom;
            if (lane == 0) nL = ev; else nR = ev;
        }
        if (xin) {
            // smoothness: forward sums and gn
            if (hR) v[0] += fabsf(nR - n0) * wxi;
            if (hD) v[1] += fabsf(nD - n0) * wyi;
            float sx = 0.f, sy = 0.f;
            if (hL) sx += sgnf(n0 - nL) * wxl;
            if (hR) sx -= sgnf(nR - n0) * wxi;
            if (hU) sy += sgnf(n0 - nU) * wyu;
            if (hD) sy -= sgnf(nD - n0) * wyi;
            const float gn = sx * c.inv_nx + sy * c.inv_ny;
            v[2] += (double)gn * p;
            // gradient matching at scale 0: sums and the sign terms of both neighbours
            float ax = 0.f, ay = 0.f;
            if (hL) ax += sgnf((p0 - pl) - (g0 - gl));
            if (hR) {
                const float dx = (pr - p0) - (gr - g0);
                v[3] += fabsf(dx);
                ax -= sgnf(dx);
            }
            if (hU) ay += sgnf((p0 - pu) - (g0 - gu_));
            if (hD) {
                const float dy = (pd - p0) - (gd - g0);
                v[4] += fabsf(dy);
                ay -= sgnf(dy);
            }
            // dL/dpred
            float grad = 0.f;
            if (valid && cnt > 0) {
                // SI
                const float d = p0 - g0;
                const float dd = 2.f * d * inv_n - sd_term;
                grad += w0 * (dd / clampf(p)) * clampgrad(p);
                // reprojection
                const float gv = (float)y - cy;
                const float bb = gv / (fy + kEps);
                const float dX = (gu * p) / (fx + kEps) - (gu * t) / (fx + kEps);
                const float dY = (gv * p) / (fy + kEps) - (gv * t) / (fy + kEps);
                const float dZ = p - t;
                const float e = sqrtf(dX * dX + dY * dY + dZ * dZ + kEps);
                grad += w3 * inv_n * (dX * a + dY * bb + dZ) / e;
            }
            float gg = (ax / nx0 + ay / ny0) * clampgrad(p) / clampf(p);
#pragma unroll
            for (int s = 1; s < kScales; ++s)
                if ((y >> s) < g.Hs[s] && (x >> s) < g.Ws[s]) gg += gps[s];
            grad += w1 * gg / (float)kScales;
            dpred[o + i] = grad + w2 * (gn / denom);
        }
        nU = n0;
        n0 = nD;
        pu = p0;
        gu_ = g0;
        wyu = wyi;
        p = pD;
        p0 = pd;
        g0 = gd;
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
        const bool hR = j + 1 < Ws, hD = r + 1 < g.Hs[s];
        const int64_t qR = hR ? q + 1 : q, qD = hD ? q + Ws : q;
        const float p0 = P[q], g0 = G[q], pr = P[qR], gr = G[qR], pd = P[qD], gd = G[qD];
        float ax = 0.f, ay = 0.f;
        if (hR) ax = fabsf((pr - p0) - (gr - g0));
        if (hD) ay = fabsf((pd - p0) - (gd - g0));
#pragma unroll
        for (int u = 1; u < kScales; ++u)
            if (u == s) { v[3 + 2 * u] += ax; v[4 + 2 * u] += ay; }
    }
    block_sum<kPB>(v, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < kPB; ++q) partB[((int64_t)b * nb + blockIdx.x) * kPB + q] = v[q];
}

// pass-B partials: block 0 the smoothness and gradient-matching sums and the five losses; blocks
// 1 + b * kc + k sample b's S_b (each of its kc blocks sums the same partials in the same order) and,
// when the smoothness weight is non-zero, the per-sample coupling dpred -= w2 S_b / (denom^2 HW) over
// chunk k of the sample
__global__ __launch_bounds__(kTPB) void k_lossR2(const double* partB, int nb, Geo g, double* dsc, float w0, float w1,
                                                 float w2, float w3, float* out5, int kc, float* __restrict__ dpred) {
    __shared__ double red[4 * (2 + 2 * kScales)];
    if (blockIdx.x > 0) {
        const int b = (blockIdx.x - 1) / kc, k = (blockIdx.x - 1) - b * kc;
        double u[1] = {0.0};
        for (int i = threadIdx.x; i < nb; i += kTPB) u[0] += partB[((int64_t)b * nb + i) * kPB + 2];
        block_sum<1>(u, red);
        if (threadIdx.x == 0) {
            if (k == 0) dsc[S_PB + g.B + b] = u[0];
            red[0] = u[0];
        }
        __syncthreads();
        if (w2 == 0.f) return;
        const int HW = g.H * g.W;
        const float mean = (float)(dsc[S_PB + b] / (double)HW);
        const float denom = mean + kEps;
        const float Sb = (float)red[0];
        const float cb = w2 * (Sb / (denom * denom * (float)HW));
        float* d = dpred + (int64_t)b * HW;
        for (int i = k * kTPB + threadIdx.x; i < HW; i += kc * kTPB) d[i] -= cb;
        return;
    }
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
// blocks per sample: ~2048 blocks in all, and at least one wave per 64-column group (pass B's walk)
int nb_per_sample(int B, int H, int W) {
    return std::max(cdiv(cdiv(W, 64), kTPB / 64), std::min(cdiv(2048, B), cdiv((int64_t)H * W, kTPB)));
}
}  // namespace

int64_t loss_workspace_floats(int B, int H, int W) {
    // pyramid (avgP, logP, logG, gP for scales 1..3), then scale-0 logs and edge weights (lp, lg, wx, wy)
    return 4 * make_geo(B, H, W).pyr_n + 4 * (int64_t)B * H * W + 64;
}
int64_t loss_part_doubles(int B, int H, int W) {
    const int nb = nb_per_sample(B, H, W);
    return (int64_t)B * nb * (kPA + kPB) + S_PB + 2 * B + 64;
}

void loss_fwd_bwd(const float* pred, const float* gt, const float* rgb, const float* K, const uint8_t* mask, int B,
                  int H, int W, const float w[4], float* out5, float* dpred, LossWorkspace ws, hipStream_t st) {
    if ((int64_t)B * H * W >= ((int64_t)1 << 31) || H < 2 || W < 2)
        throw std::runtime_error("loss: B*H*W must stay below 2^31 and H, W >= 2");
    Geo g = make_geo(B, H, W);
    const int64_t HW = (int64_t)H * W, n = (int64_t)B * HW;
    const int nb = nb_per_sample(B, H, W);
    double* dsc = ws.part;
    double* partA = dsc + S_PB + 2 * B + 16;
    double* partB = partA + (int64_t)B * nb * kPA;
    float* avgP = ws.pyr;
    float* logP = avgP + g.pyr_n;
    float* logG = logP + g.pyr_n;
    float* gP = logG + g.pyr_n;
    float* lp0 = gP + g.pyr_n;
    float* lg0 = lp0 + n;
    float* wx = lg0 + n;
    float* wy = wx + n;
    SmoothCtx c;
    c.inv_nx = 1.f / ((float)B * H * (W - 1));
    c.inv_ny = 1.f / ((float)B * (H - 1) * W);
    CAD_NO_ALIAS("loss_fwd_bwd", {aview(dpred, n, 1, 0, 1, 4, "dpred"), aview(ws.pyr, 1, 1, 0, 4 * g.pyr_n + 4 * n, 4, "workspace")},
                 {aview(pred, n, 1, 0, 1, 4, "pred"), aview(gt, n, 1, 0, 1, 4, "gt"), aview(rgb, 3 * n, 1, 0, 1, 4, "rgb"),
                  aview(mask, n, 1, 0, 1, 1, "mask")});

    hipLaunchKernelGGL(k_lossA, dim3(nb, B), dim3(kTPB), 0, st, pred, gt, rgb, K, mask, g, lp0, lg0, wx, wy, partA, nb);
    if (g.pyr_n > 0) {
        const int nby = cdiv(g.Hs[1], 4), nbx = cdiv(g.Ws[1], 4), tb = B * nby * nbx;
        hipLaunchKernelGGL(k_lossPyr, dim3(std::max(1, std::min(8192, cdiv(tb, 256)))), dim3(256), 0, st, pred, gt, g, nby,
                           nbx, tb, avgP, logP, logG);
        hipLaunchKernelGGL(k_lossPyrG, dim3(std::max(1, std::min(8192, cdiv(g.pyr_n, 256)))), dim3(256), 0, st, avgP, logP,
                           logG, g, gP);
    }
    hipLaunchKernelGGL(k_lossR1, dim3(B + 1), dim3(kTPB), 0, st, partA, nb, g, dsc);
    // pass B's walk: ncg 64-column groups x bands of rpb rows over the sample's nb * 4 waves
    const int ncg = cdiv(W, 64);
    const int rpb = cdiv(H, std::max(1, nb * (kTPB / 64) / ncg));
    if ((int64_t)cdiv(H, rpb) * ncg > (int64_t)nb * (kTPB / 64)) throw std::runtime_error("loss: pass-B walk does not cover the map");
    hipLaunchKernelGGL(k_lossB, dim3(nb, B), dim3(kTPB), 0, st, pred, gt, K, mask, lp0, lg0, wx, wy, logP, logG, gP, g,
                       dsc, w[0], w[1], w[2], w[3], c, dpred, partB, nb, ncg, rpb);
    const int kc = std::max(1, std::min(64, cdiv(HW, kTPB * 8)));
    hipLaunchKernelGGL(k_lossR2, dim3(1 + B * kc), dim3(kTPB), 0, st, partB, nb, g, dsc, w[0], w[1], w[2], w[3], out5, kc,
                       dpred);
}

}  // namespace cad
