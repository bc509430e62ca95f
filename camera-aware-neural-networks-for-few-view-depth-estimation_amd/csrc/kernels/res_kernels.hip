// Memory-bound kernels of the config-5 network (ResNet-50 encoder + U-Net decoder, resunet.cpp):
// im2col / col2im for the strided and 7x7 convolutions (their contractions run as dense GEMMs on the
// pre-split bf16 engine), MaxPool2d(3, 2, 1) with its gather backward, the bottleneck's
// BN + residual + ReLU join and its backward mask, strided row adds / subsampling for the 1x1
// stride-2 shortcut, and the transposed weight twins of the dgrad GEMMs.  NHWC; twins are bf16 rows
// (gemm_ps.hpp layout with one plane).  Every kernel writes each output element from one thread
// (no atomics): results are deterministic.
//
// Semantics follow torch (there is no reference model for config 5):
// MaxPool2d(3, 2, 1) takes the first maximum in window scan order (strict >), NaN propagates.
#include <algorithm>
#include <stdexcept>

#include "gemm_s3.hpp"   // split1 (fp32 -> bf16 round-to-nearest-even)
#include "ew_load.hpp"
#include "kernels.hpp"
#include "mx8_quant.hpp"

namespace cad {
namespace {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline int ew_blocks(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(n, 256)), 16384); }

__device__ __forceinline__ uint16_t bf16_bits(float x) {
    const __bf16 b = (__bf16)x;
    return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf16_val(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }
}  // namespace

// ------------------------------------------------------------------------------------------
// im2col: col[pix_out][k], k = (ky*KW + kx)*C + c (tap-major, channel inner), zero outside the
// image and for k >= KH*KW*C (the row is padded to Kp, a multiple of 8).  One thread per 8-k group.
// ------------------------------------------------------------------------------------------
template <class T>
__global__ void k_im2col(const T* __restrict__ x, int64_t ldx, int xcoff, int C, int B, int H, int W, int KH, int KW,
                         int S, int P, int Ho, int Wo, uint16_t* __restrict__ col, int Kp, int64_t n8) {
    const int G = Kp >> 3;
    const int KC = KH * KW * C;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t po = i / G;
        const int k0 = (int)(i - po * G) * 8;
        const int ox = (int)(po % Wo);
        const int64_t t = po / Wo;
        const int oy = (int)(t % Ho);
        const int b = (int)(t / Ho);
        uint16_t o[8];
        if (C % 8 == 0 && k0 < KC) {   // the 8 k of one tap: 8 consecutive channels
            const int tap = k0 / C, c = k0 - tap * C;
            const int iy = oy * S - P + tap / KW, ix = ox * S - P + tap % KW;
            if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
                const T* s = x + (((int64_t)b * H + iy) * W + ix) * ldx + xcoff + c;
                if constexpr (sizeof(T) == 2) {
                    *reinterpret_cast<uint4*>(col + po * Kp + k0) = *reinterpret_cast<const uint4*>(s);
                    continue;
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] = bf16_bits(s[e]);
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = 0;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = k0 + e;
                float v = 0.f;
                if (k < KC) {
                    const int tap = k / C, c = k - tap * C;
                    const int iy = oy * S - P + tap / KW, ix = ox * S - P + tap % KW;
                    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
                        const T xv = x[(((int64_t)b * H + iy) * W + ix) * ldx + xcoff + c];
                        if constexpr (sizeof(T) == 2) v = bf16_val(xv);
                        else v = xv;
                    }
                }
                o[e] = bf16_bits(v);
            }
        }
        uint4 pk;
        pk.x = o[0] | ((uint32_t)o[1] << 16);
        pk.y = o[2] | ((uint32_t)o[3] << 16);
        pk.z = o[4] | ((uint32_t)o[5] << 16);
        pk.w = o[6] | ((uint32_t)o[7] << 16);
        *reinterpret_cast<uint4*>(col + po * Kp + k0) = pk;
    }
}
// the 4-channel fp32 case (the stem's NHWC4 image): an 8-k group is two taps, each one 16-byte load;
// one thread per group, 32-bit index arithmetic (the 64-bit divisions of the general kernel made it
// ~4x slower than its 2-byte stores allow)
__global__ void k_im2col_c4(const float* __restrict__ x, int ldx, int xcoff, int H, int W, int KW, int taps, int S,
                            int P, int Ho, int Wo, uint16_t* __restrict__ col, int Kp, uint32_t n8) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n8) return;
    const uint32_t G = (uint32_t)Kp >> 3;
    const uint32_t po = i / G, g = i - po * G;
    const uint32_t ox = po % (uint32_t)Wo, t = po / (uint32_t)Wo;
    const uint32_t oy = t % (uint32_t)Ho, b = t / (uint32_t)Ho;
    uint32_t w[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int tap = 2 * (int)g + h;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tap < taps) {
            const int ky = tap / KW, kx = tap - ky * KW;
            const int iy = (int)oy * S - P + ky, ix = (int)ox * S - P + kx;
            if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                v = *reinterpret_cast<const float4*>(x + ((int64_t)((int)b * H + iy) * W + ix) * ldx + xcoff);
        }
        w[2 * h] = bf16_bits(v.x) | ((uint32_t)bf16_bits(v.y) << 16);
        w[2 * h + 1] = bf16_bits(v.z) | ((uint32_t)bf16_bits(v.w) << 16);
    }
    *reinterpret_cast<uint4*>(col + (int64_t)po * Kp + g * 8) = make_uint4(w[0], w[1], w[2], w[3]);
}

void im2col_f32(const float* x, int64_t ldx, int xcoff, int C, int B, int H, int W, int KH, int KW, int S, int P,
                void* col, int Kp, hipStream_t st) {
    const int Ho = (H + 2 * P - KH) / S + 1, Wo = (W + 2 * P - KW) / S + 1;
    if (Kp % 8 || Kp < KH * KW * C) throw std::runtime_error("im2col: row padding");
    const int64_t n8 = (int64_t)B * Ho * Wo * (Kp / 8);
    if (C == 4 && ldx % 4 == 0 && xcoff % 4 == 0 && n8 < ((int64_t)1 << 31) && ldx < ((int64_t)1 << 31)) {
        hipLaunchKernelGGL(k_im2col_c4, dim3(cdiv(n8, 256)), dim3(256), 0, st, x, (int)ldx, xcoff, H, W, KW, KH * KW, S, P,
                           Ho, Wo, (uint16_t*)col, Kp, (uint32_t)n8);
        return;
    }
    hipLaunchKernelGGL(k_im2col<float>, dim3(ew_blocks(n8)), dim3(256), 0, st, x, ldx, xcoff, C, B, H, W, KH, KW, S, P,
                       Ho, Wo, (uint16_t*)col, Kp, n8);
}
void im2col_ps(Split x, int C, int B, int H, int W, int KH, int KW, int S, int P, void* col, int Kp, hipStream_t st) {
    const int Ho = (H + 2 * P - KH) / S + 1, Wo = (W + 2 * P - KW) / S + 1;
    if (Kp % 8 || Kp < KH * KW * C || x.ld % 8 || x.coff % 8) throw std::runtime_error("im2col: alignment");
    const int64_t n8 = (int64_t)B * Ho * Wo * (Kp / 8);
    hipLaunchKernelGGL(k_im2col<uint16_t>, dim3(ew_blocks(n8)), dim3(256), 0, st, (const uint16_t*)x.p, x.ld, x.coff,
                       C, B, H, W, KH, KW, S, P, Ho, Wo, (uint16_t*)col, Kp, n8);
}

// col2im (gather): dx[pix_in][c] = sum over the taps that read pix_in of dcol[pix_out][tap*C + c],
// in tap order; overwrites dx (ld lddx).  One thread per (input pixel, 4 channels); C % 4 == 0.
__global__ void k_col2im(const float* __restrict__ dcol, int Kc, int C, int B, int H, int W, int KH, int KW, int S,
                         int P, int Ho, int Wo, float* __restrict__ dx, int64_t lddx, int64_t n4) {
    const int C4 = C >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C4;
        const int c = (int)(i - p * C4) * 4;
        const int ix = (int)(p % W);
        const int64_t t = p / W;
        const int iy = (int)(t % H);
        const int b = (int)(t / H);
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int ky = 0; ky < KH; ++ky) {
            const int ny = iy + P - ky;
            if (ny < 0 || ny % S) continue;
            const int oy = ny / S;
            if (oy >= Ho) continue;
            for (int kx = 0; kx < KW; ++kx) {
                const int nx = ix + P - kx;
                if (nx < 0 || nx % S) continue;
                const int ox = nx / S;
                if (ox >= Wo) continue;
                const float4 v = *reinterpret_cast<const float4*>(
                    dcol + (((int64_t)b * Ho + oy) * Wo + ox) * Kc + (ky * KW + kx) * C + c);
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
        }
        *reinterpret_cast<float4*>(dx + p * lddx + c) = s;
    }
}
void col2im(const float* dcol, int Kc, int C, int B, int H, int W, int KH, int KW, int S, int P, float* dx,
            int64_t lddx, hipStream_t st) {
    const int Ho = (H + 2 * P - KH) / S + 1, Wo = (W + 2 * P - KW) / S + 1;
    if (C % 4 || Kc % 4 || lddx % 4) throw std::runtime_error("col2im: alignment");
    const int64_t n4 = (int64_t)B * H * W * C / 4;
    CAD_NO_ALIAS("col2im", {aview(dx, (int64_t)B * H * W, lddx, 0, C, 4, "dx")},
                 {aview(dcol, (int64_t)B * Ho * Wo, Kc, 0, Kc, 4, "dcol")});
    hipLaunchKernelGGL(k_col2im, dim3(ew_blocks(n4)), dim3(256), 0, st, dcol, Kc, C, B, H, W, KH, KW, S, P, Ho, Wo, dx,
                       lddx, n4);
}

// ------------------------------------------------------------------------------------------
// MaxPool2d(3, stride 2, padding 1): argmax code ky*3 + kx per output element (uint8)
// ------------------------------------------------------------------------------------------
__global__ void k_maxpool3s2_fwd(const float* __restrict__ x, int C, int B, int H, int W, int Ho, int Wo,
                                 float* __restrict__ out, uint8_t* __restrict__ idx, uint16_t* __restrict__ os,
                                 int64_t n4) {
    const int C4 = C >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t op = i / C4;
        const int c = (int)(i - op * C4) * 4;
        const int ox = (int)(op % Wo);
        const int64_t t = op / Wo;
        const int oy = (int)(t % Ho);
        const int b = (int)(t / Ho);
        float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        uint8_t arg[4] = {255, 255, 255, 255};
        for (int ky = 0; ky < 3; ++ky) {
            const int iy = 2 * oy - 1 + ky;
            if ((unsigned)iy >= (unsigned)H) continue;
            for (int kx = 0; kx < 3; ++kx) {
                const int ix = 2 * ox - 1 + kx;
                if ((unsigned)ix >= (unsigned)W) continue;
                const float4 v = *reinterpret_cast<const float4*>(x + (((int64_t)b * H + iy) * W + ix) * C + c);
                const float va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (arg[e] == 255 || va[e] > best[e] || isnan(va[e])) {   // torch: (val > max) || isnan(val)
                        best[e] = va[e];
                        arg[e] = (uint8_t)(ky * 3 + kx);
                    }
            }
        }
        const float4 o = make_float4(best[0], best[1], best[2], best[3]);
        if (out) *reinterpret_cast<float4*>(out + op * C + c) = o;
        if (os) *reinterpret_cast<uint2*>(os + op * C + c) = split1(o).p[0];
        *reinterpret_cast<uchar4*>(idx + op * C + c) = make_uchar4(arg[0], arg[1], arg[2], arg[3]);
    }
}
void maxpool3s2_fwd(const float* x, int C, int B, int H, int W, float* out, uint8_t* idx, void* out_split,
                    hipStream_t st) {
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const int64_t n4 = (int64_t)B * Ho * Wo * C / 4;
    hipLaunchKernelGGL(k_maxpool3s2_fwd, dim3(ew_blocks(n4)), dim3(256), 0, st, x, C, B, H, W, Ho, Wo, out, idx,
                       (uint16_t*)out_split, n4);
}
// gather: dx[(b,iy,ix)][c] = sum over the (<= 4) windows holding (iy,ix) whose argmax is it, in
// window order; overwrites dx
// (I: the index type — 32-bit when the element count allows: the 64-bit divisions of the position
// decode cost more than the kernel's memory traffic)
template <class I>
__global__ void k_maxpool3s2_bwd(const float* __restrict__ dout, const uint8_t* __restrict__ idx, int C, int B, int H,
                                 int W, int Ho, int Wo, float* __restrict__ dx, int64_t n4, const float* __restrict__ add,
                                 int64_t ldadd) {
    const I C4 = (I)(C >> 2);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const I p = (I)i / C4;
        const int c = (int)((I)i - p * C4) * 4;
        const int ix = (int)(p % (I)W);
        const I t = p / (I)W;
        const int iy = (int)(t % (I)H);
        const int b = (int)(t / (I)H);
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        for (int oy = iy / 2; oy <= (iy + 1) / 2 && oy < Ho; ++oy) {
            const int ky = iy - 2 * oy + 1;
            if (ky < 0 || ky > 2) continue;
            for (int ox = ix / 2; ox <= (ix + 1) / 2 && ox < Wo; ++ox) {
                const int kx = ix - 2 * ox + 1;
                if (kx < 0 || kx > 2) continue;
                const int code = ky * 3 + kx;
                const int64_t op = ((int64_t)b * Ho + oy) * Wo + ox;
                const uchar4 a = *reinterpret_cast<const uchar4*>(idx + op * C + c);
                if (a.x != code && a.y != code && a.z != code && a.w != code) continue;
                const float4 d = *reinterpret_cast<const float4*>(dout + op * C + c);
                if (a.x == code) s[0] += d.x;
                if (a.y == code) s[1] += d.y;
                if (a.z == code) s[2] += d.z;
                if (a.w == code) s[3] += d.w;
            }
        }
        if (add) {   // (the separate add pass's single add, in the same order)
            const float4 q = *reinterpret_cast<const float4*>(add + (int64_t)p * ldadd + c);
            s[0] += q.x; s[1] += q.y; s[2] += q.z; s[3] += q.w;
        }
        *reinterpret_cast<float4*>(dx + (int64_t)p * C + c) = make_float4(s[0], s[1], s[2], s[3]);
    }
}
void maxpool3s2_bwd(const float* dout, const uint8_t* idx, int C, int B, int H, int W, float* dx, hipStream_t st,
                    const float* add, int64_t ldadd) {
    if (add && (ldadd < C || ldadd % 4)) throw std::runtime_error("maxpool3s2_bwd: added matrix layout");
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const int64_t n4 = (int64_t)B * H * W * C / 4;
    CAD_NO_ALIAS("maxpool3s2_bwd", {aview(dx, (int64_t)B * H * W, C, 0, C, 4, "dx")},
                 {aview(dout, (int64_t)B * Ho * Wo, C, 0, C, 4, "dout"), aview(idx, (int64_t)B * Ho * Wo, C, 0, C, 1, "argmax"),
                  aview(add, (int64_t)B * H * W, ldadd, 0, C, 4, "add")});
    if (n4 < ((int64_t)1 << 31))
        hipLaunchKernelGGL(k_maxpool3s2_bwd<uint32_t>, dim3(cdiv(n4, 256)), dim3(256), 0, st, dout, idx, C, B, H, W, Ho, Wo,
                           dx, n4, add, ldadd);
    else
        hipLaunchKernelGGL(k_maxpool3s2_bwd<int64_t>, dim3(ew_blocks(n4)), dim3(256), 0, st, dout, idx, C, B, H, W, Ho, Wo,
                           dx, n4, add, ldadd);
}

// ------------------------------------------------------------------------------------------
// bottleneck join: out = relu(y*s + t + r), r = yd*sd + td (projection shortcut) or x (identity,
// row stride ldx); out fp32 dense [M][C] and its bf16 twin
// ------------------------------------------------------------------------------------------
// QX: also the MX-fp8 copy of the twin's values (q / qs, ldq bytes per row; the next block's first
// contraction reads it instead of quantising the twin again); needs C % 32 == 0: the 8 lanes of a
// 32-channel block are consecutive and group-aligned in this grid-stride walk
template <bool YB, bool QX = false>
__global__ void k_bn_add_relu(const float* __restrict__ y, const float* __restrict__ s, const float* __restrict__ t,
                              const float* __restrict__ yd, const float* __restrict__ sd, const float* __restrict__ td,
                              const float* __restrict__ x, int64_t ldx, int C, float* __restrict__ out,
                              uint16_t* __restrict__ os, int64_t n4, uint8_t* __restrict__ mq = nullptr,
                              uint8_t* __restrict__ ms = nullptr, int64_t ldq = 0) {
    const int C4 = C >> 2;
#pragma unroll 4
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / C4;
        const int c = (int)(i - r * C4) * 4;
        const float4 v = load4<YB>(y, i * 4);
        const float4 a = *reinterpret_cast<const float4*>(s + c), b = *reinterpret_cast<const float4*>(t + c);
        float4 q;
        if (yd) {
            const float4 w = load4<YB>(yd, i * 4);
            const float4 e = *reinterpret_cast<const float4*>(sd + c), f = *reinterpret_cast<const float4*>(td + c);
            q = make_float4(w.x * e.x + f.x, w.y * e.y + f.y, w.z * e.z + f.z, w.w * e.w + f.w);
        } else {
            q = *reinterpret_cast<const float4*>(x + r * ldx + c);
        }
        const float4 o = make_float4(fmaxf(v.x * a.x + b.x + q.x, 0.f), fmaxf(v.y * a.y + b.y + q.y, 0.f),
                                     fmaxf(v.z * a.z + b.z + q.z, 0.f), fmaxf(v.w * a.w + b.w + q.w, 0.f));
        *reinterpret_cast<float4*>(out + i * 4) = o;
        const uint2 tw = split1(o).p[0];
        if (os) *reinterpret_cast<uint2*>(os + i * 4) = tw;
        if constexpr (QX)
            mx8_store_group(make_float4(__uint_as_float(tw.x << 16), __uint_as_float(tw.x & 0xFFFF0000u),
                                        __uint_as_float(tw.y << 16), __uint_as_float(tw.y & 0xFFFF0000u)),
                            mq, ms, ldq, r, c);
    }
}
void bn_add_relu(const float* y, const float* scale, const float* shift, const float* yd, const float* dscale,
                 const float* dshift, const float* x, int64_t ldx, int C, int64_t M, float* out, void* out_split,
                 hipStream_t st, bool y_bf16, const Mx8* qx) {
    const int64_t n4 = M * C / 4;
    CAD_NO_ALIAS("bn_add_relu", {aview(out, M, C, 0, C, 4, "out"), aview(out_split, M, C, 0, C, 2, "out twin")},
                 {aview(y, M, C, 0, C, y_bf16 ? 2 : 4, "y"), aview(yd, M, C, 0, C, y_bf16 ? 2 : 4, "projection y"),
                  aview(yd ? nullptr : x, M, ldx, 0, C, 4, "shortcut x")}, true);
    if (qx) {
        if (C % 32 || qx->ld % 128 || qx->coff || !qx->q || !qx->s) throw std::runtime_error("bn_add_relu: MX-fp8 copy layout");
        auto* q = static_cast<uint8_t*>(const_cast<void*>(qx->q));
        auto* qs = static_cast<uint8_t*>(const_cast<void*>(qx->s));
        if (y_bf16)
            hipLaunchKernelGGL((k_bn_add_relu<true, true>), dim3(ew_blocks(n4)), dim3(256), 0, st, y, scale, shift, yd, dscale,
                               dshift, x, ldx, C, out, (uint16_t*)out_split, n4, q, qs, qx->ld);
        else
            hipLaunchKernelGGL((k_bn_add_relu<false, true>), dim3(ew_blocks(n4)), dim3(256), 0, st, y, scale, shift, yd,
                               dscale, dshift, x, ldx, C, out, (uint16_t*)out_split, n4, q, qs, qx->ld);
        return;
    }
    if (y_bf16)
        hipLaunchKernelGGL(k_bn_add_relu<true>, dim3(ew_blocks(n4)), dim3(256), 0, st, y, scale, shift, yd, dscale, dshift,
                           x, ldx, C, out, (uint16_t*)out_split, n4);
    else
        hipLaunchKernelGGL(k_bn_add_relu<false>, dim3(ew_blocks(n4)), dim3(256), 0, st, y, scale, shift, yd, dscale, dshift,
                           x, ldx, C, out, (uint16_t*)out_split, n4);
}
// gs = g * [out > 0]  (g rows ldg at channel offset gcoff; out and gs dense [M][C])
__global__ void k_relu_mask(const float* __restrict__ g, int64_t ldg, int gcoff, const float* __restrict__ out, int C,
                            float* __restrict__ gs, int64_t n4) {
    const int C4 = C >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / C4;
        const int c = (int)(i - r * C4) * 4;
        const float4 v = *reinterpret_cast<const float4*>(g + r * ldg + gcoff + c);
        const float4 o = *reinterpret_cast<const float4*>(out + i * 4);
        *reinterpret_cast<float4*>(gs + i * 4) =
            make_float4(o.x > 0.f ? v.x : 0.f, o.y > 0.f ? v.y : 0.f, o.z > 0.f ? v.z : 0.f, o.w > 0.f ? v.w : 0.f);
    }
}
void relu_mask(const float* g, int64_t ldg, int gcoff, const float* out, int C, int64_t M, float* gs, hipStream_t st) {
    const int64_t n4 = M * C / 4;
    CAD_NO_ALIAS("relu_mask", {aview(gs, M, C, 0, C, 4, "gs")},
                 {aview(g, M, ldg, gcoff, C, 4, "g"), aview(out, M, C, 0, C, 4, "out")}, true);
    hipLaunchKernelGGL(k_relu_mask, dim3(ew_blocks(n4)), dim3(256), 0, st, g, ldg, gcoff, out, C, gs, n4);
}

__global__ void k_mask_inplace(float* y, int64_t ldy, int ycoff, const float* mask, int C, int64_t n4) {
    const int C4 = C >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / C4;
        const int64_t o = r * ldy + ycoff + (i - r * C4) * 4;
        const float4 m = *reinterpret_cast<const float4*>(mask + o);
        float4 v = *reinterpret_cast<const float4*>(y + o);
        v = make_float4(m.x > 0.f ? v.x : 0.f, m.y > 0.f ? v.y : 0.f, m.z > 0.f ? v.z : 0.f, m.w > 0.f ? v.w : 0.f);
        *reinterpret_cast<float4*>(y + o) = v;
    }
}
void mask_inplace(float* y, int64_t ldy, int ycoff, const float* mask, int C, int64_t M, hipStream_t st) {
    if (C % 4 || ldy % 4 || ycoff % 4) throw std::runtime_error("mask_inplace: alignment");
    CAD_NO_ALIAS("mask_inplace", {aview(y, M, ldy, ycoff, C, 4, "y (in place)")}, {aview(mask, M, ldy, ycoff, C, 4, "mask")});
    const int64_t n4 = M * C / 4;
    hipLaunchKernelGGL(k_mask_inplace, dim3(ew_blocks(n4)), dim3(256), 0, st, y, ldy, ycoff, mask, C, n4);
}

// dst[(b, S*oy, S*ox)][c] += src[(b, oy, ox)][scoff + c] for the Ho x Wo grid of src (S = 1 or 2);
// dst rows of ld lddst over a B x H x W grid
__global__ void k_add_strided(float* __restrict__ dst, int64_t lddst, const float* __restrict__ src, int64_t ldsrc,
                              int scoff, int C, int H, int W, int Ho, int Wo, int S, int64_t n4) {
    const int C4 = C >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t op = i / C4;
        const int c = (int)(i - op * C4) * 4;
        const int ox = (int)(op % Wo);
        const int64_t t = op / Wo;
        const int oy = (int)(t % Ho);
        const int b = (int)(t / Ho);
        float* q = dst + (((int64_t)b * H + S * oy) * W + S * ox) * lddst + c;
        const float4 v = *reinterpret_cast<const float4*>(src + op * ldsrc + scoff + c);
        float4 d = *reinterpret_cast<float4*>(q);
        d.x += v.x; d.y += v.y; d.z += v.z; d.w += v.w;
        *reinterpret_cast<float4*>(q) = d;
    }
}
void add_strided(float* dst, int64_t lddst, const float* src, int64_t ldsrc, int scoff, int C, int B, int H, int W,
                 int S, hipStream_t st) {
    const int Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
    const int64_t n4 = (int64_t)B * Ho * Wo * C / 4;
    // dst is accumulated in place (declared); src must be another buffer
    CAD_NO_ALIAS("add_strided", {aview(dst, (int64_t)B * H * W, lddst, 0, C, 4, "dst")},
                 {aview(src, (int64_t)B * Ho * Wo, ldsrc, scoff, C, 4, "src")});
    hipLaunchKernelGGL(k_add_strided, dim3(ew_blocks(n4)), dim3(256), 0, st, dst, lddst, src, ldsrc, scoff, C, H, W,
                       Ho, Wo, S, n4);
}

// bf16 twin rows: dst[(b,oy,ox)][dcoff + c] = src[(b, S*oy, S*ox)][scoff + c] (16-B pieces; C % 8 == 0)
__global__ void k_copy_twin(const uint16_t* __restrict__ src, int64_t lds, int scoff, uint16_t* __restrict__ dst,
                            int64_t ldd, int dcoff, int C, int H, int W, int Ho, int Wo, int S, int64_t n8) {
    const int G = C >> 3;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t op = i / G;
        const int c = (int)(i - op * G) * 8;
        const int ox = (int)(op % Wo);
        const int64_t t = op / Wo;
        const int oy = (int)(t % Ho);
        const int b = (int)(t / Ho);
        const int64_t ip = ((int64_t)b * H + S * oy) * W + S * ox;
        *reinterpret_cast<uint4*>(dst + op * ldd + dcoff + c) = *reinterpret_cast<const uint4*>(src + ip * lds + scoff + c);
    }
}
void copy_twin(Split src, int C, int B, int H, int W, int S, void* dst, int64_t ldd, int dcoff, hipStream_t st) {
    if (C % 8 || src.ld % 8 || src.coff % 8 || ldd % 8 || dcoff % 8) throw std::runtime_error("copy_twin: alignment");
    const int Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
    const int64_t n8 = (int64_t)B * Ho * Wo * C / 8;
    CAD_NO_ALIAS("copy_twin", {aview(dst, (int64_t)B * Ho * Wo, ldd, dcoff, C, 2, "dst")},
                 {aview(src.p, (int64_t)B * H * W, src.ld, src.coff, C, 2, "src")});
    hipLaunchKernelGGL(k_copy_twin, dim3(ew_blocks(n8)), dim3(256), 0, st, (const uint16_t*)src.p, src.ld, src.coff,
                       (uint16_t*)dst, ldd, dcoff, C, H, W, Ho, Wo, S, n8);
}

// wt[k][n] (bf16, rows of N) = w[n][k] (fp32, rows of ldw), n < N, k < K
__global__ void k_transpose_split(const float* __restrict__ w, int64_t ldw, int N, int K, uint16_t* __restrict__ wt) {
    __shared__ float tile[32][33];
    const int n0 = blockIdx.y * 32, k0 = blockIdx.x * 32;
    for (int r = threadIdx.y; r < 32; r += blockDim.y) {
        const int n = n0 + r, k = k0 + threadIdx.x;
        tile[r][threadIdx.x] = (n < N && k < K) ? w[(int64_t)n * ldw + k] : 0.f;
    }
    __syncthreads();
    for (int r = threadIdx.y; r < 32; r += blockDim.y) {
        const int k = k0 + r, n = n0 + threadIdx.x;
        if (k < K && n < N) wt[(int64_t)k * N + n] = bf16_bits(tile[threadIdx.x][r]);
    }
}
void transpose_split(const float* w, int64_t ldw, int N, int K, void* wt, hipStream_t st) {
    hipLaunchKernelGGL(k_transpose_split, dim3(cdiv(K, 32), cdiv(N, 32)), dim3(32, 8), 0, st, w, ldw, N, K,
                       (uint16_t*)wt);
}

}  // namespace cad
