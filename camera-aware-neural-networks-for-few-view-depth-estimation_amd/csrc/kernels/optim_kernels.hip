// Global-norm gradient clipping + Adam with coupled L2 weight decay over the flat parameter slab.
// Reference semantics:
//   clip_grad_norm_(params, max_norm) — LibTorch torch/nn/utils/clip_grad.h:22-85: total = ||g||_2
//     over all params, coef = min(1, max_norm / (total + 1e-6)), g *= coef (called at
//     tensorboard_trainer_enhanced.h:300-302).
//   torch::optim::Adam(AdamOptions(lr).weight_decay(wd)) — enhanced.h:97-101, step at :304:
//     g += wd*p; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
//     p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).
// Data-parallel: `prescale` (1/world) folds the gradient all-reduce mean into the same pass.
#include <algorithm>
#include <cmath>

#include "kernels.hpp"

namespace cad {
namespace {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
}

int sumsq_blocks(int64_t n) { return std::max(1, std::min(2048, cdiv(n, 256 * 16))); }

__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ g, int64_t n4, double* part) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 v = reinterpret_cast<const float4*>(g)[i];
        s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// norm_coef[0] = total norm of (prescale * g); norm_coef[1] = prescale * clamp(max/(total+1e-6), max=1)
__global__ __launch_bounds__(256) void k_clip_final(const double* part, int nb, float max_norm, float prescale,
                                                    float* norm_coef) {
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double tot = (red[0] + red[1] + red[2] + red[3]) * (double)prescale * (double)prescale;
        const float total = (float)sqrt(tot);
        const float coef = fminf(max_norm / (total + 1e-6f), 1.f);
        norm_coef[0] = total;
        norm_coef[1] = prescale * coef;
    }
}

void grad_norm_clip(const float* g, int64_t n, float max_norm, float prescale, double* scratch,
                    float* norm_coef, hipStream_t st) {
    const int nb = sumsq_blocks(n / 4);
    hipLaunchKernelGGL(k_sumsq, dim3(nb), dim3(256), 0, st, g, n / 4, scratch);
    hipLaunchKernelGGL(k_clip_final, dim3(1), dim3(256), 0, st, scratch, nb, max_norm, prescale, norm_coef);
}

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v, int64_t n4, const float* __restrict__ norm_coef,
                                              float lr_bc1, float b1, float b2, float eps, float wd, float sqrt_bc2) {
    const float coef = norm_coef[1];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 pv = reinterpret_cast<float4*>(p)[i];
        float4 gv = reinterpret_cast<float4*>(g)[i];
        float4 mv = reinterpret_cast<float4*>(m)[i];
        float4 vv = reinterpret_cast<float4*>(v)[i];
        float* pa = &pv.x; float* ga = &gv.x; float* ma = &mv.x; float* va = &vv.x;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float gc = ga[e] * coef;           // clip_grad_norm_: g.mul_(clip_coef_clamped)
            ga[e] = gc;
            const float gd = gc + wd * pa[e];        // grad.add(p, weight_decay)
            ma[e] = ma[e] * b1 + (1.f - b1) * gd;    // exp_avg.mul_(b1).add_(g, 1-b1)
            va[e] = va[e] * b2 + (1.f - b2) * gd * gd;
            const float denom = sqrtf(va[e]) / sqrt_bc2 + eps;
            pa[e] = pa[e] - lr_bc1 * (ma[e] / denom);
        }
        reinterpret_cast<float4*>(p)[i] = pv;
        reinterpret_cast<float4*>(g)[i] = gv;
        reinterpret_cast<float4*>(m)[i] = mv;
        reinterpret_cast<float4*>(v)[i] = vv;
    }
}

void adam_step(float* p, float* g, float* m, float* v, int64_t n, const float* norm_coef, float lr,
               float b1, float b2, float eps, float wd, int step, hipStream_t st) {
    const double bc1 = 1.0 - std::pow((double)b1, step);
    const double bc2 = 1.0 - std::pow((double)b2, step);
    const int64_t n4 = n / 4;
    const int nb = std::max(1, std::min(8192, cdiv(n4, 256)));
    hipLaunchKernelGGL(k_adam, dim3(nb), dim3(256), 0, st, p, g, m, v, n4, norm_coef, (float)(lr / bc1), b1, b2, eps,
                       wd, (float)std::sqrt(bc2));
}

}  // namespace cad
