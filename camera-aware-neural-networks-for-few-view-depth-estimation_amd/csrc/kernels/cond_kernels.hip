// Per-pixel ray directions from camera intrinsics, computed on device
// instead of the reference's offline .bin files.
// Reference: RayDirectionComputer::computeRayDirections
//   (src/preprocessing/ray_direction_computer.cpp:17-62): fx_inv = 1/fx, fy_inv = 1/fy,
//   x = (u - cx) * fx_inv, y = (v - cy) * fy_inv, r = (x, y, 1) / sqrt(x^2 + y^2 + 1).
// Output layout: NCHW (B, 3, H, W), the (3,H,W) reshape the loader applies
// (sunrgbd_loader.cpp:346-347).
#include <algorithm>

#include "kernels.hpp"

namespace cad {

__global__ void k_rays(const float* __restrict__ K, int B, int H, int W, float* __restrict__ rays) {
    const int64_t HW = (int64_t)H * W, n = (int64_t)B * HW;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / HW);
        const int64_t p = i - b * HW;
        const int u = (int)(p % W), v = (int)(p / W);
        const float* k = K + b * 9;
        const float fx_inv = 1.0f / k[0], fy_inv = 1.0f / k[4];
        const float x = ((float)u - k[2]) * fx_inv;
        const float y = ((float)v - k[5]) * fy_inv;
        const float z = 1.0f;
        // (x*x + y*y) + 1 with one rounding per operation, as the fp32 reference evaluates it (no FMA
        // contraction: a contracted norm moves a ray by an fp32 ulp, which flips its bf16 rounding)
        const float nrm = sqrtf(__fadd_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)), z));
        float* o = rays + (int64_t)b * 3 * HW + p;
        o[0] = x / nrm;
        o[HW] = y / nrm;
        o[2 * HW] = z / nrm;
    }
}

void ray_directions(const float* K, int B, int H, int W, float* rays_nchw, hipStream_t st) {
    const int64_t n = (int64_t)B * H * W;
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256));
    hipLaunchKernelGGL(k_rays, dim3(nb), dim3(256), 0, st, K, B, H, W, rays_nchw);
}

}  // namespace cad
