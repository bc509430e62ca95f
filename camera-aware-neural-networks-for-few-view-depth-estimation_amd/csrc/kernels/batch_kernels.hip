// Batch assembly on device (SURVEY.md §8(a) a13 + §8(f) rank 2): decoded samples (u8 RGB, u16 depth,
// any size) -> the (B,3,H,W) rgb / (B,1,H,W) depth batch the step consumes, with the loader's resize
// and train-time augmentation, instead of per-sample LibTorch CPU ops and a host->device copy.
//
// Reference (src/data/sunrgbd_loader.cpp):
//   loadRGB :221-233      rgb = u8 / 255.0f (after cv::COLOR_BGR2RGB)
//   loadDepth :235-259    depth = u16 * (1/1000) (cv::Mat::convertTo CV_32F, single-precision scale)
//   getSample :158-166    resizeSample, then (train + augmentation) augmentSample and resizeSample again
//   resizeSample :445-489 rgb: interpolate bilinear, align_corners = false; depth: interpolate nearest
//   applyCrop :389-414    crop rows [cy, cy+ch), cols [cx, cx+cw) (torch Slice: clamped to the image)
//   applyHorizontalFlip :416-430, applyColorJitter :432-443  clamp(rgb * contrast + brightness - 1, 0, 1)
// ATen semantics restated (upsample_bilinear2d / upsample_nearest2d, CPU, fp32, output size given):
//   scale = (float)in / out; bilinear src = max(scale * (dst + 0.5f) - 0.5f, 0), i0 = min(floor(src),
//   in - 1), i1 = i0 + (i0 < in - 1), l1 = clamp(src - i0, 0, 1), l0 = 1 - l1,
//   out = (x00 l0w + x01 l1w) l0h + (x10 l0w + x11 l1w) l1h; nearest src = min(floor(dst * scale), in - 1).
// Intrinsics are updated on the host with the reference's own float operations (cad_api.cpp).
//
// Work: ~30 B of HBM traffic per output pixel (u8 gather + fp32 writes, plus one fp32 round trip for
// augmented samples): far below the step's cost, so one thread per output pixel and no tiling.
#include <algorithm>

#include "kernels.hpp"

namespace cad {
namespace {

struct Lin {   // one axis of a bilinear sample
    int i0, i1;
    float l0, l1;
};
__device__ __forceinline__ Lin lin_axis(int dst, int in, int out) {
    Lin r;
    if (in == out) {   // resizeSample returns early: exact copy
        r.i0 = r.i1 = dst;
        r.l0 = 1.f;
        r.l1 = 0.f;
        return r;
    }
    const float scale = (float)in / (float)out;
    float src = __fsub_rn(__fmul_rn(scale, (float)dst + 0.5f), 0.5f);
    if (src < 0.f) src = 0.f;
    r.i0 = min((int)floorf(src), in - 1);
    r.i1 = r.i0 + (r.i0 < in - 1 ? 1 : 0);
    r.l1 = fminf(fmaxf(src - (float)r.i0, 0.f), 1.f);
    r.l0 = 1.f - r.l1;
    return r;
}
__device__ __forceinline__ int nearest_axis(int dst, int in, int out) {
    if (in == out) return dst;
    const float scale = (float)in / (float)out;
    return min((int)floorf(__fmul_rn((float)dst, scale)), in - 1);
}
__device__ __forceinline__ float lerp2(float x00, float x01, float x10, float x11, const Lin& h, const Lin& w) {
    const float t0 = __fadd_rn(__fmul_rn(x00, w.l0), __fmul_rn(x01, w.l1));
    const float t1 = __fadd_rn(__fmul_rn(x10, w.l0), __fmul_rn(x11, w.l1));
    return __fadd_rn(__fmul_rn(t0, h.l0), __fmul_rn(t1, h.l1));
}
__device__ __forceinline__ float jitter(float v, const BatchSample& s) {
    if (!s.jitter) return v;
    const float t = __fsub_rn(__fadd_rn(__fmul_rn(v, s.contrast), s.brightness), 1.0f);
    return fminf(fmaxf(t, 0.f), 1.f);
}

// stage 1: decoded sample (h0 x w0, HWC u8 / HW u16) -> H x W planes (rgb [3][H][W], depth [H][W])
__global__ void k_batch_resize(const BatchSample* __restrict__ smp, int H, int W, float* __restrict__ rgb_out,
                               float* __restrict__ depth_out, float* __restrict__ rgb_tmp, float* __restrict__ depth_tmp) {
    const int b = blockIdx.y;
    const BatchSample& s = smp[b];
    const int64_t HW = (int64_t)H * W;
    float* rgb = s.aug ? rgb_tmp : rgb_out;
    float* dep = s.aug ? depth_tmp : depth_out;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
        const Lin ly = lin_axis(y, s.h0, H), lx = lin_axis(x, s.w0, W);
        const uint8_t* r0 = s.rgb + ((int64_t)ly.i0 * s.w0) * 3;
        const uint8_t* r1 = s.rgb + ((int64_t)ly.i1 * s.w0) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int cs = s.bgr ? 2 - c : c;
            const float x00 = (float)r0[lx.i0 * 3 + cs] / 255.0f, x01 = (float)r0[lx.i1 * 3 + cs] / 255.0f;
            const float x10 = (float)r1[lx.i0 * 3 + cs] / 255.0f, x11 = (float)r1[lx.i1 * 3 + cs] / 255.0f;
            rgb[((int64_t)b * 3 + c) * HW + p] = lerp2(x00, x01, x10, x11, ly, lx);
        }
        // depth has its own size (kv2: 512x424 depth under a 1920x1080 image); nearest from it
        const int ny = nearest_axis(y, s.dh0, H), nx = nearest_axis(x, s.dw0, W);
        dep[(int64_t)b * HW + p] = __fmul_rn((float)s.depth[(int64_t)ny * s.dw0 + nx], s.depth_scale);
    }
}

// stage 2 (augmented samples): crop [cy, cy+ch) x [cx, cx+cw) of the stage-1 image, optional
// horizontal flip, colour jitter, resize back to H x W
__global__ void k_batch_augment(const BatchSample* __restrict__ smp, int H, int W, const float* __restrict__ rgb_tmp,
                                const float* __restrict__ depth_tmp, float* __restrict__ rgb_out,
                                float* __restrict__ depth_out) {
    const int b = blockIdx.y;
    const BatchSample& s = smp[b];
    if (!s.aug) return;
    const int64_t HW = (int64_t)H * W;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
        const Lin ly = lin_axis(y, s.ch, H), lx = lin_axis(x, s.cw, W);
        // crop-image column j -> stage-1 column (flip mirrors inside the crop)
        auto col = [&](int j) { return s.cx + (s.flip ? s.cw - 1 - j : j); };
        const int64_t y0 = s.cy + ly.i0, y1 = s.cy + ly.i1;
        const int c0 = col(lx.i0), c1 = col(lx.i1);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float* src = rgb_tmp + ((int64_t)b * 3 + c) * HW;
            const float x00 = jitter(src[y0 * W + c0], s), x01 = jitter(src[y0 * W + c1], s);
            const float x10 = jitter(src[y1 * W + c0], s), x11 = jitter(src[y1 * W + c1], s);
            rgb_out[((int64_t)b * 3 + c) * HW + p] = lerp2(x00, x01, x10, x11, ly, lx);
        }
        const int ny = nearest_axis(y, s.ch, H), nx = nearest_axis(x, s.cw, W);
        depth_out[(int64_t)b * HW + p] = depth_tmp[(int64_t)b * HW + (int64_t)(s.cy + ny) * W + col(nx)];
    }
}

}  // namespace

void batch_assemble(const BatchSample* samples_dev, int B, int H, int W, bool any_aug, float* rgb, float* depth,
                    float* rgb_tmp, float* depth_tmp, hipStream_t st) {
    const int64_t HW = (int64_t)H * W;
    const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, (HW + 255) / 256)), (unsigned)B);
    hipLaunchKernelGGL(k_batch_resize, grid, dim3(256), 0, st, samples_dev, H, W, rgb, depth, rgb_tmp, depth_tmp);
    if (any_aug)
        hipLaunchKernelGGL(k_batch_augment, grid, dim3(256), 0, st, samples_dev, H, W, rgb_tmp, depth_tmp, rgb, depth);
}

}  // namespace cad
