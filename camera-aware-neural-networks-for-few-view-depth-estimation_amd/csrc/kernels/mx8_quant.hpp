// MX-fp8 (OCP MX, E4M3 elements, one E8M0 scale per 32 elements) element quantisation shared by the
// quantiser kernel (mx8_kernels.hip), the GEMM operand loaders (gemm_mx8.hpp) and the BN-apply
// passes that write a pre-quantised copy of their output (nn_kernels.hip, res_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cad {

constexpr float kE4M3Max = 448.f;

// shared exponent of a block with max |v| = amax (MX spec: floor(log2 amax) - emax_elem)
__device__ __forceinline__ int mx8_shared_exp(float amax) {
    const int e = (int)((__float_as_uint(amax) >> 23) & 0xFF) - 127;   // zero / subnormal: -127
    const int s = e - 8;
    return s < -127 ? -127 : (s > 127 ? 127 : s);
}
// 2^-shared as an fp32 (shared in [-127, 126] is all this is called with: amax < 2^128)
__device__ __forceinline__ float mx8_inv_scale(int shared) { return __uint_as_float((uint32_t)(127 - shared) << 23); }

// four values (already multiplied by 2^-shared) -> four e4m3 bytes (round to nearest even, saturated)
__device__ __forceinline__ uint32_t mx8_pack4(float a, float b, float c, float d) {
    auto sat = [](float x) { return fminf(fmaxf(x, -kE4M3Max), kE4M3Max); };
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a), sat(b), 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c), sat(d), w, true);
    return (uint32_t)w;
}

// the MX block of 32 channels held by 8 consecutive, group-aligned lanes (4 channels each; every lane
// of the group active): amax over the group, then each lane's four E4M3 bytes, lane c % 32 == 0 the
// scale byte — the bytes k_mx8_quantize writes for the same 32 values (a max is order-independent)
__device__ __forceinline__ void mx8_store_group(float4 v, uint8_t* __restrict__ q, uint8_t* __restrict__ s, int64_t ldq,
                                                int64_t r, int c) {
    float amax = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    amax = fmaxf(amax, __shfl_xor(amax, 1));
    amax = fmaxf(amax, __shfl_xor(amax, 2));
    amax = fmaxf(amax, __shfl_xor(amax, 4));
    const int sh = mx8_shared_exp(amax);
    const float inv = mx8_inv_scale(sh < 127 ? sh : 126);
    *reinterpret_cast<uint32_t*>(q + r * ldq + c) = mx8_pack4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
    if ((c & 31) == 0) s[r * (ldq >> 5) + (c >> 5)] = (uint8_t)(sh + 127);
}

}  // namespace cad
