// Four consecutive activations of an fp32 or bf16 row tensor as a float4 (the bf16 engine stores its
// pre-BN conv outputs as bf16: YB = true).  Element index e (multiple of 4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cad {
template <bool YB>
__device__ __forceinline__ float4 load4(const float* p, int64_t e) {
    if constexpr (YB) {
        const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p) + e);
        return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                           __uint_as_float(u.y & 0xffff0000u));
    } else {
        return *reinterpret_cast<const float4*>(p + e);
    }
}
}  // namespace cad
