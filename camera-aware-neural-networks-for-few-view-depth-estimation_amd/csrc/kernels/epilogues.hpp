// GEMM epilogue functors shared by the conv / dense kernel families (conv_kernels.hip,
// mx8_kernels.hip): what gemm_epilogue_t / win_epilogue do with a finished accumulator tile.
#pragma once
#include "gemm_mfma.hpp"

namespace cad {

// Row-major epilogues: C[m][c_coff + n] with row stride ldc; the engine stores through a buffer
// descriptor based at row_base (gemm_mfma.hpp gemm_epilogue).
struct EpiStore {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;
    static constexpr bool ADD = false;
    static constexpr bool SPLIT = false;
    __device__ static const float* row_base(const GemmArgs& a, int m0, int) {
        return a.C + (int64_t)m0 * a.ldc + a.c_coff;
    }
};
struct EpiStoreStats : EpiStore {
    static constexpr bool STATS = true;
};
// C[m][n] = acc + R[m][n], R = a.bias read as a matrix with C's row stride and channel offset (the
// config-5 bottleneck's identity shortcut gradient added in the dgrad that produces the block-input
// gradient: no separate add pass)
struct EpiStoreAdd : EpiStore {
    static constexpr bool ADD = true;
    __device__ static const float* add_base(const GemmArgs& a, int m0) {
        return a.bias + (int64_t)m0 * a.ldc + a.c_coff;
    }
};
// bf16 outputs (round-to-nearest-even; a.C addresses bf16 rows of ldc elements): the pre-BN conv
// outputs of the bf16 engine.  BN partials are taken from the rounded values BN normalises.
struct EpiStoreB16 {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = true;
    static constexpr bool ADD = false;
    static constexpr bool SPLIT = false;
    __device__ static const float* row_base(const GemmArgs& a, int m0, int) {
        return reinterpret_cast<const float*>(reinterpret_cast<const char*>(a.C) + ((int64_t)m0 * a.ldc + a.c_coff) * 2);
    }
};
struct EpiStoreStatsB16 : EpiStoreB16 {
    static constexpr bool STATS = true;
};
// window epilogue only: columns [0, split_n) fp32 into C, [split_n, N) bf16 into C2 (the decoder conv1
// dgrad writes dcat's skip half for the encoder's BN backward and the up half straight into the twin
// the ConvT gradients read)
struct EpiStoreSplitB16 : EpiStore {
    static constexpr bool SPLIT = true;
};
// ... with the lower columns also bf16 (C: bf16 rows of ldc elements)
struct EpiStoreSplit2B16 : EpiStoreB16 {
    static constexpr bool SPLIT = true;
};
// ConvTranspose2d(k2,s2) pixel shuffle: n = (q=(dy,dx), co) -> high-res pixel (2y+dy, 2x+dx).
// The column (q, co) is fixed per lane and sub-block, and rows advance in small steps, so the
// epilogue carries (x, y, b) incrementally instead of dividing per element (STRUCTURED epilogue).
struct EpiConvT {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;
    static constexpr bool ADD = false;
    static constexpr bool STRUCTURED = true;
    __device__ void operator()(const GemmArgs& a, int m, int n, float v, int) const {
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const int x = m % a.W, t = m / a.W, y = t % a.H, b = t / a.H;
        const int64_t hp = ((int64_t)b * (2 * a.H) + 2 * y + (q >> 1)) * (2 * a.W) + 2 * x + (q & 1);
        a.C[hp * a.ldc + a.c_coff + co] = v + a.bias[co];
    }
    // one lane's 16 accumulator rows of a 32x32 sub-block: rows mbase + (r&3) + 8(r>>2), column n
    __device__ void block(const GemmArgs& a, int mbase, int n, const floatx16& acc) const {
        if (n >= a.N) return;
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const float bias = a.bias[co];
        float* dst = a.C + a.c_coff + co;
        const int64_t W2 = 2 * a.W;
        int x = mbase % a.W, t = mbase / a.W, y = t % a.H, b = t / a.H;
        int cur = 0;   // row offset that (x, y, b) currently describe
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int off = (r & 3) + 8 * (r >> 2);
            x += off - cur;
            cur = off;
            while (x >= a.W) { x -= a.W; if (++y == a.H) { y = 0; ++b; } }
            if (mbase + off < a.M) {
                const int64_t hp = ((int64_t)b * (2 * a.H) + 2 * y + (q >> 1)) * W2 + 2 * x + (q & 1);
                dst[hp * a.ldc] = acc[r] + bias;
            }
        }
    }
};
// EpiConvT writing bf16 (a.C addresses bf16 rows of ldc elements): the bf16 engine's up half of
// the decoder concat, written straight into the consumers' twin
struct EpiConvTB16 {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;   // (row-major store path unused: structured)
    static constexpr bool ADD = false;
    static constexpr bool STRUCTURED = true;
    __device__ void operator()(const GemmArgs&, int, int, float, int) const {}
    __device__ void block(const GemmArgs& a, int mbase, int n, const floatx16& acc) const {
        if (n >= a.N) return;
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const float bias = a.bias[co];
        uint16_t* dst = reinterpret_cast<uint16_t*>(const_cast<float*>(a.C)) + a.c_coff + co;
        const int64_t W2 = 2 * a.W;
        int x = mbase % a.W, t = mbase / a.W, y = t % a.H, b = t / a.H;
        int cur = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int off = (r & 3) + 8 * (r >> 2);
            x += off - cur;
            cur = off;
            while (x >= a.W) { x -= a.W; if (++y == a.H) { y = 0; ++b; } }
            if (mbase + off < a.M) {
                const int64_t hp = ((int64_t)b * (2 * a.H) + 2 * y + (q >> 1)) * W2 + 2 * x + (q & 1);
                dst[hp * a.ldc] = __builtin_bit_cast(uint16_t, (__bf16)(acc[r] + bias));
            }
        }
    }
};
struct EpiSlab {   // split-K partial: slab z holds C[m][n] of K-slice z
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;
    static constexpr bool ADD = false;
    __device__ static const float* row_base(const GemmArgs& a, int m0, int z) {
        return a.C + (int64_t)z * a.slab_stride + (int64_t)m0 * a.ldc;
    }
};

}  // namespace cad
