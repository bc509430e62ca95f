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
// ... with the added matrix's own row stride a.ldc2 (config 5: a decoder concat's skip-half gradient
// added to the block-output gradient a projection block's conv1 dgrad produces)
struct EpiStoreAddLd : EpiStoreAdd {
    static constexpr bool ADD_LD = true;
    __device__ static const float* add_base(const GemmArgs& a, int m0) { return a.bias + (int64_t)m0 * a.ldc2; }
};
// ... then zeroed where the fp32 matrix a.C2 (same rows / offset as C) is not > 0: config 5's block-input
// gradient masked by the previous block's ReLU output (the separate k_relu_mask pass, fused)
struct EpiStoreAddMask : EpiStoreAdd {
    static constexpr bool MASK = true;
    __device__ static const float* mask_base(const GemmArgs& a, int m0) {
        return static_cast<const float*>(a.C2) + (int64_t)m0 * a.ldc + a.c_coff;
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
// window epilogue only (round 5): the store, plus the BatchNorm backward's column sums of the BN whose
// output gradient this GEMM produces (a DoubleConv's conv2 input gradient dL/da1 feeding bn1's
// backward): per tile, sum dz and sum dz xhat with dz = v [y scale + shift > 0], xhat = (y - mean)
// invstd, v the stored value (bf16-rounded for OB16) and y the BN input (a.bn_g: rows of a.bn_ldg,
// bf16 for YB) — OpBnBwd's arithmetic, fp64 per lane — into a.bn_part[tile][2][N].  The separate
// column-reduction pass over (dL/da1, y) is then not needed.
template <bool OB16, bool YB>
struct EpiStoreBnSums {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = OB16;
    static constexpr bool ADD = false;
    static constexpr bool SPLIT = false;
    static constexpr bool BNSUMS = true;
    static constexpr bool Y_BF16 = YB;
};

// ConvTranspose2d(k2,s2) pixel shuffle: n = (q=(dy,dx), co) -> high-res pixel (2y+dy, 2x+dx).
// The column (q, co) is fixed per lane and sub-block (STRUCTURED epilogue).  When W % 32 == 0 a
// 32-row block is one run of 32 pixels of one image row (blocks start at multiples of 32), so its
// high-res rows are hp0 + dy*2W + dx + 2*off: one buffer descriptor at hp0 (wave-uniform), the lane's
// (dy, dx, co, h) part in the vector offset and the row's 2*off*ldc in the scalar offset — no per-element
// index arithmetic.  Other widths carry (x, y, b) incrementally per row.
// OB16: bf16 output (a.C addresses bf16 rows of ldc elements: the bf16 engine's up half of the decoder
// concat, written straight into the consumers' twin); fp32 otherwise.
template <bool OB16>
struct EpiConvTOut {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;   // (row-major store path unused: structured)
    static constexpr bool ADD = false;
    static constexpr bool STRUCTURED = true;
    static constexpr int ES = OB16 ? 2 : 4;
    __device__ void operator()(const GemmArgs& a, int m, int n, float v, int) const {
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const int x = m % a.W, t = m / a.W, y = t % a.H, b = t / a.H;
        const int64_t hp = ((int64_t)b * (2 * a.H) + 2 * y + (q >> 1)) * (2 * a.W) + 2 * x + (q & 1);
        put(a, hp * a.ldc + a.c_coff + co, v + a.bias[co]);
    }
    // bf16 output, W % 32 == 0, cout % (32 NJ) == 0: per 32-row block i, the wave writes its 32 x 32 NJ
    // bf16 values into its LDS slice (row stride 32 NJ + 8 elements) and stores them back as 16-byte pieces
    // of the high-res rows (one 2-byte store per element moved 128 B per instruction: the level-0 ConvT
    // ran at ~3 TB/s, store-issue bound)
    static constexpr bool WAVE_STORE = OB16;
    template <int NJ>
    __device__ static constexpr int lds_floats_per_wave() { return 32 * (32 * NJ + 8) / 2; }
    template <int MI, int NJ>
    __device__ bool wave_store(const GemmArgs& a, const floatx16 (&acc)[MI][NJ], int mw0, int nw0, float* ldsf) const {
        constexpr int WC = 32 * NJ, RS = WC + 8, CH = WC / 8;   // columns, LDS row stride, 16-B pieces per row
        const int cout = a.N >> 2;
        // 16-byte stores: the row stride and channel offset must keep every piece 16-byte aligned
        if (a.W % 32 != 0 || cout % WC != 0 || a.ldc % 8 != 0 || a.c_coff % 8 != 0) return false;
        if (nw0 >= a.N) return true;   // N % WC == 0: the wave's columns are wholly in or out
        const int lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
        const int q = nw0 / cout, co0 = nw0 - q * cout;
        float bias[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bias[j] = a.bias[co0 + 32 * j + c];
        uint16_t* L = reinterpret_cast<uint16_t*>(ldsf);
        const int64_t W2 = 2 * a.W;
        const int64_t qoff = (q >> 1) * W2 + (q & 1);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int mb0 = __builtin_amdgcn_readfirstlane(mw0 + 32 * i);
            if (mb0 >= a.M) break;   // M % 32 == 0: blocks wholly in or out
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous block's reads are done
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    L[(4 * h + (r & 3) + 8 * (r >> 2)) * RS + 32 * j + c] =
                        __builtin_bit_cast(uint16_t, (__bf16)(acc[i][j][r] + bias[j]));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // all lanes' writes visible to the wave
            const int x0 = mb0 % a.W, t = mb0 / a.W, y0 = t % a.H, b0 = t / a.H;
            const int64_t hp0 = ((int64_t)b0 * (2 * a.H) + 2 * y0) * W2 + 2 * x0;
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const float*>(
                reinterpret_cast<const char*>(a.C) + (hp0 * a.ldc + a.c_coff + co0) * 2));
#pragma unroll
            for (int k = 0; k < 32 * CH / 64; ++k) {
                const int id = lane + 64 * k, row = id / CH, ch = id % CH;
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 v = *reinterpret_cast<const u32x4*>(L + row * RS + ch * 8);
                const uint32_t off = (uint32_t)(((qoff + 2 * row) * a.ldc + 8 * ch) * 2);
                __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
            }
        }
        return true;
    }
    __device__ static void put(const GemmArgs& a, int64_t e, float v) {
        if constexpr (OB16)
            reinterpret_cast<uint16_t*>(const_cast<float*>(a.C))[e] = __builtin_bit_cast(uint16_t, (__bf16)v);
        else
            const_cast<float*>(a.C)[e] = v;
    }
    // one lane's 16 accumulator rows of a 32x32 sub-block: rows mbase + (r&3) + 8(r>>2), column n
    __device__ void block(const GemmArgs& a, int mbase, int n, const floatx16& acc) const {
        if (n >= a.N) return;
        const int cout = a.N >> 2;
        const int q = n / cout, co = n - q * cout;
        const float bias = a.bias[co];
        const int64_t W2 = 2 * a.W;
        if (a.W % 32 == 0) {
            const int h = (threadIdx.x & 63) >> 5;
            const int mb0 = __builtin_amdgcn_readfirstlane(mbase - 4 * h);
            if (mb0 >= a.M) return;   // M % 32 == 0 here: a block is wholly in or out
            const int x0 = mb0 % a.W, t = mb0 / a.W, y0 = t % a.H, b0 = t / a.H;
            const int64_t hp0 = ((int64_t)b0 * (2 * a.H) + 2 * y0) * W2 + 2 * x0;
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const float*>(
                reinterpret_cast<const char*>(a.C) + (hp0 * a.ldc + a.c_coff) * ES));
            const uint32_t lane = (uint32_t)((((q >> 1) * W2 + (q & 1) + 8 * h) * a.ldc + co) * ES);
            const uint32_t rstride = (uint32_t)(2 * a.ldc * ES);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t so = (uint32_t)((r & 3) + 8 * (r >> 2)) * rstride;
                const float v = acc[r] + bias;
                if constexpr (OB16)
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (__bf16)v), rs, lane, so, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rs, lane, so, 0);
            }
            return;
        }
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
                put(a, hp * a.ldc + a.c_coff + co, acc[r] + bias);
            }
        }
    }
};
using EpiConvT = EpiConvTOut<false>;
using EpiConvTB16 = EpiConvTOut<true>;
struct EpiSlab {   // split-K partial: slab z holds C[m][n] of K-slice z
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;
    static constexpr bool ADD = false;
    __device__ static const float* row_base(const GemmArgs& a, int m0, int z) {
        return a.C + (int64_t)z * a.slab_stride + (int64_t)m0 * a.ldc;
    }
};

}  // namespace cad
