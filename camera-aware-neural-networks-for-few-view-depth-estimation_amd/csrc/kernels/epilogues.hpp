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
// ---------------------------------------------------------------------------------------------
// Recomputed convolution (enc1.conv1: K = 9 x 8 on the raw image — cheaper to recompute from its
// 16-byte-per-pixel input than to store and re-read its fp32 output, 256 B per pixel at f = 64).
// The same GEMM (same kernel, tile and K order) is launched once per consumer, and the epilogue does
// the consumer's work on the accumulators, which equal the values the stored path would have written:
//   EpiStatsOnly     BN statistics only (the forward's EpiStoreStats without its store);
//   EpiBnRelu<OB16>  a = relu(y scale + shift) (k_bn_relu_fwd_rows' arithmetic), fp32 or bf16 rows;
//   EpiBnBwdSums<GB> per-tile fp64 partials of sum dz, sum dz xhat (dz = g [z > 0], xhat =
//                    (y - mean) invstd: OpBnBwd's arithmetic) -> a.bn_part [tile][2][N];
//   EpiBnBwdApply<GB, OB16>  dy = k0 dz - k1 - k2 xhat (k_bn_relu_bwd_rows' arithmetic).
// g (the upstream gradient a.bn_g, rows of a.bn_ldg) is bf16 (GB) or fp32.
// ---------------------------------------------------------------------------------------------
struct EpiStatsOnly : EpiStore {
    static constexpr bool STATS = true;
    static constexpr bool NOSTORE = true;
};
__device__ __forceinline__ float epi_bn_relu(float y, float s, float t) { return fmaxf(__fmaf_rn(y, s, t), 0.f); }
// One lane's view of a 32x32 block in the structured epilogues: rows mb0 + 4h + (r & 3) + 8 (r >> 2)
// (h = lane >> 5; mb0 uniform over the wave), column n.  Gradient loads and output stores go through
// buffer descriptors based at the block's first row (32-bit offsets whatever the tensor's size), all
// 16 loads issued before any use.
struct EpiRows {
    int h, mb0;
    __device__ EpiRows(int mbase) : h((threadIdx.x & 63) >> 5), mb0(mbase - 4 * ((threadIdx.x & 63) >> 5)) {}
    __device__ int row(int r) const { return 4 * h + (r & 3) + 8 * (r >> 2); }
};
template <bool GB>
__device__ __forceinline__ void epi_load_g16(const GemmArgs& a, const EpiRows& e, int n, float (&g)[16]) {
    constexpr int ES = GB ? 2 : 4;
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(reinterpret_cast<const float*>(static_cast<const char*>(a.bn_g) + (int64_t)e.mb0 * a.bn_ldg * ES));
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = e.row(r);
        const uint32_t off = e.mb0 + row < a.M ? (uint32_t)(((int64_t)row * a.bn_ldg + n) * ES) : kOOB;
        if constexpr (GB)
            g[r] = (float)__builtin_bit_cast(__bf16, (uint16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0));
        else
            g[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
    }
}
template <bool OB16>
__device__ __forceinline__ void epi_store16(const GemmArgs& a, const EpiRows& e, int n, const float (&v)[16]) {
    constexpr int ES = OB16 ? 2 : 4;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const float*>(
        reinterpret_cast<const char*>(a.C) + ((int64_t)e.mb0 * a.ldc + a.c_coff) * ES));
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = e.row(r);
        const uint32_t off = e.mb0 + row < a.M ? (uint32_t)(((int64_t)row * a.ldc + n) * ES) : kOOB;
        if constexpr (OB16)
            __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (__bf16)v[r]), rs, off, 0, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[r]), rs, off, 0, 0);
    }
}
template <bool OB16>
struct EpiBnRelu {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;   // (row-major store path unused: structured)
    static constexpr bool ADD = false;
    static constexpr bool STRUCTURED = true;
    __device__ void operator()(const GemmArgs&, int, int, float, int) const {}
    // one lane's 16 accumulator rows of a 32x32 block: rows mbase + (r&3) + 8(r>>2), column n
    __device__ void block(const GemmArgs& a, int mbase, int n, const floatx16& acc) const {
        if (n >= a.N) return;
        const EpiRows e(mbase);
        const float sc = a.bn_scale[n], sh = a.bn_shift[n];
        float o[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] = epi_bn_relu(acc[r], sc, sh);
        epi_store16<OB16>(a, e, n, o);
    }
};
// The BN column parameters and dL/da of up to 4 blocks (MI x NJ), loaded before any block is
// processed (gemm_epilogue_t's prefetch hook): the recomputed convolutions have K = 72, so the epilogue's
// memory latency, not the MFMA loop, sets their time.
template <bool GB>
struct EpiBnPrefetch {
    float g[4][16];
    float sc[4], sh[4], mu[4], is[4];
    template <int MI, int NJ>
    __device__ void prefetch(const GemmArgs& a, int mbase, int nbase) {
        static_assert(MI * NJ <= 4, "prefetch capacity");
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int n = min(nbase + 32 * j, a.N - 1);
            sc[j] = a.bn_scale[n], sh[j] = a.bn_shift[n], mu[j] = a.bn_mean[n], is[j] = a.bn_invstd[n];
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) epi_load_g16<GB>(a, EpiRows(mbase + 32 * i), min(nbase + 32 * j, a.N - 1), g[i * NJ + j]);
    }
};
template <bool GB>
struct EpiBnBwdSums : EpiBnPrefetch<GB> {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;
    static constexpr bool ADD = false;
    static constexpr bool STRUCTURED = true;
    static constexpr bool FINISH = true;
    static constexpr bool PREFETCH = true;
    double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};   // per block column j (NJ <= 4)
    __device__ void operator()(const GemmArgs&, int, int, float, int) const {}
    __device__ void block_p(const GemmArgs& a, int mbase, int n, const floatx16& acc, int b, int j) {
        if (n >= a.N) return;
        const EpiRows e(mbase);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (e.mb0 + e.row(r) >= a.M) continue;
            const float y = acc[r];
            const float z = __fmaf_rn(y, this->sc[j], this->sh[j]);
            const float dz = z > 0.f ? this->g[b][r] : 0.f;
            const float xh = (y - this->mu[j]) * this->is[j];
            s0[j] += dz;
            s1[j] += (double)dz * xh;
        }
    }
    // lanes L, L + 32 (same column) -> waves of one column group (LDS, fp64) -> a.bn_part[tile][2][N]
    template <int WM, int WN, int NJ>
    __device__ void finish(const GemmArgs& a, float* ldsf, int tile_x, int n0) {
        static_assert(NJ <= 4, "columns per lane");
        constexpr int BN = 32 * NJ * WN;
        double* lds = reinterpret_cast<double*>(ldsf);
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        const int wm = wave / WN, wn = wave % WN;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const double t0 = s0[j] + __shfl_xor(s0[j], 32), t1 = s1[j] + __shfl_xor(s1[j], 32);
            if (lane < 32) {
                double* r = lds + ((int64_t)wm * BN + wn * 32 * NJ + j * 32 + lane) * 2;
                r[0] = t0;
                r[1] = t1;
            }
        }
        __syncthreads();
        for (int c = tid; c < BN; c += 256) {
            double u0 = 0.0, u1 = 0.0;
#pragma unroll
            for (int w = 0; w < WM; ++w) {
                u0 += lds[((int64_t)w * BN + c) * 2];
                u1 += lds[((int64_t)w * BN + c) * 2 + 1];
            }
            const int n = n0 + c;
            if (n < a.N) {
                a.bn_part[((int64_t)tile_x * 2) * a.N + n] = u0;
                a.bn_part[((int64_t)tile_x * 2 + 1) * a.N + n] = u1;
            }
        }
    }
};
template <bool GB, bool OB16>
struct EpiBnBwdApply : EpiBnPrefetch<GB> {
    static constexpr bool STATS = false;
    static constexpr bool BF16 = false;
    static constexpr bool ADD = false;
    static constexpr bool STRUCTURED = true;
    static constexpr bool PREFETCH = true;
    __device__ void operator()(const GemmArgs&, int, int, float, int) const {}
    __device__ void block_p(const GemmArgs& a, int mbase, int n, const floatx16& acc, int b, int j) const {
        if (n >= a.N) return;
        const EpiRows e(mbase);
        const float k0 = a.bn_coef[n], k1 = a.bn_coef[a.N + n], k2 = a.bn_coef[2 * a.N + n];
        float o[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float y = acc[r];
            const float z = __fmaf_rn(y, this->sc[j], this->sh[j]);
            const float dz = z > 0.f ? this->g[b][r] : 0.f;
            const float xh = (y - this->mu[j]) * this->is[j];
            o[r] = __fsub_rn(__fmaf_rn(k0, dz, -k1), __fmul_rn(k2, xh));
        }
        epi_store16<OB16>(a, e, n, o);
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
