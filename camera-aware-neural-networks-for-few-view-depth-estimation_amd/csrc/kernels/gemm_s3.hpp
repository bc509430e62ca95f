// fp32 GEMM on the bf16 matrix cores by exact operand splitting ("S3" engine), and the plain bf16
// engine ("B1") that shares its staging.
//
// Every fp32 operand x is split EXACTLY into three bf16 terms, x = x0 + x1 + x2:
//   x0 = x with the low 16 bits cleared (8 significant bits), r = x - x0 (exact, <= 16 bits),
//   x1 = r with the low 16 bits cleared, x2 = r - x1 (exact, <= 8 bits: a bf16 with zero low half).
// A product is then a*b = sum_{p,q} a_p b_q with |a_p b_q| <= 2^-8(p+q) |a b|; the six terms with
// p + q <= 2 are issued to v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact in fp32) and
// accumulated in fp32, smallest first.  The dropped terms a1b2 + a2b1 + a2b2 are < 2^-23 |a b|, i.e.
// the same order as one fp32 rounding, so the result carries fp32 accuracy (measured against fp64
// in tests/test_gpu_ops.py next to the exact-fp32 MFMA engine).  Cost: 6 bf16 MFMAs of 32 cycles
// per 16-deep k step instead of 8 f32 MFMAs of 64 cycles: 2.67x fewer matrix-core cycles.
// Inf/NaN operands give NaN (the split of an infinity is inf - inf); the hot path never carries them.
//
// B1 (NP = 1 plane): each fp32 operand is rounded to the nearest bf16 (v_cvt_pk_bf16_f32) and one
// product per k is issued — bf16 operands, fp32 accumulation: the arithmetic of BASELINE configs
// 3-5 ("bf16").  Its result equals the fp64 contraction of the bf16-rounded operands up to fp32
// accumulation error (tests/test_gpu_ops.py).
//
// Staging: the Kc loaders of gemm_mfma.hpp (k-contiguous global rows, float4 per thread) fill
// registers; the stage store converts each float4 into NP bf16x4 and writes NP LDS planes.
// KB = 16 (one k16 step per stage): 32-B rows, no padding, the 16-B half h of row r is stored at
// half h ^ ((r >> 3) & 1), which makes the ds_read_b128 fragment reads conflict-free in all four
// lane groups of the instruction (MI355X_MICROARCH.md §LDS).  Unpadded planes keep a 128x128 S3
// tile at 48 KB of LDS (double-buffered), three workgroups per CU.  KB = 32 (two k16 steps, B1):
// rows padded to 40 bf16 = 80 B, the conflict-free b128 stride of the f32 engine's Kc image.
// Fragment of a 32x32x16 MFMA: lane l holds A[row l&31][k = 8(l>>5) + j], j < 8 (one
// ds_read_b128 per plane); B likewise by column.
#pragma once
#include "gemm_mfma.hpp"

namespace cad {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// three packed bf16x4 planes (as 2 x u32 each) of one float4
struct Split4 {
    uint2 p[3];
};
__device__ __forceinline__ Split4 split3(float4 v) {
    const float x[4] = {v.x, v.y, v.z, v.w};
    uint32_t h[4], m[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const uint32_t u = __float_as_uint(x[e]);
        const uint32_t uh = u & 0xFFFF0000u;
        const float r = x[e] - __uint_as_float(uh);
        const uint32_t ur = __float_as_uint(r) & 0xFFFF0000u;
        const float r2 = r - __uint_as_float(ur);
        h[e] = uh >> 16;
        m[e] = ur >> 16;
        l[e] = __float_as_uint(r2) >> 16;
    }
    Split4 s;
    s.p[0] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    s.p[1] = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
    s.p[2] = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
    return s;
}

// one round-to-nearest-even bf16x4 plane of one float4 (B1)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
struct Split1 {
    uint2 p[1];
};
__device__ __forceinline__ Split1 split1(float4 v) {
    const bf16x2_t lo = __builtin_convertvector((f32x2_t){v.x, v.y}, bf16x2_t);
    const bf16x2_t hi = __builtin_convertvector((f32x2_t){v.z, v.w}, bf16x2_t);
    Split1 s;
    s.p[0] = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
    return s;
}
template <int NP>
__device__ __forceinline__ auto split_np(float4 v) {
    static_assert(NP == 3 || NP == 1, "planes");
    if constexpr (NP == 3) return split3(v);
    else return split1(v);
}

// Stage geometry: KB k per LDS stage = KB/16 bf16 MFMA k-steps.
template <int KB>
struct S3 {
    static_assert(KB == 16 || KB == 32 || KB == 64, "S3/B1 stage depth (64: pre-split B1 only)");
    static constexpr bool SWZ = KB == 16;
    static constexpr int LDK = SWZ ? 16 : KB + 8;   // bf16 elements per plane row (80 / 144 B: conflict-free b128)
    static constexpr int KSTEPS = KB / 16;
};

// LDS bf16 elements of one operand image: NP planes x ROWS x LDK
template <int ROWS, int KB, int NP = 3>
struct S3Lds {
    static constexpr int ELEMS = NP * ROWS * S3<KB>::LDK;
};
// element offset of (row r, k) in a plane
template <int KB>
__device__ __forceinline__ int s3_off(int r, int k) {
    if constexpr (S3<KB>::SWZ) return r * 16 + (((k >> 3) ^ ((r >> 3) & 1)) << 3) + (k & 7);
    else return r * S3<KB>::LDK + k;
}

// store the loader's float4s (Kc mapping of KS<KB>) as NP bf16 planes
template <int ROWS, int KB, int NP, int NV>
__device__ __forceinline__ void s3_store(uint16_t* s, const float4 (&v)[NV]) {
    using G = KS<KB>;
    constexpr int PL = ROWS * S3<KB>::LDK;   // elements per plane
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const auto sp = split_np<NP>(v[j]);
        const int off = s3_off<KB>(t / G::TPR + G::RPP * j, (t % G::TPR) * 4);
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(s + p * PL + off) = sp.p[p];
    }
}

// fp32 Kc image in natural k order ([rows][KB+4] floats; kc_store of gemm_mfma.hpp writes the
// same addresses — the f32 engine's k permutation lives only in its fragment reads)
template <int ROWS, int KB, int NV>
__device__ __forceinline__ void kc_store_nat(float* s, const float4 (&v)[NV]) {
    kc_store<ROWS, KB>(s, v);
}

// fragments of the NP planes for 32-row block rb, k16 step q
template <int ROWS, int KB, int NP>
__device__ __forceinline__ void s3_frag(const uint16_t* s, int rb, int q, bf16x8 (&f)[NP]) {
    constexpr int PL = ROWS * S3<KB>::LDK;
    const int lane = threadIdx.x & 63;
    const uint16_t* base = s + s3_off<KB>(rb + (lane & 31), q * 16 + (lane >> 5) * 8);
#pragma unroll
    for (int p = 0; p < NP; ++p) f[p] = *reinterpret_cast<const bf16x8*>(base + p * PL);
}

// A operand kept fp32 in LDS ([rows][KB+4] floats, the Kc image of gemm_mfma.hpp in natural k
// order) and split after the fragment read: used by S3 when every A row is read by ONE wave
// (WN == 1), so splitting at read costs no more VALU than splitting at store, and the fp32 image is
// 2/3 the bytes (the 256x64 tile then fits two workgroups per CU).
template <int ROWS, int KB>
__device__ __forceinline__ void s3_frag_f32(const float* s, int rb, int q, bf16x8 (&f)[3]) {
    const int lane = threadIdx.x & 63;
    const float* base = s + (rb + (lane & 31)) * KS<KB>::LDK + q * 16 + (lane >> 5) * 8;
    const float4 v0 = *reinterpret_cast<const float4*>(base);
    const float4 v1 = *reinterpret_cast<const float4*>(base + 4);
    const Split4 s0 = split3(v0), s1 = split3(v1);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const uint4 u = make_uint4(s0.p[p].x, s0.p[p].y, s1.p[p].x, s1.p[p].y);
        f[p] = __builtin_bit_cast(bf16x8, u);
    }
}

// zeroed accumulators of one wave: MI x NJ blocks of 32x32
template <int MI, int NJ>
__device__ __forceinline__ void acc_zero(floatx16 (&acc)[MI][NJ]) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
}

// the MFMAs of one k16 step on NP-plane fragments: S3 issues the six products with p + q <= 2,
// smallest terms first ((2,0) (1,1) (0,2) (1,0) (0,1) (0,0)); B1 the single bf16 product
template <int NP, int MI, int NJ>
__device__ __forceinline__ void s3_mfma(floatx16 (&acc)[MI][NJ], const bf16x8 (&fa)[MI][NP], const bf16x8 (&fb)[NJ][NP]) {
    if constexpr (NP == 3) {
        constexpr int P[6] = {2, 1, 0, 1, 0, 0};
        constexpr int Q[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][P[t]], fb[j][Q[t]], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0);
    }
}

// The S3/B1 engine for Kc x Kc operands (conv3x3 fwd/dgrad, ConvT fwd/dgrad).  Same tiling,
// loaders, pipeline and epilogue as gemm_body (gemm_mfma.hpp); only the LDS image and the MFMA
// differ.  AF32: A staged fp32 and split at fragment read (see s3_frag_f32); S3 with WN == 1 only.
template <int NP, int WM, int WN, int MI, int NJ, int KB, class LA, class LB, class Epi, class InitA, class InitB>
__device__ __forceinline__ void gemm_body_s3(const GemmArgs& a, InitA init_a, InitB init_b, Epi epi) {
    constexpr bool AF32 = NP == 3 && WN == 1;
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    // LDS element counts in bf16 units (an fp32 A image counts 2 per float)
    constexpr int SA = AF32 ? 2 * BM * KS<KB>::LDK : S3Lds<BM, KB, NP>::ELEMS;
    constexpr int SB = S3Lds<BN, KB, NP>::ELEMS;
    __shared__ __attribute__((aligned(16))) uint16_t lds[2 * (SA + SB)];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const TileId tile = xcd_tile();
    const int m0 = tile.x * BM, n0 = tile.y * BN;

    const int nk_total = (a.K + KB - 1) / KB;
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nk_total, kbeg + a.kstages_per_split);

    LA la; LB lb;
    init_a(la, m0, tid, kbeg);
    init_b(lb, n0, tid, kbeg);

    floatx16 acc[MI][NJ];
    acc_zero(acc);

    float4 ra[LA::NV], rb[LB::NV];
    auto load_ab = [&]() {
        la.load(ra);
        lb.load(rb);
    };
    auto stage_store = [&](int buf) {
        la.finish(ra);
        lb.finish(rb);
        uint16_t* da = lds + buf * (SA + SB);
        if constexpr (AF32) kc_store_nat<BM, KB>(reinterpret_cast<float*>(da), ra);
        else s3_store<BM, KB, NP>(da, ra);
        s3_store<BN, KB, NP>(da + SA, rb);
    };
    auto stage_compute = [&](int buf) {
        const uint16_t* sa = lds + buf * (SA + SB);
        const uint16_t* sb = sa + SA;
#pragma unroll
        for (int q = 0; q < S3<KB>::KSTEPS; ++q) {
            bf16x8 fa[MI][NP], fb[NJ][NP];
#pragma unroll
            for (int j = 0; j < NJ; ++j) s3_frag<BN, KB, NP>(sb, wn * 32 * NJ + j * 32, q, fb[j]);
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                if constexpr (AF32) s3_frag_f32<BM, KB>(reinterpret_cast<const float*>(sa), wm * 32 * MI + i * 32, q, fa[i]);
                else s3_frag<BM, KB, NP>(sa, wm * 32 * MI + i * 32, q, fa[i]);
            }
            s3_mfma<NP>(acc, fa, fb);
        }
    };

    if (kbeg < kend) {
        load_ab();
        stage_store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        if (more) load_ab();
        stage_compute(cur);
        if (more) stage_store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    gemm_epilogue_t<WM, WN, MI, NJ>(a, acc, tile, reinterpret_cast<float*>(lds), epi);
}

// ------------------------------------------------------------------------------------------
// S3/B1 engine for MNc x MNc operands (the weight-gradient GEMMs: k = pixel is the strided index).
// LDS planes are [KB k-rows][ROWS] bf16 (see S3M for the row stride / swizzle).  The MNc loader's
// float4 (4 consecutive rows at one k) is converted and stored with one ds_write_b64 per plane;
// fragments are read with ds_read_b64_tr_b16, which hands lane i of each 16-lane group column i of
// 4 consecutive k-rows: two such reads give a lane its 8 consecutive k of one row — exactly the
// 32x32x16 operand map — with no register transpose.
// ------------------------------------------------------------------------------------------
typedef short v4i16 __attribute__((ext_vector_type(4)));

// k-row stride: 128+ rows are unpadded with the 16-B chunks of k-row kr XORed by 4(kr & 3), which
// moves the four k-rows of a transposed read to disjoint bank quarters; 64-row planes (too narrow
// for that XOR) keep a 64-B pad instead.
template <int ROWS>
struct S3M {
    static constexpr bool SWZ = ROWS >= 128;
    static constexpr int STRIDE = SWZ ? ROWS * 2 : ROWS * 2 + 64;    // bytes per k-row of a plane
    // byte offset of (k-row kr, column c), c a multiple of 4
    __device__ static __forceinline__ int off(int kr, int c) {
        if constexpr (SWZ) return kr * STRIDE + ((((c >> 3) ^ ((kr & 3) << 2))) << 4) + (c & 7) * 2;
        else return kr * STRIDE + c * 2;
    }
};

template <int ROWS, int KB, int NP, int NV>
__device__ __forceinline__ void s3m_store(char* s, const float4 (&v)[NV]) {
    using Base = MNcBase<ROWS, KB>;
    constexpr int PL = KB * S3M<ROWS>::STRIDE;   // bytes per plane
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const auto sp = split_np<NP>(v[j]);
        const int off = S3M<ROWS>::off(t / Base::TPR + Base::KSTEP * j, (t % Base::TPR) * 4);
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(s + p * PL + off) = sp.p[p];
    }
}

template <int ROWS, int KB, int NP>
__device__ __forceinline__ void s3m_frag(const char* s, int rb, int q, bf16x8 (&f)[NP]) {
    constexpr int PL = KB * S3M<ROWS>::STRIDE;
    const int lane = threadIdx.x & 63;
    const int g = (lane >> 4) & 1, h = lane >> 5, i = lane & 15;
    const int krow = q * 16 + 8 * h + (i >> 2);
    const int col = rb + 16 * g + 4 * (i & 3);
    const char* b0 = s + S3M<ROWS>::off(krow, col);       // k-rows 8h + 0..3
    const char* b1 = s + S3M<ROWS>::off(krow + 4, col);   // k-rows 8h + 4..7
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        typedef __attribute__((address_space(3))) v4i16 lds_v4;
        const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(b0 + p * PL));
        const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(b1 + p * PL));
        const uint2 ul = __builtin_bit_cast(uint2, lo), uh = __builtin_bit_cast(uint2, hi);
        f[p] = __builtin_bit_cast(bf16x8, make_uint4(ul.x, ul.y, uh.x, uh.y));
    }
}

template <int NP, int WM, int WN, int MI, int NJ, int KB, class LA, class LB, class Epi, class InitA, class InitB>
__device__ __forceinline__ void gemm_body_s3m(const GemmArgs& a, InitA init_a, InitB init_b, Epi epi) {
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    constexpr int SA = NP * KB * S3M<BM>::STRIDE, SB = NP * KB * S3M<BN>::STRIDE;   // bytes
    __shared__ __attribute__((aligned(16))) char lds[2 * (SA + SB)];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const TileId tile = xcd_tile();
    const int m0 = tile.x * BM, n0 = tile.y * BN;

    const int nk_total = (a.K + KB - 1) / KB;
    const int kbeg = tile.z * a.kstages_per_split;
    const int kend = min(nk_total, kbeg + a.kstages_per_split);

    LA la; LB lb;
    init_a(la, m0, tid, kbeg);
    init_b(lb, n0, tid, kbeg);

    floatx16 acc[MI][NJ];
    acc_zero(acc);

    auto stage_store = [&](int buf, float4 (&xa)[LA::NV], float4 (&xb)[LB::NV]) {
        la.finish(xa);
        lb.finish(xb);
        char* da = lds + buf * (SA + SB);
        s3m_store<BM, KB, NP>(da, xa);
        s3m_store<BN, KB, NP>(da + SA, xb);
    };
    const bool live = wave_live(a, m0, n0, wm * 32 * MI, wn * 32 * NJ);
    auto stage_compute = [&](int buf) {
        if (!live) return;
        const char* sa = lds + buf * (SA + SB);
        const char* sb = sa + SA;
#pragma unroll
        for (int q = 0; q < S3<KB>::KSTEPS; ++q) {
            bf16x8 fa[MI][NP], fb[NJ][NP];
#pragma unroll
            for (int j = 0; j < NJ; ++j) s3m_frag<BN, KB, NP>(sb, wn * 32 * NJ + j * 32, q, fb[j]);
#pragma unroll
            for (int i = 0; i < MI; ++i) s3m_frag<BM, KB, NP>(sa, wm * 32 * MI + i * 32, q, fa[i]);
            s3_mfma<NP>(acc, fa, fb);
        }
    };

    float4 ra[LA::NV], rb[LB::NV];
    if (kbeg < kend) {
        la.load(ra);
        lb.load(rb);
        stage_store(0, ra, rb);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        if (more) { la.load(ra); lb.load(rb); }
        stage_compute(cur);
        if (more) stage_store(cur ^ 1, ra, rb);
        __syncthreads();
        cur ^= 1;
    }
    gemm_epilogue_t<WM, WN, MI, NJ>(a, acc, tile, reinterpret_cast<float*>(lds), epi);
}

}  // namespace cad
