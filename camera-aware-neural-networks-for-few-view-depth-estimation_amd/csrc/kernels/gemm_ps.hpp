// Pre-split operand engine ("PS"): the S3 / B1 contractions (gemm_s3.hpp) fed from operand tensors
// that were split into bf16 planes ONCE, by the kernel that produced them (or a split pass right
// after it), instead of by every GEMM workgroup that reads them.
//
// Why: an im2col operand element is fetched by ~9 x (N / BN) workgroups; splitting it at every fetch
// cost the S3 main loop ~100 VALU instructions per wave per k16 step beside its 24 MFMAs — measured
// on MI355X, removing that work lifts the 128x128 S3 conv GEMMs from ~190 to ~297 TFLOP/s
// (fp32-equivalent).  Here the main loop only moves bytes: buffer_load_dwordx4 -> ds_write_b128.
//
// Split tensor layout (NP planes; NP = 3 exact split, NP = 1 bf16 round-to-nearest): a row of `ld`
// channels is stored as ld/8 groups of 8 channels; group g holds NP consecutive 16-B planes of 8
// bf16.  byte(row, c, p) = row * ld * 2 * NP + (c >> 3) * 16 * NP + p * 16 + (c & 7) * 2.
// Channel offsets and channel counts must be multiples of 8 (every U-Net conv except enc1.conv1's
// 3/4-channel input, which keeps the in-loader split).  For NP = 1 this is plain NHWC bf16.
//
// Loaders fill caller-owned register sets (Regs: uint4 per 16-B piece; the bodies keep one, loaded
// one compute phase ahead — see ps_pipeline) and write them to the LDS images of gemm_s3.hpp unchanged (planes [rows][LDK] for k-contiguous
// operands, [k-rows][rows] for the weight-gradient operands), so fragment reads and MFMAs are shared.
#pragma once
#include "gemm_s3.hpp"

namespace cad {

__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ const float* ps_at(const float* base, int64_t bytes) {
    return reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + bytes);
}

// k-contiguous operands.  One stage of a row is NG = KB/8 groups x NP planes = PPR 16-B pieces,
// contiguous in memory (the split layout above).  Thread t owns pieces t + 256 j of the stage
// (row = piece / PPR), so consecutive lanes read consecutive 16-B pieces of the same row: one load
// instruction covers ~64*16/(PPR*16) whole row-stages instead of one 16-B piece of 32-64 rows
// (which measured 1.3x slower than the in-loader split: 6x the address-unit work per stage).
template <int ROWS, int KB, int NP>
struct PKc {
    static constexpr int NG = KB / 8;                      // 8-k groups per stage
    static constexpr int PPR = NG * NP;                    // 16-B pieces per row and stage
    static constexpr int TASKS = ROWS * PPR;
    static constexpr int NV = (TASKS + 255) / 256;
    static_assert(TASKS % 64 == 0, "whole waves per task slot");
};

template <int ROWS, int KB, int NP>
struct PsKcBase {
    using G = PKc<ROWS, KB, NP>;
    static constexpr int NV = G::NV;
    using Regs = uint4[NV];
    int lofs[NV];   // element offset in the operand image (plane * PL + swizzled (row, 8g))
    int grp[NV];    // the piece's 8-k group in the stage
    int prow[NV];   // the piece's tile row
    __device__ static constexpr bool valid(int j) { return 256 * (j + 1) <= G::TASKS; }
    __device__ bool act(int j) const { return valid(j) || (int)threadIdx.x + 256 * j < G::TASKS; }
    __device__ void init_lds(int tid) {
        constexpr int PL = ROWS * S3<KB>::LDK;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int task = tid + 256 * j;
            const int row = task / G::PPR, piece = task - row * G::PPR;
            const int g = piece / NP, p = piece - g * NP;
            prow[j] = row;
            grp[j] = g;
            lofs[j] = p * PL + s3_off<KB>(row < ROWS ? row : 0, g * 8);
        }
    }
    // byte offset of the piece inside its row-stage: (g * NP + p) * 16
    __device__ uint32_t piece_off(int tid, int j) const { return (uint32_t)((tid + 256 * j) % G::PPR) * 16; }
    __device__ void store(const Regs& v, uint16_t* s) const {   // s: the operand image (plane 0)
#pragma unroll
        for (int j = 0; j < NV; ++j)
            if (act(j)) *reinterpret_cast<uint4*>(s + lofs[j]) = v[j];
    }
};

// op(r, k) = P[r][coff + k], r < nrows, k < K (weights [co][tap][ci], ConvT operands); K % 8 == 0
template <int ROWS, int KB, int NP>
struct PsKcDense : PsKcBase<ROWS, KB, NP> {
    using Base = PsKcBase<ROWS, KB, NP>;
    using G = typename Base::G;
    __amdgpu_buffer_rsrc_t rs;
    uint32_t roff[G::NV];
    int K, k0;
    int cim, cin, tap, ci;   // cim: channel-major conv K order (GemmArgs::cimajor)
    __device__ void init(const float* P, int64_t ld, int coff, int nrows, int K_, int row0, int tid, int kbeg,
                         int cim_ = 0, int cin_ = 0) {
        Base::init_lds(tid);
        K = K_;
        k0 = kbeg * KB;
        cim = cim_; cin = cin_;
        if (cim) { tap = kbeg % 9; ci = (kbeg / 9) * KB; }
        const int64_t rowB = ld * 2 * NP;
        rs = make_rsrc(ps_at(P, (int64_t)row0 * rowB + (int64_t)(coff >> 3) * 16 * NP));
#pragma unroll
        for (int j = 0; j < G::NV; ++j)
            roff[j] = (this->act(j) && row0 + this->prow[j] < nrows)
                          ? (uint32_t)(this->prow[j] * rowB) + this->piece_off(tid, j) : kOOB;
    }
    __device__ void load(typename Base::Regs& v) {
        if (cim) {   // every stage is whole (K = 9 cin, cin % KB == 0)
            const uint32_t ko = (uint32_t)((tap * cin + ci) >> 3) * 16 * NP;
#pragma unroll
            for (int j = 0; j < G::NV; ++j) v[j] = bload16(rs, roff[j] != kOOB ? roff[j] + ko : kOOB);
            if (++tap == 9) { tap = 0; ci += KB; }
            return;
        }
        const uint32_t ko = (uint32_t)(k0 >> 3) * 16 * NP;
#pragma unroll
        for (int j = 0; j < G::NV; ++j)
            v[j] = bload16(rs, (k0 + 8 * this->grp[j] < K && roff[j] != kOOB) ? roff[j] + ko : kOOB);
        k0 += KB;
    }
};

// (tap, ci) of each 8-k group of the current stage: group 0 carried across stages, the rest derived
template <int NG>
struct GroupTaps {
    int tap[NG], ci[NG];
    __device__ void from(int tap0, int ci0, int cin) {
        tap[0] = tap0; ci[0] = ci0;
#pragma unroll
        for (int g = 1; g < NG; ++g) {
            int c = ci[g - 1] + 8, t = tap[g - 1];
            if (c >= cin) { c -= cin; ++t; }
            tap[g] = t; ci[g] = c;
        }
    }
};

// op(pix, k=(tap,ci)) = X[(b, y+ky-1, x+kx-1)][coff + ci], zero outside the image; cin % 8 == 0
template <int ROWS, int KB, int NP>
struct PsKcIm2col3x3 : PsKcBase<ROWS, KB, NP> {
    using Base = PsKcBase<ROWS, KB, NP>;
    using G = typename Base::G;
    __amdgpu_buffer_rsrc_t rs;
    int rowB;
    uint32_t poff[G::NV];   // byte offset of the piece's pixel (+ piece offset) from the block base
    int y[G::NV], x[G::NV];
    bool ok[G::NV];
    int H, W, cin, tap, ci, cim;
    __device__ void init(const float* P, int64_t ld, int coff, int cin_, int B, int H_, int W_, int row0, int tid,
                         int kbeg, int cim_ = 0) {
        Base::init_lds(tid);
        H = H_; W = W_; cin = cin_; rowB = (int)(ld * 2 * NP);
        cim = cim_;
        const int pb = max(row0 - W_ - 1, 0);   // first pixel of the block's halo window
        rs = make_rsrc(ps_at(P, (int64_t)pb * rowB + (int64_t)(coff >> 3) * 16 * NP));
        if (cim) {
            tap = kbeg % 9;
            ci = (kbeg / 9) * KB;
        } else {
            const int k = kbeg * KB;
            tap = k / cin;
            ci = k - tap * cin;
        }
        const int M = B * H * W;
#pragma unroll
        for (int j = 0; j < G::NV; ++j) {
            const int r = row0 + this->prow[j];
            ok[j] = this->act(j) && r < M;
            const int rr = ok[j] ? r : 0;
            x[j] = rr % W;
            y[j] = (rr / W) % H;
            // the piece's plane: piece_off minus its group's (g * NP * 16) part
            poff[j] = (uint32_t)((rr - pb) * rowB) + this->piece_off(tid, j) - (uint32_t)(this->grp[j] * NP * 16);
        }
    }
    __device__ void load(typename Base::Regs& v) {
        if (cim) {   // one tap per stage, groups = consecutive channels
            const int dy = tap / 3 - 1, dx = tap - 3 * (tap / 3) - 1;
            const int off = (dy * W + dx) * rowB + (ci >> 3) * 16 * NP;
#pragma unroll
            for (int j = 0; j < G::NV; ++j) {
                const int yy = y[j] + dy, xx = x[j] + dx;
                const bool g = ok[j] && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
                v[j] = bload16(rs, g ? poff[j] + (uint32_t)(off + this->grp[j] * 16 * NP) : kOOB);
            }
            if (++tap == 9) { tap = 0; ci += KB; }
            return;
        }
        GroupTaps<G::NG> gt;
        gt.from(tap, ci, cin);
#pragma unroll
        for (int j = 0; j < G::NV; ++j) {
            int t = gt.tap[0], c = gt.ci[0];
#pragma unroll
            for (int g = 1; g < G::NG; ++g)
                if (this->grp[j] == g) { t = gt.tap[g]; c = gt.ci[g]; }
            const bool kin = t < 9;
            const int tt = kin ? t : 0;
            const int dy = tt / 3 - 1, dx = tt - 3 * (tt / 3) - 1;
            const int yy = y[j] + dy, xx = x[j] + dx;
            const bool g = ok[j] && kin && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            const int off = (dy * W + dx) * rowB + (c >> 3) * 16 * NP;
            v[j] = bload16(rs, g ? poff[j] + (uint32_t)off : kOOB);
        }
        tapci_advance<KB>(tap, ci, cin);
    }
};

// op(lowres pix (b,y,x), k=(q=(dy,dx), co)) = G[(b, 2y+dy, 2x+dx)][coff + co]; cout % 8 == 0
template <int ROWS, int KB, int NP>
struct PsKcUpGather : PsKcBase<ROWS, KB, NP> {
    using Base = PsKcBase<ROWS, KB, NP>;
    using G = typename Base::G;
    __amdgpu_buffer_rsrc_t rs;
    int rowB;
    uint32_t hoff[G::NV];
    int W2, cout, q, co;
    __device__ void init(const float* P, int64_t ld, int coff, int cout_, int B, int H, int W, int row0, int tid,
                         int kbeg) {
        Base::init_lds(tid);
        rowB = (int)(ld * 2 * NP); cout = cout_; W2 = 2 * W;
        const int k = kbeg * KB;
        q = k / cout;
        co = k - q * cout;
        const int M = B * H * W;
        auto hr = [&](int r) {
            const int xx = r % W, t = r / W, yy = t % H, b = t / H;
            return ((int64_t)b * (2 * H) + 2 * yy) * W2 + 2 * xx;
        };
        const int64_t hb = hr(min(row0, M - 1));
        rs = make_rsrc(ps_at(P, hb * rowB + (int64_t)(coff >> 3) * 16 * NP));
#pragma unroll
        for (int j = 0; j < G::NV; ++j) {
            const int r = row0 + this->prow[j];
            hoff[j] = (this->act(j) && r < M)
                          ? (uint32_t)((hr(r) - hb) * rowB) + this->piece_off(tid, j) - (uint32_t)(this->grp[j] * NP * 16)
                          : kOOB;
        }
    }
    __device__ void load(typename Base::Regs& v) {
        GroupTaps<G::NG> gt;
        gt.from(q, co, cout);
#pragma unroll
        for (int j = 0; j < G::NV; ++j) {
            int t = gt.tap[0], c = gt.ci[0];
#pragma unroll
            for (int g = 1; g < G::NG; ++g)
                if (this->grp[j] == g) { t = gt.tap[g]; c = gt.ci[g]; }
            const bool kin = t < 4;
            const int qq = kin ? t : 0;
            const uint32_t off = (uint32_t)(((qq >> 1) * W2 + (qq & 1)) * rowB + (c >> 3) * 16 * NP);
            v[j] = bload16(rs, kin && hoff[j] != kOOB ? hoff[j] + off : kOOB);
        }
        tapci_advance<KB>(q, co, cout);
    }
};

// --------------------------------------------------------------------------------------------
// MNc (weight-gradient) operands: op(row r, k = pixel), rows contiguous in memory.  A chunk is 8
// consecutive rows at one pixel; TPR chunks per k-row, KSTEP k-rows per pass of 256 threads.
// --------------------------------------------------------------------------------------------
template <int ROWS, int KB>
struct PMNc {
    static constexpr int TPR = ROWS / 8;
    static constexpr int KSTEP = 256 / TPR;
    static constexpr int TASKS = TPR * KB;
    static constexpr int NV = TASKS >= 256 ? TASKS / 256 : 1;
    static constexpr bool PARTIAL = TASKS < 256;
};

template <int ROWS, int KB, int NP>
struct PsMNcBase {
    using G = PMNc<ROWS, KB>;
    static constexpr int NV = G::NV;
    using Regs = uint4[NV][NP];
    int lofs[NV];   // byte offset of the chunk in a plane (gemm_s3.hpp S3M)
    bool act;
    __device__ void init_lds(int tid) {
        act = !G::PARTIAL || tid < G::TASKS;
#pragma unroll
        for (int j = 0; j < NV; ++j) lofs[j] = S3M<ROWS>::off(tid / G::TPR + G::KSTEP * j, (tid % G::TPR) * 8);
    }
    __device__ void store(const Regs& v, char* s) const {   // s: plane 0 of the operand image
        constexpr int PL = KB * S3M<ROWS>::STRIDE;
        if (!act) return;
#pragma unroll
        for (int j = 0; j < NV; ++j)
#pragma unroll
            for (int p = 0; p < NP; ++p) *reinterpret_cast<uint4*>(s + p * PL + lofs[j]) = v[j][p];
    }
};

// op(r, k) = P[k][coff + r], r < nrows (nrows % 8 == 0), k < Kp
template <int ROWS, int KB, int NP>
struct PsMNcDense : PsMNcBase<ROWS, KB, NP> {
    using Base = PsMNcBase<ROWS, KB, NP>;
    using G = typename Base::G;
    __amdgpu_buffer_rsrc_t rs;
    uint32_t koff;   // byte offset of the thread's k-row 0 (advances KB rows per stage)
    int rowB, Kp, k0;
    bool rok;
    __device__ void init(const float* P, int64_t ld, int coff, int nrows, int Kp_, int row0, int tid, int kbeg) {
        Base::init_lds(tid);
        rowB = (int)(ld * 2 * NP); Kp = Kp_;
        const int r = row0 + (tid % G::TPR) * 8;
        rok = this->act && r < nrows;
        const int kb0 = kbeg * KB;
        rs = make_rsrc(ps_at(P, (int64_t)kb0 * rowB + (int64_t)((coff + row0) >> 3) * 16 * NP));
        k0 = kb0 + tid / G::TPR;
        koff = (uint32_t)((tid / G::TPR) * rowB + (tid % G::TPR) * 16 * NP);
    }
    __device__ void load(typename Base::Regs& v) {
#pragma unroll
        for (int j = 0; j < G::NV; ++j) {
            const int k = k0 + G::KSTEP * j;
            const bool g = rok && k < Kp;
#pragma unroll
            for (int p = 0; p < NP; ++p)
                v[j][p] = bload16(rs, g ? koff + (uint32_t)(G::KSTEP * j * rowB) + p * 16 : kOOB);
        }
        k0 += KB;
        koff += (uint32_t)(KB * rowB);
    }
};

// op(j=(tap,ci), k=pix) = X[(b,y+ky-1,x+kx-1)][coff + ci]; cin % 8 == 0
template <int ROWS, int KB, int NP>
struct PsMNcIm2col3x3 : PsMNcBase<ROWS, KB, NP> {
    using Base = PsMNcBase<ROWS, KB, NP>;
    using G = typename Base::G;
    __amdgpu_buffer_rsrc_t rs;
    int rowB, H, W, Kp, dy, dx, pb;
    int tapoff;   // byte offset of the thread's (tap, ci) chunk relative to its pixel
    int k[G::NV], x[G::NV], y[G::NV];
    bool rok;
    __device__ void init(const float* P, int64_t ld, int coff, int cin, int B, int H_, int W_, int row0, int tid,
                         int kbeg) {
        Base::init_lds(tid);
        rowB = (int)(ld * 2 * NP); H = H_; W = W_; Kp = B * H_ * W_;
        const int j = row0 + (tid % G::TPR) * 8;
        rok = this->act && j < 9 * cin;
        const int jj = rok ? j : 0;
        const int tap = jj / cin, ci = jj - tap * cin;
        dy = tap / 3 - 1; dx = tap % 3 - 1;
        pb = max(kbeg * KB - W_ - 1, 0);
        rs = make_rsrc(ps_at(P, (int64_t)pb * rowB + (int64_t)(coff >> 3) * 16 * NP));
        tapoff = (dy * W + dx) * rowB + (ci >> 3) * 16 * NP;
#pragma unroll
        for (int i = 0; i < G::NV; ++i) {
            k[i] = kbeg * KB + tid / G::TPR + G::KSTEP * i;
            const int kk = k[i] < Kp ? k[i] : 0;
            x[i] = kk % W;
            y[i] = (kk / W) % H;
        }
    }
    __device__ void load(typename Base::Regs& v) {
#pragma unroll
        for (int j = 0; j < G::NV; ++j) {
            const int yy = y[j] + dy, xx = x[j] + dx;
            const bool g = rok && k[j] < Kp && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
            const uint32_t off = (uint32_t)((k[j] - pb) * rowB + tapoff);
#pragma unroll
            for (int p = 0; p < NP; ++p) v[j][p] = bload16(rs, g ? off + p * 16 : kOOB);
            int b = 0;
            px_advance<KB>(x[j], y[j], b, W, H);
            k[j] += KB;
        }
    }
};

// op(j=(q,co), k=lowres pix (b,y,x)) = G[(b,2y+dy,2x+dx)][coff + co]; cout % 8 == 0
template <int ROWS, int KB, int NP>
struct PsMNcUpGather : PsMNcBase<ROWS, KB, NP> {
    using Base = PsMNcBase<ROWS, KB, NP>;
    using G = typename Base::G;
    __amdgpu_buffer_rsrc_t rs;
    int64_t hb;
    int rowB, H, W, Kp, qy, qx, cooff;
    int k[G::NV], x[G::NV], y[G::NV], b[G::NV];
    bool rok;
    __device__ void init(const float* P, int64_t ld, int coff, int cout, int B, int H_, int W_, int row0, int tid,
                         int kbeg) {
        Base::init_lds(tid);
        rowB = (int)(ld * 2 * NP); H = H_; W = W_; Kp = B * H_ * W_;
        const int j = row0 + (tid % G::TPR) * 8;
        rok = this->act && j < 4 * cout;
        const int jj = rok ? j : 0;
        const int q = jj / cout, co = jj - q * cout;
        qy = q >> 1; qx = q & 1;
        cooff = (co >> 3) * 16 * NP;
        {
            const int kk = min(kbeg * KB, Kp - 1);
            const int xx = kk % W, t = kk / W, yy = t % H, bb = t / H;
            hb = ((int64_t)bb * (2 * H) + 2 * yy) * (2 * W) + 2 * xx;
        }
        rs = make_rsrc(ps_at(P, hb * rowB + (int64_t)(coff >> 3) * 16 * NP));
#pragma unroll
        for (int i = 0; i < G::NV; ++i) {
            k[i] = kbeg * KB + tid / G::TPR + G::KSTEP * i;
            const int kk = k[i] < Kp ? k[i] : 0;
            x[i] = kk % W;
            const int t = kk / W;
            y[i] = t % H;
            b[i] = t / H;
        }
    }
    __device__ void load(typename Base::Regs& v) {
#pragma unroll
        for (int j = 0; j < G::NV; ++j) {
            const bool g = rok && k[j] < Kp;
            const int64_t hp = ((int64_t)b[j] * (2 * H) + 2 * y[j] + qy) * (2 * W) + 2 * x[j] + qx;
            const uint32_t off = (uint32_t)((hp - hb) * rowB + cooff);
#pragma unroll
            for (int p = 0; p < NP; ++p) v[j][p] = bload16(rs, g ? off + p * 16 : kOOB);
            px_advance<KB>(x[j], y[j], b[j], W, H);
            k[j] += KB;
        }
    }
};

// --------------------------------------------------------------------------------------------
// engine bodies: double-buffered LDS, one barrier per stage, one register set per operand (the
// loads of stage k+1 are in flight while stage k is computed).  A two-set variant (loads two
// compute phases ahead) measured slower on MI355X: the second set costs ~50 VGPRs and a wave per
// SIMD (B1 128x128 GEMMs 700 -> 544 TFLOP/s), more than the deeper prefetch returns.
// --------------------------------------------------------------------------------------------
template <class LA, class LB, class Compute, class StoreAB>
__device__ __forceinline__ void ps_pipeline(LA& la, LB& lb, int kbeg, int kend, Compute compute, StoreAB store_ab) {
    typename LA::Regs ra;
    typename LB::Regs rb;
    if (kbeg < kend) {
        la.load(ra);
        lb.load(rb);
        store_ab(0, ra, rb);
    }
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
        const bool more = kt + 1 < kend;
        if (more) { la.load(ra); lb.load(rb); }
        compute(cur);
        if (more) store_ab(cur ^ 1, ra, rb);
        __syncthreads();
        cur ^= 1;
    }
}

template <int NP, int WM, int WN, int MI, int NJ, int KB, class LA, class LB, class Epi, class InitA, class InitB>
__device__ __forceinline__ void gemm_body_ps(const GemmArgs& a, InitA init_a, InitB init_b, Epi epi) {
    constexpr int BM = 32 * MI * WM, BN = 32 * NJ * WN;
    constexpr int SA = S3Lds<BM, KB, NP>::ELEMS, SB = S3Lds<BN, KB, NP>::ELEMS;
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

    auto store_ab = [&](int buf, const typename LA::Regs& xa, const typename LB::Regs& xb) {
        uint16_t* da = lds + buf * (SA + SB);
        la.store(xa, da);
        lb.store(xb, da + SA);
    };
    auto compute = [&](int buf) {
        const uint16_t* sa = lds + buf * (SA + SB);
        const uint16_t* sb = sa + SA;
#pragma unroll
        for (int q = 0; q < S3<KB>::KSTEPS; ++q) {
            bf16x8 fa[MI][NP], fb[NJ][NP];
#pragma unroll
            for (int j = 0; j < NJ; ++j) s3_frag<BN, KB, NP>(sb, wn * 32 * NJ + j * 32, q, fb[j]);
#pragma unroll
            for (int i = 0; i < MI; ++i) s3_frag<BM, KB, NP>(sa, wm * 32 * MI + i * 32, q, fa[i]);
            s3_mfma<NP>(acc, fa, fb);
        }
    };
    ps_pipeline(la, lb, kbeg, kend, compute, store_ab);
    gemm_epilogue_t<WM, WN, MI, NJ>(a, acc, tile, reinterpret_cast<float*>(lds), epi);
}

template <int NP, int WM, int WN, int MI, int NJ, int KB, class LA, class LB, class Epi, class InitA, class InitB>
__device__ __forceinline__ void gemm_body_psm(const GemmArgs& a, InitA init_a, InitB init_b, Epi epi) {
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

    auto store_ab = [&](int buf, const typename LA::Regs& xa, const typename LB::Regs& xb) {
        char* da = lds + buf * (SA + SB);
        la.store(xa, da);
        lb.store(xb, da + SA);
    };
    const bool live = wave_live(a, m0, n0, wm * 32 * MI, wn * 32 * NJ);
    auto compute = [&](int buf) {
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
    ps_pipeline(la, lb, kbeg, kend, compute, store_ab);
    gemm_epilogue_t<WM, WN, MI, NJ>(a, acc, tile, reinterpret_cast<float*>(lds), epi);
}

// --------------------------------------------------------------------------------------------
// the split pass: fp32 rows [M][ldx] (channels [xcoff, xcoff + C)) -> NP-plane split rows
// --------------------------------------------------------------------------------------------
template <int NP>
__device__ __forceinline__ void split8_store(char* dst, float4 a, float4 b) {
    const auto sa = split_np<NP>(a);
    const auto sb = split_np<NP>(b);
#pragma unroll
    for (int p = 0; p < NP; ++p)
        *reinterpret_cast<uint4*>(dst + p * 16) = make_uint4(sa.p[p].x, sa.p[p].y, sb.p[p].x, sb.p[p].y);
}

}  // namespace cad
