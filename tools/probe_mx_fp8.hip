// Probe: operand / scale lane maps of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3) on gfx950.
// One wave computes C = (A * 2^sa) (B * 2^sb) for exact small-integer e4m3 data; the host evaluates
// candidate lane maps and reports which one the hardware matches (exact integer arithmetic).
//   hipcc --offload-arch=gfx950 -O2 tools/probe_mx_fp8.hip -o tools/probe_mx_fp8 && ./tools/probe_mx_fp8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k_probe(const uint8_t* afr, const uint8_t* bfr, const uint8_t* asc, const uint8_t* bsc, float* out) {
    const int l = threadIdx.x;
    v8i a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = *reinterpret_cast<const int*>(afr + l * 32 + 4 * i);
        b[i] = *reinterpret_cast<const int*>(bfr + l * 32 + 4 * i);
    }
    v16f c;
    for (int i = 0; i < 16; ++i) c[i] = 0.f;
    const int sa = asc[l], sb = bsc[l];
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
    for (int i = 0; i < 16; ++i) out[l * 16 + i] = c[i];
}

static uint8_t e4m3(int v) {   // small integers |v| <= 8
    if (v == 0) return 0;
    const int s = v < 0 ? 0x80 : 0;
    int m = v < 0 ? -v : v;
    int e = 0;
    while ((m >> e) > 1) ++e;                 // m in [2^e, 2^(e+1))
    const int frac = ((m << 3) >> e) & 7;     // exact for these values
    return (uint8_t)(s | ((e + 7) << 3) | frac);
}

int main() {
    const int M = 32, N = 32, K = 64;
    std::vector<int> A(M * K), B(K * N);
    unsigned st = 12345;
    auto rnd = [&]() { st = st * 1103515245u + 12345u; return (int)((st >> 16) % 9) - 4; };
    for (auto& x : A) x = rnd();
    for (auto& x : B) x = rnd();
    // scale exponents per (row, kblock) / (col, kblock)
    int sA[32][2], sB[32][2];
    for (int r = 0; r < 32; ++r)
        for (int q = 0; q < 2; ++q) { sA[r][q] = (r * 3 + q * 5) % 4 - 1; sB[r][q] = (r * 7 + q) % 3 - 1; }
    // candidate k maps: lane half h, element j -> k
    auto kmap = [](int cand, int h, int j) {
        if (cand == 0) return 32 * h + j;                                   // contiguous blocks
        if (cand == 1) return j < 16 ? 16 * h + j : 32 + 16 * h + (j - 16); // interleaved 16s
        return 8 * h + (j % 8) + 16 * (j / 8);                              // interleaved 8s
    };
    for (int cand = 0; cand < 3; ++cand) {
        std::vector<uint8_t> af(64 * 32), bf(64 * 32), as(64), bs(64);
        for (int l = 0; l < 64; ++l) {
            const int r = l & 31, h = l >> 5;
            for (int j = 0; j < 32; ++j) {
                const int k = kmap(cand, h, j);
                af[l * 32 + j] = e4m3(A[r * K + k]);
                bf[l * 32 + j] = e4m3(B[k * N + r]);
            }
            as[l] = (uint8_t)(127 + sA[r][h]);
            bs[l] = (uint8_t)(127 + sB[r][h]);
        }
        uint8_t *da, *db, *dsa, *dsb;
        float* dout;
        hipMalloc(&da, 2048); hipMalloc(&db, 2048); hipMalloc(&dsa, 64); hipMalloc(&dsb, 64);
        hipMalloc(&dout, 64 * 16 * 4);
        hipMemcpy(da, af.data(), 2048, hipMemcpyHostToDevice);
        hipMemcpy(db, bf.data(), 2048, hipMemcpyHostToDevice);
        hipMemcpy(dsa, as.data(), 64, hipMemcpyHostToDevice);
        hipMemcpy(dsb, bs.data(), 64, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dout);
        std::vector<float> out(64 * 16);
        hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
        // expected with the scale of the k-block the element belongs to (block = k / 32)
        double maxerr = 0;
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 16; ++i) {
                const int col = l & 31, row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
                double ref = 0;
                for (int k = 0; k < K; ++k)
                    ref += A[row * K + k] * B[k * N + col] * std::ldexp(1.0, sA[row][k / 32] + sB[col][k / 32]);
                maxerr = std::fmax(maxerr, std::fabs(ref - out[l * 16 + i]));
            }
        std::printf("candidate %d: max |err| = %g%s\n", cand, maxerr, maxerr == 0 ? "  <-- MATCH" : "");
        hipFree(da); hipFree(db); hipFree(dsa); hipFree(dsb); hipFree(dout);
    }
    return 0;
}
