// Probe: arithmetic of v_mfma_f64_16x16x4_f64 on this GPU.  For random A (16x4), B (4x16),
// C (16x16) compare D with CPU models: (a) fma chain over k ascending, (b) fma chain
// descending, (c) products and sums with one rounding each (k ascending), (d) the exact
// value of C + sum_k A B rounded once (__float128).  Prints mismatch counts per model.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_mfma(const double* A, const double* B, const double* C, double* D, int ntile)
{
    const int l = threadIdx.x, t = blockIdx.x;
    if (t >= ntile) return;
    const double* a = A + t * 64;
    const double* b = B + t * 64;
    const double* c = C + t * 256;
    const double av = a[(l & 15) * 4 + (l >> 4)];    // A[i = l & 15][k = l >> 4], A row-major 16x4
    const double bv = b[(l >> 4) * 16 + (l & 15)];   // B[k = l >> 4][j = l & 15], B row-major 4x16
    d4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = c[((l >> 4) + 4 * r) * 16 + (l & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[t * 256 + ((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

int main(int argc, char** argv)
{
    const int ntile = argc > 1 ? atoi(argv[1]) : 4096;
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::uniform_int_distribution<int> ex(-30, 30);
    auto rnd = [&]() { return std::ldexp(u(g), ex(g) / 6); };
    std::vector<double> A(ntile * 64), B(ntile * 64), C(ntile * 256), D(ntile * 256);
    for (auto& x : A) x = rnd();
    for (auto& x : B) x = rnd();
    for (auto& x : C) x = rnd();
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 8); hipMalloc(&dB, B.size() * 8); hipMalloc(&dC, C.size() * 8); hipMalloc(&dD, D.size() * 8);
    hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(ntile), dim3(64), 0, 0, dA, dB, dC, dD, ntile);
    hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost);
    long bad[4] = {0, 0, 0, 0}, total = 0;
    for (int t = 0; t < ntile; ++t)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                const double* a = &A[t * 64 + i * 4];
                const double* b = &B[t * 64];
                const double c = C[t * 256 + i * 16 + j], d = D[t * 256 + i * 16 + j];
                double m0 = c, m1 = c, m2 = c;
                for (int k = 0; k < 4; ++k) m0 = std::fma(a[k], b[k * 16 + j], m0);
                for (int k = 3; k >= 0; --k) m1 = std::fma(a[k], b[k * 16 + j], m1);
                for (int k = 0; k < 4; ++k) {
                    volatile double p = a[k] * b[k * 16 + j];
                    m2 = m2 + p;
                }
                __float128 q = c;
                for (int k = 0; k < 4; ++k) q += (__float128)a[k] * (__float128)b[k * 16 + j];
                const double m3 = (double)q;
                const double ms[4] = {m0, m1, m2, m3};
                for (int s = 0; s < 4; ++s)
                    if (std::memcmp(&ms[s], &d, 8) != 0) ++bad[s];
                ++total;
            }
    printf("outputs %ld  mismatches: fma-asc %ld  fma-desc %ld  unfused-asc %ld  exact-once %ld\n", total, bad[0],
           bad[1], bad[2], bad[3]);
    return 0;
}
