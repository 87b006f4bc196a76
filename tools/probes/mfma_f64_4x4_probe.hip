// Probe: lane layout and arithmetic of v_mfma_f64_4x4x4_4b_f64 (4 blocks of D(4x4) += A(4x4) B(4x4)).
// Checks the lane map against a k-ascending fma chain (and an unfused chain) on random data.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__global__ void k(const double* A, const double* B, const double* C, double* D, int ntile)
{
    const int l = threadIdx.x, t = blockIdx.x;
    if (t >= ntile) return;
    double acc = C[t * 64 + l];
    acc = __builtin_amdgcn_mfma_f64_4x4x4f64(A[t * 64 + l], B[t * 64 + l], acc, 0, 0, 0);
    D[t * 64 + l] = acc;
}

int main()
{
    const int ntile = 2048;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::vector<double> A(ntile * 64), B(ntile * 64), C(ntile * 64), D(ntile * 64);
    for (auto& x : A) x = u(g);
    for (auto& x : B) x = u(g);
    for (auto& x : C) x = u(g);
    double *dA, *dB, *dC, *dD;
    (void)hipMalloc(&dA, A.size() * 8); (void)hipMalloc(&dB, B.size() * 8);
    (void)hipMalloc(&dC, C.size() * 8); (void)hipMalloc(&dD, D.size() * 8);
    (void)hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(ntile), dim3(64), 0, 0, dA, dB, dC, dD, ntile);
    (void)hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost);
    // the map found with one-hot operands (mfma_f64_4x4_map.hip): block b = lane bits 2-3,
    // A[b][i][k] at lane 16 k + 4 b + i, B[b][k][j] at 16 k + 4 b + j, D[b][i][j] at 16 i + 4 b + j
    for (int ma = 0; ma < 1; ++ma)
        for (int mb = 0; mb < 1; ++mb)
            for (int md = 0; md < 1; ++md) {
                auto la = [&](int b, int i, int kk) { return 16 * kk + 4 * b + i; };
                auto lb = [&](int b, int kk, int j) { return 16 * kk + 4 * b + j; };
                auto ld = [&](int b, int i, int j) { return 16 * i + 4 * b + j; };
                long bad = 0, badu = 0, tot = 0;
                for (int t = 0; t < ntile; ++t)
                    for (int b = 0; b < 4; ++b)
                        for (int i = 0; i < 4; ++i)
                            for (int j = 0; j < 4; ++j) {
                                const int o = t * 64;
                                double f = C[o + ld(b, i, j)], q = f;
                                for (int kk = 0; kk < 4; ++kk) {
                                    f = std::fma(A[o + la(b, i, kk)], B[o + lb(b, kk, j)], f);
                                    volatile double p = A[o + la(b, i, kk)] * B[o + lb(b, kk, j)];
                                    q = q + p;
                                }
                                const double d = D[o + ld(b, i, j)];
                                if (std::memcmp(&f, &d, 8)) ++bad;
                                if (std::memcmp(&q, &d, 8)) ++badu;
                                ++tot;
                            }
                printf("fma-chain mismatches %ld / %ld, unfused %ld\n", bad, tot, badu);
            }
    return 0;
}
