// Probe: lane map of v_mfma_f64_4x4x4_4b_f64 with one-hot A: for each A lane a, which D lanes
// receive which B lane's value.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(double* D)
{
    const int l = threadIdx.x, a = blockIdx.x;
    const double av = l == a ? 1.0 : 0.0, bv = 1000.0 + l;
    double acc = 0.0;
    acc = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv, acc, 0, 0, 0);
    D[a * 64 + l] = acc;
}

int main()
{
    double* dD;
    (void)hipMalloc(&dD, 64 * 64 * 8);
    hipLaunchKernelGGL(k, dim3(64), dim3(64), 0, 0, dD);
    static double D[64 * 64];
    (void)hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
    for (int a = 0; a < 64; ++a) {
        printf("A lane %2d ->", a);
        for (int l = 0; l < 64; ++l)
            if (D[a * 64 + l] != 0.0) printf(" D%d=B%d", l, (int)(D[a * 64 + l] - 1000.0));
        printf("\n");
    }
    return 0;
}
