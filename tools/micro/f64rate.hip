// fp64 VALU issue rate and dependent latency on one CU (diagnostic microbenchmark)
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CHAINS>
__global__ void k(double* out, long long* cyc, int iters, double a, double b)
{
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3 + c;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = x[c] * a + b;   // v_mul + v_add (no contraction)
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int CH>
void run(int threads)
{
    double* o; long long* c; hipMalloc(&o, 1 << 20); hipMalloc(&c, 4096);
    const int iters = 4096;
    hipLaunchKernelGGL(k<CH>, dim3(1), dim3(threads), 0, 0, o, c, iters, 1.0000001, 1e-9);
    hipLaunchKernelGGL(k<CH>, dim3(1), dim3(threads), 0, 0, o, c, iters, 1.0000001, 1e-9);
    long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    double ops = 2.0 * iters * CH;   // per lane-chain: mul + add
    printf("threads %4d chains %2d: %.2f cycles per wave-instruction per wave (%lld cycles)\n", threads, CH,
           (double)h / ops, h);
    hipFree(o); hipFree(c);
}
int main()
{
    run<1>(64); run<4>(64); run<8>(64); run<16>(64);
    run<8>(256); run<8>(512); run<8>(1024); run<16>(1024);
    return 0;
}
