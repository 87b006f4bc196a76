// selftest.hip -- device evaluation of the deterministic math and the noise stream, so the
// parity tests can check them bit for bit against the CPU oracle.
#include <hip/hip_runtime.h>

#include <vector>

#include "stomp_engine.h"
#include "stomp_math.h"

namespace {

__global__ void k_math(const double* x, int n, double* e, double* l, double* s, double* c, double* q)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    e[i] = stomp::det_exp(v);
    l[i] = v > 0.0 ? stomp::det_log(v) : 0.0;
    stomp::det_sincos(v, &s[i], &c[i]);
    q[i] = v >= 0.0 ? sqrt(v) : 0.0;
}

__global__ void k_normals(uint64_t seed, int it, int joint, int rollout, int n, double* z)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * p >= n) return;
    double z0, z1;
    stomp::normal_pair(seed, it, joint, rollout, p, &z0, &z1);
    z[2 * p] = z0;
    if (2 * p + 1 < n) z[2 * p + 1] = z1;
}

}  // namespace

extern "C" int stomp_device_selftest(const double* x, int32_t n, double* oe, double* ol, double* os, double* oc,
                                     double* oq)
{
    if (n <= 0) return 0;
    double* d = nullptr;
    if (hipMalloc(&d, sizeof(double) * n * 6) != hipSuccess) return STOMP_E_DEVICE;
    hipMemcpy(d, x, sizeof(double) * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_math, dim3((n + 255) / 256), dim3(256), 0, 0, d, n, d + n, d + 2 * n, d + 3 * n, d + 4 * n,
                       d + 5 * n);
    hipError_t st = hipDeviceSynchronize();
    if (st == hipSuccess) {
        hipMemcpy(oe, d + n, sizeof(double) * n, hipMemcpyDeviceToHost);
        hipMemcpy(ol, d + 2 * n, sizeof(double) * n, hipMemcpyDeviceToHost);
        hipMemcpy(os, d + 3 * n, sizeof(double) * n, hipMemcpyDeviceToHost);
        hipMemcpy(oc, d + 4 * n, sizeof(double) * n, hipMemcpyDeviceToHost);
        hipMemcpy(oq, d + 5 * n, sizeof(double) * n, hipMemcpyDeviceToHost);
    }
    hipFree(d);
    return st == hipSuccess ? 0 : STOMP_E_DEVICE;
}

extern "C" int stomp_device_normals(uint64_t seed, int32_t it, int32_t joint, int32_t rollout, int32_t n, double* z)
{
    if (n <= 0) return 0;
    double* d = nullptr;
    if (hipMalloc(&d, sizeof(double) * n) != hipSuccess) return STOMP_E_DEVICE;
    const int pairs = (n + 1) / 2;
    hipLaunchKernelGGL(k_normals, dim3((pairs + 63) / 64), dim3(64), 0, 0, seed, it, joint, rollout, n, d);
    hipError_t st = hipDeviceSynchronize();
    if (st == hipSuccess) hipMemcpy(z, d, sizeof(double) * n, hipMemcpyDeviceToHost);
    hipFree(d);
    return st == hipSuccess ? 0 : STOMP_E_DEVICE;
}
