// update_device.h -- one tile of theta += M u (policy_improvement.cpp:380, covariant_trajectory_policy
// .cpp:318-323): 16 outputs of one joint.  Used by k_update, a launch of its own (the variant that
// applied the update in blocks of the next rollout launch was measured and rejected).
#pragma once

#include <hip/hip_runtime.h>

namespace stomp {

constexpr int kUpdCols = 16;                                  // outputs per tile
constexpr int kUpdLoads = (128 * kUpdCols + 255) / 256;       // 8-byte loads per lane per batch (one batch while N <= 128)

// LDS of one tile: M^T's 16 columns of every row, then u
__host__ __device__ inline size_t update_tile_lds_bytes(int N) { return ((size_t)N * kUpdCols + N) * sizeof(double); }

// Tile (c0 .. c0 + 15, joint d) by a 256-lane workgroup: the tile's columns of every M^T row staged
// in LDS with all the loads in flight at once, then 16 lanes run the k-ascending chain out of LDS
// (one rounding per multiply and per add, exactly N terms).  u_all (multi-GPU): u summed over the
// gathered block partials in block order.  stopped: nothing is written.  delta: delta = M u and
// theta untouched.  Returns after the tile's stores are issued (lanes >= 16 return earlier).
__device__ __forceinline__ void update_tile(int J, int N, const double* MT, const double* u, const double* u_all,
                                            int nb_total, double* theta, bool stopped, double* delta, int c0, int d,
                                            double* ms, int tid)
{
    double* us = ms + (size_t)N * kUpdCols;
    const int nc = min(kUpdCols, N - c0);
    const size_t JN = (size_t)J * N;
    const int total = N * kUpdCols;
    for (int f0 = 0; f0 < total; f0 += kUpdLoads * 256) {
        double v[kUpdLoads];
#pragma unroll
        for (int q = 0; q < kUpdLoads; ++q) {
            // clamped addresses: every lane loads, the stores below keep the rows that exist
            const int f = f0 + tid + q * 256;
            const int k = min(f / kUpdCols, N - 1), c = min(f % kUpdCols, nc - 1);
            v[q] = MT[(size_t)k * N + c0 + c];
        }
        if (tid < N) {
            double uv = 0.0;
            if (f0 == 0) {
                if (u_all) {
                    for (int b = 0; b < nb_total; ++b) uv += u_all[(size_t)b * JN + (size_t)d * N + tid];
                } else {
                    uv = u[(size_t)d * N + tid];
                }
                us[tid] = uv;
            }
        }
#pragma unroll
        for (int q = 0; q < kUpdLoads; ++q) {
            const int f = f0 + tid + q * 256;
            if (f < total) ms[f] = v[q];
        }
    }
    __syncthreads();
    if (tid >= kUpdCols) return;
    double s = 0.0;
    int k = 0;
    // 32 terms' LDS reads in flight per wait (8 at a time: cfg2 16.27k -> 16.48k it/s,
    // profiles/ab/r6_update_batch.txt)
    constexpr int kB = 32;
    for (; k + kB <= N; k += kB) {
        double a[kB], x[kB];
#pragma unroll
        for (int q = 0; q < kB; ++q) {
            a[q] = ms[(k + q) * kUpdCols + tid];
            x[q] = us[k + q];
        }
#pragma unroll
        for (int q = 0; q < kB; ++q) s += a[q] * x[q];
    }
    for (; k < N; ++k) s += ms[k * kUpdCols + tid] * us[k];
    if (tid >= nc || stopped) return;
    const int i = c0 + tid;
    if (delta) delta[(size_t)d * N + i] = s;   // improvePolicy's update alone (PolicyImprovement API)
    else theta[(size_t)d * N + i] += 1.0 * s;
}

}  // namespace stomp
