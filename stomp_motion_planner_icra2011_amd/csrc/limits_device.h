// limits_device.h -- StompOptimizer::handleJointLimits (stomp_optimizer.cpp:562-616) for one wave
// holding one joint's row of the trajectory in registers (lane l: waypoints l, l + 64, l + 128,
// l + 192; N <= 256).  Used by the rollout kernel's joint-limit phase (k_cost.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace stomp {

// max of x over the 64 lanes of the wave (every lane active): DPP within rows of 16, then
// the four row results through scalar registers
__device__ __forceinline__ unsigned wave_max_u32(unsigned x)
{
    x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false));    // quad_perm 1,0,3,2
    x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false));    // quad_perm 2,3,0,1
    x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false));   // row_half_mirror
    x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false));   // row_mirror
    const unsigned a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 16);
    const unsigned c = __builtin_amdgcn_readlane(x, 32), d = __builtin_amdgcn_readlane(x, 48);
    return max(max(a, b), max(c, d));
}

// the violated waypoint a pass corrects (wave-uniform), -1 when none is left: the largest
// |amount| > 1e-6, the first index on ties (stomp_optimizer.cpp:574-593).  U: register slots per
// lane (waypoints lane + 64 u, u < U; N <= 64 U)
template <int U = 4>
__device__ __forceinline__ int jl_argmax(const double* v, int N, int lane, double jmin, double jmax)
{
    double cand = 0.0;   // absamt > 1e-6 > 0 marks a candidate
    int ci = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = lane + 64 * u;
        if (t < N) {
            const double x = v[u];
            double absamt = 0.0;
            if (x > jmax) absamt = fabs(jmax - x);
            else if (x < jmin) absamt = fabs(jmin - x);
            if (absamt > 1e-6 && absamt > cand) { cand = absamt; ci = t; }   // t ascending per lane
        }
    }
    // wave argmax, first index on ties: the bits of a non-negative double order like
    // the value, so the max is two 32-bit DPP reductions; ballots pick the least t
    const unsigned long long key = (unsigned long long)__double_as_longlong(cand);
    const unsigned hi = (unsigned)(key >> 32), lo = (unsigned)key;
    const unsigned mh = wave_max_u32(hi);
    const unsigned ml = wave_max_u32(hi == mh ? lo : 0u);
    if ((mh | ml) == 0u) return -1;   // no violation left (wave-uniform)
    const bool match = hi == mh && lo == ml;
    int cm = 0;
    for (int blk = 0; blk * 64 < N; ++blk) {
        const unsigned long long b = __ballot(match && (ci >> 6) == blk);
        if (b) { cm = blk * 64 + __ffsll((long long)b) - 1; break; }
    }
    return cm;
}

// row += (amount / Q(cm, cm)) Q[:, cm] (stomp_optimizer.cpp:596-606); qv: this lane's entries of
// column cm, qd = Q(cm, cm)
template <int U = 4>
__device__ __forceinline__ void jl_apply(double* v, int N, int lane, int cm, double jmin, double jmax,
                                         const double* qv, double qd)
{
    double vu = v[0];
#pragma unroll
    for (int u = 1; u < U; ++u)
        if ((cm >> 6) == u) vu = v[u];   // uniform select
    const unsigned long long bits = (unsigned long long)__double_as_longlong(vu);
    const unsigned vlo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)bits, cm & 63);
    const unsigned vhi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(bits >> 32), cm & 63);
    const double x = __longlong_as_double((long long)(((unsigned long long)vhi << 32) | vlo));
    const double amount = x > jmax ? jmax - x : jmin - x;
    const double mult = amount / qd;
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (lane + 64 * u < N) v[u] += mult * qv[u];
}

}  // namespace stomp
