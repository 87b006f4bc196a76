// device_fk.h -- device-side kinematics, distance-field lookup and potential.
//
// KDL conventions restated (orocos KDL is third party, reached from
// treefksolverjointposaxis_partial.cpp:125,168 and stomp_collision_point.h:138-141):
// Rotation::Rot2, Rotation*Rotation, Frame*Frame and Frame*Vector, each sum
// evaluated left to right with one rounding per operation.
#pragma once

#include "kernels.h"
#include "stomp_math.h"

namespace stomp {

struct Frame {
    double R[9];
    double p[3];
};

__device__ __forceinline__ void rotmul(const double* A, const double* B, double* C)
{
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// the pose rotation rot * Rot2(axis, q) of a joint segment (q_index >= 0), (st, ct) = (sin q, cos q)
__device__ __forceinline__ void pose_rotation(const DevSegment& sg, double st, double ct, double* R)
{
    const double* a = sg.axis;
    const double vt = 1.0 - ct;
    const double m_vt_0 = vt * a[0], m_vt_1 = vt * a[1], m_vt_2 = vt * a[2];
    const double m_st_0 = a[0] * st, m_st_1 = a[1] * st, m_st_2 = a[2] * st;
    const double m_vt_0_1 = m_vt_0 * a[1], m_vt_0_2 = m_vt_0 * a[2], m_vt_1_2 = m_vt_1 * a[2];
    double Rq[9];
    Rq[0] = ct + m_vt_0 * a[0];
    Rq[1] = -m_st_2 + m_vt_0_1;
    Rq[2] = m_st_1 + m_vt_0_2;
    Rq[3] = m_st_2 + m_vt_0_1;
    Rq[4] = ct + m_vt_1 * a[1];
    Rq[5] = -m_st_0 + m_vt_1_2;
    Rq[6] = -m_st_1 + m_vt_0_2;
    Rq[7] = m_st_0 + m_vt_1_2;
    Rq[8] = ct + m_vt_2 * a[2];
    if (sg.rot_identity) {   // rot * Rq with rot = 1 is Rq (up to the sign of zeros; the oracle skips it too)
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = Rq[k];
    } else {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                R[3 * i + j] = sg.rot[3 * i + 0] * Rq[0 + j] + sg.rot[3 * i + 1] * Rq[3 + j] + sg.rot[3 * i + 2] * Rq[6 + j];
    }
}

// out = parent * Frame(rot, trans) * Frame(Rot2(axis, q), 0), with (st, ct) = (sin q, cos q)
// precomputed; parent == nullptr is the identity (root segment).  out must not alias parent.
__device__ __forceinline__ void compose(const DevSegment& sg, const Frame* parent, double st, double ct, Frame& out)
{
    Frame pose;
    if (sg.q_index >= 0) {
        const double* a = sg.axis;
        const double vt = 1.0 - ct;
        const double m_vt_0 = vt * a[0], m_vt_1 = vt * a[1], m_vt_2 = vt * a[2];
        const double m_st_0 = a[0] * st, m_st_1 = a[1] * st, m_st_2 = a[2] * st;
        const double m_vt_0_1 = m_vt_0 * a[1], m_vt_0_2 = m_vt_0 * a[2], m_vt_1_2 = m_vt_1 * a[2];
        double Rq[9];
        Rq[0] = ct + m_vt_0 * a[0];
        Rq[1] = -m_st_2 + m_vt_0_1;
        Rq[2] = m_st_1 + m_vt_0_2;
        Rq[3] = m_st_2 + m_vt_0_1;
        Rq[4] = ct + m_vt_1 * a[1];
        Rq[5] = -m_st_0 + m_vt_1_2;
        Rq[6] = -m_st_1 + m_vt_0_2;
        Rq[7] = m_st_0 + m_vt_1_2;
        Rq[8] = ct + m_vt_2 * a[2];
        if (sg.rot_identity) {   // rot * Rq with rot = 1 is Rq (up to the sign of zeros; the oracle skips it too)
#pragma unroll
            for (int k = 0; k < 9; ++k) pose.R[k] = Rq[k];
        } else {
            rotmul(sg.rot, Rq, pose.R);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) pose.R[k] = sg.rot[k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) pose.p[k] = sg.trans[k];
    if (!parent) {
        out = pose;
        return;
    }
    if (sg.q_index < 0 && sg.rot_identity) {   // parent * 1
#pragma unroll
        for (int k = 0; k < 9; ++k) out.R[k] = parent->R[k];
    } else {
        rotmul(parent->R, pose.R, out.R);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
        out.p[i] = parent->R[3 * i + 0] * pose.p[0] + parent->R[3 * i + 1] * pose.p[1] +
                   parent->R[3 * i + 2] * pose.p[2] + parent->p[i];
}

__device__ __forceinline__ void apply(const double* R, const double* P, const double* v, double* o)
{
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = R[3 * i + 0] * v[0] + R[3 * i + 1] * v[1] + R[3 * i + 2] * v[2] + P[i];
}

// One FK program step (see FkOp).  Saved-frame moves are per-element selects under a
// wave-uniform branch: branchy assignment lets the optimiser sink the stores through a
// pointer select and send the frames to scratch.
__device__ __forceinline__ void fk_op(const DevSegment& sg, int base, int save, double st, double ct, Frame& C,
                                      Frame& S0, Frame& S1)
{
    Frame nf;
    if (base == kBaseChain) {
        compose(sg, &C, st, ct, nf);
    } else if (base == kBaseRoot) {
        compose(sg, nullptr, st, ct, nf);
    } else {
        Frame P;
#pragma unroll
        for (int k = 0; k < 9; ++k) P.R[k] = base == 0 ? S0.R[k] : S1.R[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) P.p[k] = base == 0 ? S0.p[k] : S1.p[k];
        compose(sg, &P, st, ct, nf);
    }
    C = nf;
    if (save >= 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            S0.R[k] = save == 0 ? C.R[k] : S0.R[k];
            S1.R[k] = save == 1 ? C.R[k] : S1.R[k];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            S0.p[k] = save == 0 ? C.p[k] : S0.p[k];
            S1.p[k] = save == 1 ? C.p[k] : S1.p[k];
        }
    }
}

// distance_field::getDistanceGradient cell rule (3rd party; call site stomp_collision_space.h:190):
// nearest cell round((p - origin) * (1/res)); cells with an index < 1 or >= n-1 read 0.
// Branch-free so a lane's gathers can all be in flight together: an out-of-range lane
// loads cell 0 and discards it.
// The cell rule in few operations.  With u = (p - o) * (1/res):
//   round(u) >= 1      <=>  u >= 0.5
//   round(u) <= n - 2  <=>  u < n - 1.5        (n - 1.5 is exact)
// and for u >= 0.5, floor(u + 0.5) == round(u): u + 0.5 is exact below 2^52 except when it
// crosses into the next binade, and there it rounds onto the same integer round(u) gives (the
// one value where floor(u + 0.5) != round(u) for u >= 0, u = 0.5 - 2^-54, is below 0.5 and
// rejected by the range test).  So the range test moves onto u and each axis costs sub, mul,
// two compares, add and floor.
// The voxel index of p (cell 0 when p reads distance 0: ok = false).  After u = (p - o) * (1/res)
// in double, the rest is integer work: for u >= 0.5, trunc(u + 0.5) = floor(u + 0.5) = round(u)
// (see above), and the range test moves onto the integer: round(u) in [1, n - 2].  A u below 0.5
// truncates to 0 or below (or saturates at INT_MIN), one past the top to n - 1 or above (or
// INT_MAX), and NaN converts to 0: every one of them fails the test, as it fails on u.
// BRICK: the engine's 4^3 brick layout (DevModel::brick) instead of [x][y][z]; a template
// parameter, not a branch, so the lookups stay one straight-line block
template <bool BRICK>
__device__ __forceinline__ unsigned sdf_cell(const DevModel& m, const double* __restrict__ p, bool& ok)
{
    const int ix = (int)((p[0] - m.ox) * m.inv_res + 0.5);
    const int iy = (int)((p[1] - m.oy) * m.inv_res + 0.5);
    const int iz = (int)((p[2] - m.oz) * m.inv_res + 0.5);
    ok = ix >= 1 && iy >= 1 && iz >= 1 && ix <= m.nx - 2 && iy <= m.ny - 2 && iz <= m.nz - 2;
    unsigned cell;
    if constexpr (BRICK) {
        const unsigned b = (((unsigned)ix >> 2) * (unsigned)m.nby + ((unsigned)iy >> 2)) * (unsigned)m.nbz +
                           ((unsigned)iz >> 2);
        cell = (b << 6) | (((unsigned)ix & 3u) << 4) | (((unsigned)iy & 3u) << 2) | ((unsigned)iz & 3u);
    } else {
        cell = ((unsigned)ix * (unsigned)m.ny + (unsigned)iy) * (unsigned)m.nz + (unsigned)iz;
    }
    return ok ? cell : 0u;
}

// Returns the voxel's squared cell distance d2 (0 outside: distance 0).
template <bool BRICK>
__device__ __forceinline__ unsigned sdf_d2(const DevModel& m, const double* __restrict__ p)
{
    bool ok;
    const unsigned v = m.sdf[sdf_cell<BRICK>(m, p, ok)];
    return ok ? v : 0u;
}

// the same with the layout chosen at run time (setup kernels)
__device__ __forceinline__ unsigned sdf_d2(const DevModel& m, const double* __restrict__ p)
{
    return m.brick ? sdf_d2<true>(m, p) : sdf_d2<false>(m, p);
}

// PropagationDistanceField::getDistance: sqrt_table_[d2], the table made as sqrt(double(i)) * resolution
__device__ __forceinline__ double sdf_metres(const DevModel& m, unsigned d2)
{
    return sqrt((double)d2) * m.res;
}

// StompCollisionSpace::getCollisionPointPotentialGradient (stomp_collision_space.h:193-228)
__device__ __forceinline__ double potential(const DevSphere& s, double dist)
{
    const double d = dist - s.radius;
    if (d >= s.clearance) return 0.0;
    if (d >= 0.0) {
        const double diff = d - s.clearance;
        const double gm = diff * s.inv_clearance;
        return 0.5 * gm * diff;
    }
    return -d + 0.5 * s.clearance;
}

}  // namespace stomp
