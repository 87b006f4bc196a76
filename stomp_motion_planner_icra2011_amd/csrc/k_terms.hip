// k_terms.hip -- the state-cost terms StompOptimizer::execute adds after the collision cost
// (stomp_optimizer.cpp:1107-1151), one workgroup per rollout, lane t = free waypoint t.
//
// Torque term (:1117-1142, StompOptimizer::getTorques :1033-1061): q at row t of the
// joint-limited group trajectory, q-dot / q-ddot by the 7-tap rules of
// StompTrajectory::getJointVelocities / getJointAccelerations (stomp_trajectory.h:286-310),
// then KDL::ChainIdSolver_RNE::CartToJnt (3rd party; constructed at
// stomp_robot_model.cpp:185-189) restated as in oracle/stomp_oracle.c so_inverse_dynamics:
// outward sweep of segment twists / accelerations, inward sweep of wrenches, and
// tq = sum_j |tau_j|.  Finally costs(t) = (state + w_con * con) + w_tq * tq, where k_rollout
// left state = w_obs * collision cost (:1148-1151), and the total (:1155).
//
// LDS: Q = [3][J][N] (q, q-dot, q-ddot; tau overwrites q-dot in the inward sweep) and the
// forward-sweep wrenches F = [nchain][6][N], lane-contiguous so a wave's accesses hit
// consecutive banks.  The per-segment table (ChainSeg) is read with wave-uniform addresses
// (scalar loads).
#include "device_fk.h"

namespace stomp {

namespace {

struct Twist {
    double v[3], w[3];   // (linear, angular)
};

__device__ __forceinline__ void vcross(const double* a, const double* b, double* c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ void rot_mul_v(const double* R, const double* v, double* o)
{
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = R[3 * i + 0] * v[0] + R[3 * i + 1] * v[1] + R[3 * i + 2] * v[2];
}

__device__ __forceinline__ void rot_inv_mul_v(const double* R, const double* v, double* o)
{
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = R[0 + i] * v[0] + R[3 + i] * v[1] + R[6 + i] * v[2];
}

// Frame::Inverse(Twist): (R^T (v - p x w), R^T w)
__device__ __forceinline__ void frame_inv_twist(const double* R, const double* p, const Twist& t, Twist& o)
{
    double pw[3], d[3];
    vcross(p, t.w, pw);
#pragma unroll
    for (int k = 0; k < 3; ++k) d[k] = t.v[k] - pw[k];
    rot_inv_mul_v(R, d, o.v);
    rot_inv_mul_v(R, t.w, o.w);
}

// RigidBodyInertia * Twist: force m v - h x w, torque I w + h x v
__device__ __forceinline__ void rbi_mul(const ChainSeg& c, const Twist& t, double* f, double* n)
{
    double hw[3], hv[3], Iw[3];
    vcross(c.h, t.w, hw);
    vcross(c.h, t.v, hv);
    rot_mul_v(c.I, t.w, Iw);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        f[k] = c.m * t.v[k] - hw[k];
        n[k] = Iw[k] + hv[k];
    }
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_terms(TermsModel m, TermsArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    const int J = m.J, N = m.N, nc = m.nchain;
    double* Q = (double*)lds_raw;            // [3][J][N]
    double* F = Q + (size_t)3 * J * N;       // [nc][6][N]
    const int e = blockIdx.x, t = threadIdx.x;
    const bool extra = e == a.num_noisy;
    const double* traj = extra ? a.x_traj : a.traj + (long long)e * J * N;
    double* state = extra ? a.x_state : a.state + (long long)e * N;
    double* total = extra ? a.x_total : (a.total ? a.total + e : nullptr);

    // q, q-dot, q-ddot for every (joint, waypoint): padding rows are start / goal
    for (int idx = t; idx < J * N; idx += BLOCK) {
        const int j = idx / N, tt = idx - j * N;
        double x[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const int r = tt + k - 3;
            x[k] = r < 0 ? m.start[j] : (r >= N ? m.goal[j] : traj[j * N + r]);
        }
        double qd = 0.0, qdd = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            qd += m.cv[k] * x[k];
            qdd += m.ca[k] * x[k];
        }
        Q[idx] = x[3];
        Q[J * N + idx] = qd;
        Q[2 * J * N + idx] = qdd;
    }
    __syncthreads();

    double tq = 0.0;
    if (t < N && m.torque) {
        // outward sweep (KDL ChainIdSolver_RNE::CartToJnt, "Sweep from root to leaf")
        const Twist ag = {{-m.g[0], -m.g[1], -m.g[2]}, {0.0, 0.0, 0.0}};
        Twist v, acc;
        for (int i = 0; i < nc; ++i) {
            const ChainSeg& c = m.chain[i];
            const int j = c.seg.q_index;
            double qv = 0.0, qdv = 0.0, qddv = 0.0;
            double S[3] = {0.0, 0.0, 0.0};   // angular part of the unit twist; linear part 0
            if (j >= 0) {
                qv = Q[j * N + t]; qdv = Q[J * N + j * N + t]; qddv = Q[2 * J * N + j * N + t];
                S[0] = c.seg.axis[0]; S[1] = c.seg.axis[1]; S[2] = c.seg.axis[2];
            }
            double st = 0.0, ct = 1.0;
            if (j >= 0) det_sincos(qv, &st, &ct);
            Frame X;
            compose(c.seg, nullptr, st, ct, X);
            Twist vj, xv, xa;
#pragma unroll
            for (int k = 0; k < 3; ++k) { vj.v[k] = 0.0 * qdv; vj.w[k] = S[k] * qdv; }
            if (i == 0) {
                v = vj;
                frame_inv_twist(X.R, X.p, ag, xa);
            } else {
                frame_inv_twist(X.R, X.p, v, xv);
                frame_inv_twist(X.R, X.p, acc, xa);
#pragma unroll
                for (int k = 0; k < 3; ++k) { v.v[k] = xv.v[k] + vj.v[k]; v.w[k] = xv.w[k] + vj.w[k]; }
            }
            // v x vj (Twist * Twist)
            double c1[3], c2[3], cw[3];
            vcross(v.w, vj.v, c1);
            vcross(v.v, vj.w, c2);
            vcross(v.w, vj.w, cw);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                acc.v[k] = xa.v[k] + 0.0 * qddv + (c1[k] + c2[k]);
                acc.w[k] = xa.w[k] + S[k] * qddv + cw[k];
            }
            // f = I a + v x* (I v)
            double fa[3], na[3], fv[3], nv[3], x1[3], x2[3], x3[3];
            rbi_mul(c, acc, fa, na);
            rbi_mul(c, v, fv, nv);
            double* Fi = F + (size_t)i * 6 * N + t;
            vcross(v.w, fv, x1);   // force:  w x f
            vcross(v.w, nv, x2);   // torque: w x n + v x f
            vcross(v.v, fv, x3);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                Fi[k * N] = fa[k] + x1[k];
                Fi[(3 + k) * N] = na[k] + (x2[k] + x3[k]);
            }
        }
        // inward sweep: tau_i = S_i . f_i, f_{i-1} += X_i f_i; tau lands in the q-dot rows
        double fo[3], no[3];   // running f_{i} (the stored one plus the children's)
        for (int i = nc - 1; i >= 0; --i) {
            const ChainSeg& c = m.chain[i];
            const double* Fi = F + (size_t)i * 6 * N + t;
            double fi[3], ni[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                fi[k] = Fi[k * N];
                ni[k] = Fi[(3 + k) * N];
            }
            if (i != nc - 1) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { fi[k] += fo[k]; ni[k] += no[k]; }
            }
            const int j = c.seg.q_index;
            if (j >= 0) {
                const double* ax = c.seg.axis;
                Q[J * N + j * N + t] = (0.0 * fi[0] + 0.0 * fi[1] + 0.0 * fi[2]) +
                                       (ax[0] * ni[0] + ax[1] * ni[1] + ax[2] * ni[2]);
            }
            if (i != 0) {
                double st = 0.0, ct = 1.0;
                if (j >= 0) det_sincos(Q[j * N + t], &st, &ct);
                Frame X;
                compose(c.seg, nullptr, st, ct, X);
                double rn[3], pf[3];
                rot_mul_v(X.R, fi, fo);
                rot_mul_v(X.R, ni, rn);
                vcross(X.p, fo, pf);
#pragma unroll
                for (int k = 0; k < 3; ++k) no[k] = rn[k] + pf[k];
            }
        }
        for (int j = 0; j < J; ++j) tq += fabs(Q[J * N + j * N + t]);
    }
    __syncthreads();
    double* cst = F;   // the costs, for the total
    if (t < N) {
        const double c = (state[t] + m.w_con * 0.0) + m.w_tq * tq;
        state[t] = c;
        cst[t] = c;
    }
    __syncthreads();
    if (t == 0 && total) {
        double s = 0.0;
        for (int k = 0; k < N; ++k) s += cst[k];
        *total = s;
    }
}

}  // namespace

size_t terms_lds_bytes(const TermsModel& m)
{
    const size_t a = (size_t)(3 * m.J + 6 * m.nchain) * m.N * sizeof(double);
    return a > (size_t)m.N * sizeof(double) ? a : (size_t)m.N * sizeof(double);
}

void launch_terms(const TermsModel& m, const TermsArgs& a, hipStream_t s)
{
    const int blocks = a.num_noisy + (a.x_traj ? 1 : 0);
    if (blocks <= 0) return;
    const size_t lds = terms_lds_bytes(m);
    if (m.N <= 128) {
        static size_t raised = 0;
        if (lds > 64 * 1024 && lds > raised) {
            (void)hipFuncSetAttribute((const void*)k_terms<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            raised = lds;
        }
        hipLaunchKernelGGL((k_terms<128>), dim3(blocks), dim3(128), lds, s, m, a);
    } else {
        static size_t raised = 0;
        if (lds > 64 * 1024 && lds > raised) {
            (void)hipFuncSetAttribute((const void*)k_terms<256>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            raised = lds;
        }
        hipLaunchKernelGGL((k_terms<256>), dim3(blocks), dim3(256), lds, s, m, a);
    }
}

}  // namespace stomp
