// k_terms.hip -- the state-cost terms StompOptimizer::execute adds after the collision cost
// (stomp_optimizer.cpp:1107-1151), one workgroup per rollout, lane t = free waypoint t.
//
// Orientation constraints (:1107-1115): the FK frame of the constrained segment along its
// root-first path, then OrientationConstraintEvaluator::getCost (constraint_evaluator.cpp:80-114)
// with KDL's GetQuaternion and bullet's setRotation / getRPY restated as in the oracle.
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

// btMatrix3x3::setRotation(btQuaternion) (bullet LinearMath, double precision)
__device__ __forceinline__ void bt_from_quat(double x, double y, double z, double w, double* M)
{
    const double d = x * x + y * y + z * z + w * w;
    const double s = 2.0 / d;
    const double xs = x * s, ys = y * s, zs = z * s;
    const double wx = w * xs, wy = w * ys, wz = w * zs;
    const double xx = x * xs, xy = x * ys, xz = x * zs;
    const double yy = y * ys, yz = y * zs, zz = z * zs;
    M[0] = 1.0 - (yy + zz); M[1] = xy - wz; M[2] = xz + wy;
    M[3] = xy + wz; M[4] = 1.0 - (xx + zz); M[5] = yz - wx;
    M[6] = xz - wy; M[7] = yz + wx; M[8] = 1.0 - (xx + yy);
}

// KDL Rotation::GetQuaternion (orocos KDL 1.0): the non-trace branches compute s in single
// precision (`float s = 2.0 * sqrtf(...)`)
__device__ __forceinline__ void kdl_quat(const double* R, double* x, double* y, double* z, double* w)
{
    const double trace = R[0] + R[4] + R[8];
    if (trace > 1e-12) {
        const double s = 0.5 / sqrt(trace + 1.0);
        *w = 0.25 / s;
        *x = (R[7] - R[5]) * s;
        *y = (R[2] - R[6]) * s;
        *z = (R[3] - R[1]) * s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        const float s = (float)(2.0 * (double)__builtin_sqrtf((float)(1.0 + R[0] - R[4] - R[8])));
        *w = (R[7] - R[5]) / (double)s;
        *x = 0.25 * (double)s;
        *y = (R[1] + R[3]) / (double)s;
        *z = (R[2] + R[6]) / (double)s;
    } else if (R[4] > R[8]) {
        const float s = (float)(2.0 * (double)__builtin_sqrtf((float)(1.0 + R[4] - R[0] - R[8])));
        *w = (R[2] - R[6]) / (double)s;
        *x = (R[1] + R[3]) / (double)s;
        *y = 0.25 * (double)s;
        *z = (R[5] + R[7]) / (double)s;
    } else {
        const float s = (float)(2.0 * (double)__builtin_sqrtf((float)(1.0 + R[8] - R[0] - R[4])));
        *w = (R[3] - R[1]) / (double)s;
        *x = (R[2] + R[6]) / (double)s;
        *y = (R[5] + R[7]) / (double)s;
        *z = 0.25 * (double)s;
    }
}

// OrientationConstraintEvaluator::getCost (constraint_evaluator.cpp:80-114) on the segment
// rotation R; returns satisfied
__device__ bool oc_cost(const OcDev& o, const double* R, double* cost)
{
    double x, y, z, w, M[9], E[9];
    kdl_quat(R, &x, &y, &z, &w);
    bt_from_quat(x, y, z, w, M);
    const double* A = o.body_fixed ? o.ninv : M;   // header frame: M N^-1; body fixed: N^-1 M
    const double* B = o.body_fixed ? M : o.ninv;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            E[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    // btMatrix3x3::getRPY -> getEulerYPR(solution 1)
    const double pi = 3.1415926535897932384626433832795029;
    double roll, pitch, yaw;
    if (fabs(E[6]) >= 1.0) {
        yaw = 0.0;
        const double delta = det_atan2(E[0], E[2]);
        if (E[6] > 0.0) {
            pitch = pi / 2.0;
            roll = pitch + delta;
        } else {
            pitch = -pi / 2.0;
            roll = -pitch + delta;
        }
    } else {
        pitch = -det_asin(E[6]);
        double sp, cp;
        det_sincos(pitch, &sp, &cp);
        roll = det_atan2(E[7] / cp, E[8] / cp);
        yaw = det_atan2(E[3] / cp, E[0] / cp);
    }
    roll = fabs(roll);
    pitch = fabs(pitch);
    yaw = fabs(yaw);
    *cost = o.weight * (o.rw * roll + o.pw * pitch + o.yw * yaw);
    return !(roll > o.tol[0] || pitch > o.tol[1] || yaw > o.tol[2]);
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_terms(TermsModel m, TermsArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    if (a.stop && *a.stop) return;
    const int J = m.J, N = m.N, nc = m.nchain;
    double* Q = (double*)lds_raw;            // [3][J][N]
    double* F = Q + (size_t)3 * J * N;       // [nc][6][N]
    const int e = blockIdx.x, t = threadIdx.x;
    const bool extra = e == a.num_noisy;
    const double* traj = extra ? a.x_traj : a.traj + (long long)e * J * N;
    double* state = extra ? a.x_state : a.state + (long long)e * N;
    double* total = extra ? a.x_total : (a.total ? a.total + e : nullptr);
    uint8_t* cso = extra ? a.x_cs : (a.cs ? a.cs + e : nullptr);

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

    // orientation constraints on the waypoint's FK frames (stomp_optimizer.cpp:1107-1115); the
    // segment frame is composed root-first along its path, as the FK of every segment does
    double con = 0.0;
    int ok = 1;
    if (t < N) {
        for (int c = 0; c < m.noc; ++c) {
            const OcDev& o = m.oc[c];
            Frame Fr;
            for (int k = 0; k < o.path_len; ++k) {
                const DevSegment& sg = m.segs[o.path[k]];
                double st = 0.0, ct = 1.0;
                if (sg.q_index >= 0) det_sincos(Q[sg.q_index * N + t], &st, &ct);
                Frame nf;
                compose(sg, k == 0 ? nullptr : &Fr, st, ct, nf);
                Fr = nf;
            }
            double cc;
            if (!oc_cost(o, Fr.R, &cc)) ok = 0;
            con += cc;
        }
    }
    const int all_ok = __syncthreads_and(ok);

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
        if (a.tq_out && e == 0) a.tq_out[t] = tq;
    }
    __syncthreads();
    double* cst = F;   // the costs, for the total
    if (t < N) {
        const double c = (state[t] + m.w_con * con) + m.w_tq * tq;
        state[t] = c;
        cst[t] = c;
    }
    __syncthreads();
    if (t == 0 && total) {
        double s = 0.0;
        for (int k = 0; k < N; ++k) s += cst[k];
        *total = s;
    }
    if (t == 0 && cso) *cso = all_ok ? 1 : 0;
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
        if (lds > 64 * 1024) lds_opt_in((const void*)k_terms<128>, lds);
        hipLaunchKernelGGL((k_terms<128>), dim3(blocks), dim3(128), lds, s, m, a);
    } else {
        if (lds > 64 * 1024) lds_opt_in((const void*)k_terms<256>, lds);
        hipLaunchKernelGGL((k_terms<256>), dim3(blocks), dim3(256), lds, s, m, a);
    }
}

}  // namespace stomp
