/*
 * oracle/stomp_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of the STOMP hot
 * path (see stomp_oracle.h for scope and the "parity unpinned" note).  All paths
 * are relative to /root/reference/stomp_motion_planner/.
 *
 * Floating-point contract: every sum is sequential in the index order the
 * reference's loops use, one rounding per operation (-ffp-contract=off), except the
 * noise path's two dense products (L z, M eps), which round once per multiply-add
 * (matvec_fma); the dense ("reference structure") and banded/triangular evaluations
 * agree bit for bit (the skipped terms are exact zeros).  Sums over rollouts use a fixed
 * blocked order (blocks of cfg.sum_block consecutive rollouts, each summed
 * sequentially from 0.0, block partials then summed sequentially from 0.0);
 * for K <= sum_block this is exactly the reference's sequential order
 * (policy_improvement.cpp:352-358, 376-379).
 *
 * cfg.ref_arith = 1 drops the two engine-contract choices and follows the reference's
 * written order everywhere: L z and M eps non-fused and k ascending over the dense matrix
 * (multivariate_gaussian.h:93, policy_improvement.cpp:477), and the rollout sums of P and
 * eps * P sequential over all K (policy_improvement.cpp:352-358, 376-379).
 * cfg.ref_arith = 2 also sums VectorXd::sum() (Rollout::getCost, policy_improvement.cpp:149-156;
 * last_trajectory_cost_ = costs.sum(), stomp_optimizer.cpp:1155) as Eigen 2's SSE2 packet
 * reduction would: two interleaved lanes, then their sum (vec_sum).
 * cfg.ref_arith = 3 also calls the C library's elementary functions where the reference does,
 * instead of the deterministic dmath.h restatements the engine shares: exp in the rollout
 * probabilities (policy_improvement.cpp:356, std::exp), sin / cos in KDL Rotation::Rot2
 * (treefksolverjointposaxis_partial.cpp:125 -> KDL frames.inl), atan2 / asin / sin / cos in
 * btMatrix3x3::getEulerYPR (constraint_evaluator.cpp:98).  The normals stay the shared Philox +
 * Box-Muller draws (the reference's boost stream cannot be reproduced), so the modes differ in
 * the arithmetic alone.
 * tests/test_reference_order.py measures how far the engine contract drifts from them on the
 * north-star quantity (best_group_trajectory_) and on the discrete decisions.
 */
#include "stomp_oracle.h"
#include "dmath.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* stomp_utils.h:49-56 */
static const double DIFF_RULES[SO_NUM_DIFF_RULES][SO_DIFF_RULE_LENGTH] = {
    {0, 0, -2 / 6.0, -3 / 6.0, 6 / 6.0, -1 / 6.0, 0},
    {0, -1 / 12.0, 16 / 12.0, -30 / 12.0, 16 / 12.0, -1 / 12.0, 0},
    {0, 1 / 12.0, -17 / 12.0, 46 / 12.0, -46 / 12.0, 17 / 12.0, -1 / 12.0}};

static char g_err[512];
static void set_err(const char* m) { snprintf(g_err, sizeof g_err, "%s", m); }
const char* so_last_error(void) { return g_err; }

struct so_problem {
    so_config cfg;
    int J, N, Nall, K, Kr, S, nseg, B;
    so_segment* segs;
    so_sphere* sph;
    double* inv_clear;     /* S */
    so_joint* joints;
    double disc;           /* trajectory discretization */
    double dt;             /* policy movement_dt_ */
    double* Dpol[SO_NUM_DIFF_RULES];   /* Nall x Nall (policy, scaled) */
    double* Rall;          /* Nall x Nall */
    double* Rinv;          /* N x N */
    double* L;             /* N x N lower */
    double* M;             /* N x N */
    double* Qinv;          /* J x N x N (scaled StompCost inverse) */
    double* theta;         /* J x N */
    double* pad_pos;       /* 12 x S x 3 */
    int pad_collision;
    /* rollouts_ (policy_improvement.h:50-63), [K][J][N] */
    double *r_params, *r_noise, *r_nproj, *r_ctrl, *r_prob, *r_state /* K x N */;
    double *x_params, *x_noise, *x_nproj, *x_ctrl, *x_state;   /* the one extra rollout */
    double *tmp_params, *tmp_noise, *tmp_nproj, *tmp_ctrl, *tmp_prob, *tmp_state; /* reused_rollouts_ */
    int reused_next, extra_added, K_gen;
    /* the reuse decisions of every ranking so far: Kr candidate indices each (-1 = the extra
     * rollout), in the order generateRollouts kept them (policy_improvement.cpp:198-224) */
    int *rank_log, rank_n, rank_cap;
    /* optimizer state */
    double* last_traj;     /* J x N (free block of group_trajectory_ after the last execute) */
    double last_cost;
    int last_cf;
    double* best_traj;     /* J x N */
    /* torque term: chain segments root side first, their rigid-body inertias */
    int torque, nchain;
    int* chain;
    double* rb_m;          /* nchain */
    double* rb_h;          /* nchain x 3: m c */
    double* rb_I;          /* nchain x 9: rotational inertia about the segment origin */
    /* path constraints */
    int noc;
    struct oc_eval* oc;
    int last_cs;           /* last_trajectory_constraints_satisfied_ */
};

/* ---------------------------------------------------------------- linear algebra */

/* Cholesky A = C C^T, C lower (row-major n x n). Returns 0 on failure. */
static int chol_lower(const double* A, int n, double* C)
{
    memset(C, 0, sizeof(double) * (size_t)n * n);
    for (int j = 0; j < n; ++j) {
        double s = A[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) s -= C[(size_t)j * n + k] * C[(size_t)j * n + k];
        if (!(s > 0.0)) return 0;
        double cjj = sqrt(s);
        C[(size_t)j * n + j] = cjj;
        for (int i = j + 1; i < n; ++i) {
            double t = A[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) t -= C[(size_t)i * n + k] * C[(size_t)j * n + k];
            C[(size_t)i * n + j] = t / cjj;
        }
    }
    return 1;
}

/* Inverse of an SPD matrix through its Cholesky factor, column by column. */
static int spd_inverse(const double* A, int n, double* X)
{
    double* C = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* y = (double*)malloc(sizeof(double) * (size_t)n);
    int ok = chol_lower(A, n, C);
    if (ok) {
        for (int c = 0; c < n; ++c) {
            for (int i = 0; i < n; ++i) {
                double s = (i == c) ? 1.0 : 0.0;
                for (int k = 0; k < i; ++k) s -= C[(size_t)i * n + k] * y[k];
                y[i] = s / C[(size_t)i * n + i];
            }
            for (int i = n - 1; i >= 0; --i) {
                double s = y[i];
                for (int k = i + 1; k < n; ++k) s -= C[(size_t)k * n + i] * X[(size_t)k * n + c];
                X[(size_t)i * n + c] = s / C[(size_t)i * n + i];
            }
        }
    }
    free(C);
    free(y);
    return ok;
}

/* (D^T D)(a,b) = sum_k D(k,a) D(k,b), k ascending */
static void gram(const double* D, int n, double* G)
{
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) {
            double s = 0.0;
            for (int k = 0; k < n; ++k) s += D[(size_t)k * n + a] * D[(size_t)k * n + b];
            G[(size_t)a * n + b] = s;
        }
}

/* ---------------------------------------------------------------- RNG
 * Build-defined replacement for boost::mt19937 + normal_distribution seeded with
 * rand() (multivariate_gaussian.h:83-94): Philox4x32-10 keyed by the problem
 * seed, counter (pair index, rollout, joint, iteration), Box-Muller. */
#define SO_MAX_J 32
#define SO_MAX_CHAIN 64
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void so_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += PHILOX_W0;
        k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#define SO_TWO_PI 6.283185307179586476925286766559
#define SO_2POW_M53 1.1102230246251565404236316680908203125e-16

void so_normals(uint64_t seed, int iteration, int joint, int rollout, int n, double* z)
{
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int p = 0; 2 * p < n; ++p) {
        uint32_t ctr[4] = {(uint32_t)p, (uint32_t)rollout, (uint32_t)joint, (uint32_t)iteration};
        uint32_t o[4];
        so_philox4x32(ctr, key, o);
        uint64_t a = ((((uint64_t)o[0]) << 32) | o[1]) >> 11;
        uint64_t b = ((((uint64_t)o[2]) << 32) | o[3]) >> 11;
        double u1 = (double)(a + 1) * SO_2POW_M53;   /* (0, 1] */
        double u2 = (double)b * SO_2POW_M53;         /* [0, 1) */
        double r = sqrt(-2.0 * dm_log(u1));
        double s, c;
        dm_sincos(SO_TWO_PI * u2, &s, &c);
        z[2 * p] = r * c;
        if (2 * p + 1 < n) z[2 * p + 1] = r * s;
    }
}

void so_diff_rules(double* out) { memcpy(out, DIFF_RULES, sizeof DIFF_RULES); }
double so_exp(double x) { return dm_exp(x); }
double so_log(double x) { return dm_log(x); }
void so_sincos(double x, double* s, double* c) { dm_sincos(x, s, c); }
double so_atan2(double y, double x) { return dm_atan2(y, x); }
double so_asin(double x) { return dm_asin(x); }

/* ---------------------------------------------------------------- KDL frames
 * KDL::Rotation::Rot2 / Rotation*Rotation / Rotation*Vector / Frame*Frame as in
 * orocos KDL (3rd party, reached from treefksolverjointposaxis_partial.cpp:125). */
typedef struct { double R[9]; double p[3]; } frame_t;

/* libm: the C library's sin / cos (ref_arith 3, as KDL calls them) instead of dm_sincos */
static void rot2(const double* a, double angle, double* R, int libm)
{
    double st, ct;
    if (libm) {
        st = sin(angle);
        ct = cos(angle);
    } else {
        dm_sincos(angle, &st, &ct);
    }
    double vt = 1.0 - ct;
    double m_vt_0 = vt * a[0], m_vt_1 = vt * a[1], m_vt_2 = vt * a[2];
    double m_st_0 = a[0] * st, m_st_1 = a[1] * st, m_st_2 = a[2] * st;
    double m_vt_0_1 = m_vt_0 * a[1], m_vt_0_2 = m_vt_0 * a[2], m_vt_1_2 = m_vt_1 * a[2];
    R[0] = ct + m_vt_0 * a[0];
    R[1] = -m_st_2 + m_vt_0_1;
    R[2] = m_st_1 + m_vt_0_2;
    R[3] = m_st_2 + m_vt_0_1;
    R[4] = ct + m_vt_1 * a[1];
    R[5] = -m_st_0 + m_vt_1_2;
    R[6] = -m_st_1 + m_vt_0_2;
    R[7] = m_st_0 + m_vt_1_2;
    R[8] = ct + m_vt_2 * a[2];
}

static void rotmul(const double* A, const double* B, double* C)
{
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

static void frame_apply(const frame_t* f, const double* v, double* out)
{
    for (int i = 0; i < 3; ++i)
        out[i] = f->R[3 * i + 0] * v[0] + f->R[3 * i + 1] * v[1] + f->R[3 * i + 2] * v[2] + f->p[i];
}

/* The segment's fixed rotation is exactly the identity (every PR2 segment): KDL's products
 * with it (rot * Rot2, parent.M * rot) return their other factor up to the sign of zero
 * entries, and both the oracle and the engine skip them. */
static int so_rot_identity(const double* r)
{
    return r[0] == 1.0 && r[1] == 0.0 && r[2] == 0.0 && r[3] == 0.0 && r[4] == 1.0 && r[5] == 0.0 &&
           r[6] == 0.0 && r[7] == 0.0 && r[8] == 1.0;
}

/* segment pose(q) composed onto the parent frame */
static void segment_frame(const so_segment* s, const frame_t* parent, double q, frame_t* out, int libm)
{
    frame_t pose;
    const int ident = so_rot_identity(s->rot);
    if (s->q_index >= 0) {
        double Rq[9];
        rot2(s->axis, q, Rq, libm);
        if (ident) memcpy(pose.R, Rq, sizeof pose.R);
        else rotmul(s->rot, Rq, pose.R);
    } else {
        memcpy(pose.R, s->rot, sizeof pose.R);
    }
    memcpy(pose.p, s->trans, sizeof pose.p);
    if (!parent) {
        *out = pose;
        return;
    }
    if (s->q_index < 0 && ident) memcpy(out->R, parent->R, sizeof out->R);
    else rotmul(parent->R, pose.R, out->R);
    for (int i = 0; i < 3; ++i)
        out->p[i] = parent->R[3 * i + 0] * pose.p[0] + parent->R[3 * i + 1] * pose.p[1] +
                    parent->R[3 * i + 2] * pose.p[2] + parent->p[i];
}

/* JntToCartFull == JntToCartPartial here: the reference frame is the root with an
 * identity pose, so inv_ref_frame * frame is exact. */
static void fk_spheres(const so_problem* P, const double* q, frame_t* frames, double* pos /* S x 3 */)
{
    for (int s = 0; s < P->nseg; ++s) {
        const so_segment* sg = &P->segs[s];
        double qv = sg->q_index >= 0 ? q[sg->q_index] : 0.0;
        segment_frame(sg, sg->parent >= 0 ? &frames[sg->parent] : NULL, qv, &frames[s], P->cfg.ref_arith >= 3);
    }
    for (int j = 0; j < P->S; ++j)   /* stomp_collision_point.h:138-141 */
        frame_apply(&frames[P->sph[j].segment], P->sph[j].pos, pos + 3 * j);
}

/* ---------------------------------------------------------------- inverse dynamics
 * KDL::ChainIdSolver_RNE::CartToJnt (orocos KDL, 3rd party, not vendored; constructed at
 * stomp_robot_model.cpp:185-189, called from StompOptimizer::getTorques
 * stomp_optimizer.cpp:1049-1053).  Restated from KDL's published recursion: outward sweep
 * v_i = X_i^-1 v_{i-1} + S_i qd_i, a_i = X_i^-1 a_{i-1} + S_i qdd_i + v_i x (S_i qd_i) (root:
 * a_0 = X_0^-1 (-gravity, 0)), f_i = I_i a_i + v_i x* (I_i v_i); inward sweep tau_i = S_i . f_i,
 * f_{i-1} += X_i f_i.  Twists / wrenches are (linear, angular) in segment coordinates with the
 * KDL Frame/Twist/Wrench/RigidBodyInertia operators below.  In this build's segment
 * convention the segment frame sits on its joint axis, so the unit twist is S = (0, axis).
 * PARITY UNPINNED against KDL (no KDL in the container). */
typedef struct { double vel[3]; double rot[3]; } twist_t;
typedef struct { double force[3]; double torque[3]; } wrench_t;

static void v_cross(const double* a, const double* b, double* c)   /* KDL Vector * Vector */
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

static void rot_mul_v(const double* R, const double* v, double* o)   /* Rotation * Vector */
{
    for (int i = 0; i < 3; ++i) o[i] = R[3 * i + 0] * v[0] + R[3 * i + 1] * v[1] + R[3 * i + 2] * v[2];
}

static void rot_inv_mul_v(const double* R, const double* v, double* o)   /* Rotation::Inverse(Vector) */
{
    for (int i = 0; i < 3; ++i) o[i] = R[0 + i] * v[0] + R[3 + i] * v[1] + R[6 + i] * v[2];
}

/* Frame::Inverse(Twist): (R^T (v - p x w), R^T w) */
static void frame_inv_twist(const double* R, const double* p, const twist_t* t, twist_t* o)
{
    double pw[3], d[3];
    v_cross(p, t->rot, pw);
    for (int k = 0; k < 3; ++k) d[k] = t->vel[k] - pw[k];
    rot_inv_mul_v(R, d, o->vel);
    rot_inv_mul_v(R, t->rot, o->rot);
}

/* Twist * Twist (motion cross product): (a.w x b.v + a.v x b.w, a.w x b.w) */
static void twist_cross(const twist_t* a, const twist_t* b, twist_t* o)
{
    double x[3], y[3];
    v_cross(a->rot, b->vel, x);
    v_cross(a->vel, b->rot, y);
    for (int k = 0; k < 3; ++k) o->vel[k] = x[k] + y[k];
    v_cross(a->rot, b->rot, o->rot);
}

/* RigidBodyInertia * Twist: (m v - h x w, I w + h x v) */
static void rbi_mul(double m, const double* h, const double* I, const twist_t* t, wrench_t* o)
{
    double hw[3], hv[3], Iw[3];
    v_cross(h, t->rot, hw);
    v_cross(h, t->vel, hv);
    rot_mul_v(I, t->rot, Iw);
    for (int k = 0; k < 3; ++k) {
        o->force[k] = m * t->vel[k] - hw[k];
        o->torque[k] = Iw[k] + hv[k];
    }
}

/* Twist * Wrench (force cross product): (w x f, w x n + v x f) */
static void twist_cross_wrench(const twist_t* t, const wrench_t* w, wrench_t* o)
{
    double a[3], b[3];
    v_cross(t->rot, w->force, o->force);
    v_cross(t->rot, w->torque, a);
    v_cross(t->vel, w->force, b);
    for (int k = 0; k < 3; ++k) o->torque[k] = a[k] + b[k];
}

/* Frame * Wrench: (R f, R n + p x (R f)) */
static void frame_wrench(const double* R, const double* p, const wrench_t* w, wrench_t* o)
{
    double rn[3], pf[3];
    rot_mul_v(R, w->force, o->force);
    rot_mul_v(R, w->torque, rn);
    v_cross(p, o->force, pf);
    for (int k = 0; k < 3; ++k) o->torque[k] = rn[k] + pf[k];
}

/* KDL::RigidBodyInertia(m, c, Ic): h = m c, I = Ic - m (c c^T - (c.c) 1) */
static void rb_inertia(const so_inertia* in, double* m, double* h, double* I)
{
    const double* c = in->com;
    const double* v = in->inertia;
    const double Ic[9] = {v[0], v[3], v[4], v[3], v[1], v[5], v[4], v[5], v[2]};
    const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    *m = in->mass;
    for (int i = 0; i < 3; ++i) {
        h[i] = in->mass * c[i];
        for (int j = 0; j < 3; ++j) I[3 * i + j] = Ic[3 * i + j] - in->mass * (c[i] * c[j] - (i == j ? cc : 0.0));
    }
}

int so_inverse_dynamics(const so_problem* P, const double* q, const double* qd, const double* qdd, double* tau)
{
    if (!P->chain) return -1;
    wrench_t f[64];
    double Rs[64][9];
    const double* g = P->cfg.gravity;
    const twist_t ag = {{-g[0], -g[1], -g[2]}, {0.0, 0.0, 0.0}};
    twist_t v = {{0}}, a = {{0}};
    for (int i = 0; i < P->nchain; ++i) {
        const so_segment* sg = &P->segs[P->chain[i]];
        const int j = sg->q_index;
        double qv = 0.0, qdv = 0.0, qddv = 0.0;
        twist_t S = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
        if (j >= 0) {
            qv = q[j]; qdv = qd[j]; qddv = qdd[j];
            for (int k = 0; k < 3; ++k) S.rot[k] = sg->axis[k];
        }
        double* R = Rs[i];
        if (j >= 0) {
            double Rq[9];
            rot2(sg->axis, qv, Rq, P->cfg.ref_arith >= 3);
            if (so_rot_identity(sg->rot)) memcpy(R, Rq, sizeof(double) * 9);
            else rotmul(sg->rot, Rq, R);
        } else {
            memcpy(R, sg->rot, sizeof(double) * 9);
        }
        const double* p = sg->trans;
        twist_t vj, xv, xa, c;
        for (int k = 0; k < 3; ++k) { vj.vel[k] = S.vel[k] * qdv; vj.rot[k] = S.rot[k] * qdv; }
        if (i == 0) {
            v = vj;
            frame_inv_twist(R, p, &ag, &xa);
        } else {
            frame_inv_twist(R, p, &v, &xv);
            frame_inv_twist(R, p, &a, &xa);
            for (int k = 0; k < 3; ++k) { v.vel[k] = xv.vel[k] + vj.vel[k]; v.rot[k] = xv.rot[k] + vj.rot[k]; }
        }
        twist_cross(&v, &vj, &c);
        for (int k = 0; k < 3; ++k) {
            a.vel[k] = xa.vel[k] + S.vel[k] * qddv + c.vel[k];
            a.rot[k] = xa.rot[k] + S.rot[k] * qddv + c.rot[k];
        }
        wrench_t Ia, Iv, vIv;
        const double m = P->rb_m[i];
        const double* h = P->rb_h + 3 * i;
        const double* I = P->rb_I + 9 * i;
        rbi_mul(m, h, I, &a, &Ia);
        rbi_mul(m, h, I, &v, &Iv);
        twist_cross_wrench(&v, &Iv, &vIv);
        for (int k = 0; k < 3; ++k) { f[i].force[k] = Ia.force[k] + vIv.force[k]; f[i].torque[k] = Ia.torque[k] + vIv.torque[k]; }
    }
    for (int i = P->nchain - 1; i >= 0; --i) {
        const so_segment* sg = &P->segs[P->chain[i]];
        if (sg->q_index >= 0) {
            /* dot(Twist, Wrench) = v . f + w . n with S = (0, axis) */
            const double* n = f[i].torque;
            const double* ff = f[i].force;
            tau[sg->q_index] = (0.0 * ff[0] + 0.0 * ff[1] + 0.0 * ff[2]) + (sg->axis[0] * n[0] + sg->axis[1] * n[1] + sg->axis[2] * n[2]);
        }
        if (i != 0) {
            wrench_t t;
            frame_wrench(Rs[i], P->segs[P->chain[i]].trans, &f[i], &t);
            for (int k = 0; k < 3; ++k) { f[i - 1].force[k] += t.force[k]; f[i - 1].torque[k] += t.torque[k]; }
        }
    }
    return 0;
}

/* StompOptimizer::getTorques (stomp_optimizer.cpp:1033-1061) + the torque sum of execute
 * (:1117-1142): q from the group trajectory row i, q-dot / q-ddot by the 7-tap rules of
 * StompTrajectory::getJointVelocities / getJointAccelerations (stomp_trajectory.h:286-310) */
static double torque_cost_at(const so_problem* P, const double* traj /* Nall x J */, int i)
{
    const int J = P->J;
    double q[SO_MAX_J], qd[SO_MAX_J], qdd[SO_MAX_J], tau[SO_MAX_J];
    const double invTime = 1.0 / P->disc, invTime2 = 1.0 / (P->disc * P->disc);
    for (int j = 0; j < J; ++j) { q[j] = traj[(size_t)i * J + j]; qd[j] = 0.0; qdd[j] = 0.0; }
    for (int k = -SO_DIFF_RULE_LENGTH / 2; k <= SO_DIFF_RULE_LENGTH / 2; ++k) {
        const double cv = invTime * DIFF_RULES[0][k + SO_DIFF_RULE_LENGTH / 2];
        const double ca = invTime2 * DIFF_RULES[1][k + SO_DIFF_RULE_LENGTH / 2];
        for (int j = 0; j < J; ++j) {
            qd[j] += cv * traj[(size_t)(i + k) * J + j];
            qdd[j] += ca * traj[(size_t)(i + k) * J + j];
        }
    }
    so_inverse_dynamics(P, q, qd, qdd, tau);
    double s = 0.0;
    for (int j = 0; j < J; ++j) s += fabs(tau[j]);
    return s;
}

/* ---------------------------------------------------------------- orientation constraints
 * OrientationConstraintEvaluator (constraint_evaluator.cpp:50-114) and the third-party
 * arithmetic it reaches, restated from the published sources (not vendored; PARITY UNPINNED):
 *   KDL Rotation::GetQuaternion (orocos KDL 1.0, frames.cpp; its non-trace branches evaluate
 *     s in single precision, `float s = 2.0 * sqrtf(...)`),
 *   tf::quaternionMsgToTF (normalises when |q|^2 is off by more than 0.1) and
 *   btMatrix3x3::setRotation / inverse / operator* / getRPY -> getEulerYPR(solution 1)
 *     (bullet LinearMath with BT_USE_DOUBLE_PRECISION, as built by ROS). */
struct oc_eval {
    int seg, body_fixed;
    int libm;              /* ref_arith 3: the C library's atan2 / asin / sin / cos */
    double ninv[9];        /* nominal_orientation_inverse_ */
    double rw, pw, yw;     /* roll/pitch/yaw weights (0 when the tolerance is >= pi) */
    double tol[3];         /* absolute roll / pitch / yaw tolerance */
    double weight;
};

static void bt_from_quat(double x, double y, double z, double w, double* M)   /* btMatrix3x3::setRotation */
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

static double bt_cofac(const double* M, int r1, int c1, int r2, int c2)
{
    return M[3 * r1 + c1] * M[3 * r2 + c2] - M[3 * r1 + c2] * M[3 * r2 + c1];
}

static void bt_inverse(const double* M, double* O)   /* btMatrix3x3::inverse */
{
    const double co0 = bt_cofac(M, 1, 1, 2, 2), co1 = bt_cofac(M, 1, 2, 2, 0), co2 = bt_cofac(M, 1, 0, 2, 1);
    const double det = M[0] * co0 + M[1] * co1 + M[2] * co2;
    const double s = 1.0 / det;
    O[0] = co0 * s; O[1] = bt_cofac(M, 0, 2, 2, 1) * s; O[2] = bt_cofac(M, 0, 1, 1, 2) * s;
    O[3] = co1 * s; O[4] = bt_cofac(M, 0, 0, 2, 2) * s; O[5] = bt_cofac(M, 0, 2, 1, 0) * s;
    O[6] = co2 * s; O[7] = bt_cofac(M, 0, 1, 2, 0) * s; O[8] = bt_cofac(M, 0, 0, 1, 1) * s;
}

/* KDL Rotation::GetQuaternion (row-major R) */
static void kdl_get_quaternion(const double* R, double* x, double* y, double* z, double* w)
{
    const double trace = R[0] + R[4] + R[8];
    if (trace > 1e-12) {
        const double s = 0.5 / sqrt(trace + 1.0);
        *w = 0.25 / s;
        *x = (R[7] - R[5]) * s;
        *y = (R[2] - R[6]) * s;
        *z = (R[3] - R[1]) * s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        const float s = (float)(2.0 * sqrtf((float)(1.0 + R[0] - R[4] - R[8])));
        *w = (R[7] - R[5]) / s;
        *x = 0.25 * s;
        *y = (R[1] + R[3]) / s;
        *z = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        const float s = (float)(2.0 * sqrtf((float)(1.0 + R[4] - R[0] - R[8])));
        *w = (R[2] - R[6]) / s;
        *x = (R[1] + R[3]) / s;
        *y = 0.25 * s;
        *z = (R[5] + R[7]) / s;
    } else {
        const float s = (float)(2.0 * sqrtf((float)(1.0 + R[8] - R[0] - R[4])));
        *w = (R[3] - R[1]) / s;
        *x = (R[2] + R[6]) / s;
        *y = (R[5] + R[7]) / s;
        *z = 0.25 * s;
    }
}

/* btMatrix3x3::getRPY -> getEulerYPR(yaw, pitch, roll, 1) */
static void bt_get_rpy(const double* M, double* roll, double* pitch, double* yaw, int libm)
{
    const double pi = 3.1415926535897932384626433832795029;
    if (fabs(M[6]) >= 1.0) {
        *yaw = 0.0;
        const double delta = libm ? atan2(M[0], M[2]) : dm_atan2(M[0], M[2]);
        if (M[6] > 0.0) {
            *pitch = pi / 2.0;
            *roll = *pitch + delta;
        } else {
            *pitch = -pi / 2.0;
            *roll = -*pitch + delta;
        }
    } else {
        double a = M[6];   /* btAsin clamps to [-1, 1] */
        if (a < -1.0) a = -1.0;
        if (a > 1.0) a = 1.0;
        *pitch = -(libm ? asin(a) : dm_asin(a));
        double sp, cp;
        if (libm) {
            sp = sin(*pitch);
            cp = cos(*pitch);
        } else {
            dm_sincos(*pitch, &sp, &cp);
        }
        (void)sp;
        *roll = libm ? atan2(M[7] / cp, M[8] / cp) : dm_atan2(M[7] / cp, M[8] / cp);
        *yaw = libm ? atan2(M[3] / cp, M[0] / cp) : dm_atan2(M[3] / cp, M[0] / cp);
    }
}

static void bt_mul(const double* A, const double* B, double* C)   /* btMatrix3x3 operator* */
{
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

/* OrientationConstraintEvaluator ctor (constraint_evaluator.cpp:50-73) */
static void oc_init(const so_orientation_constraint* c, struct oc_eval* o)
{
    double x = c->orientation[0], y = c->orientation[1], z = c->orientation[2], w = c->orientation[3];
    const double l2 = x * x + y * y + z * z + w * w;
    if (fabs(l2 - 1.0) > 0.1f) {   /* tf::quaternionMsgToTF: QUATERNION_TOLERANCE 0.1f */
        const double inv = 1.0 / sqrt(l2);
        x *= inv; y *= inv; z *= inv; w *= inv;
    }
    double nom[9];
    bt_from_quat(x, y, z, w, nom);
    bt_inverse(nom, o->ninv);
    o->seg = c->segment;
    o->body_fixed = c->body_fixed;
    o->tol[0] = c->absolute_roll_tolerance;
    o->tol[1] = c->absolute_pitch_tolerance;
    o->tol[2] = c->absolute_yaw_tolerance;
    o->weight = c->weight;
    o->rw = o->pw = o->yw = 1.0;
    if (o->tol[1] >= M_PI) o->pw = 0.0;
    if (o->tol[0] >= M_PI) o->rw = 0.0;
    if (o->tol[2] >= M_PI) o->yw = 0.0;
}

/* OrientationConstraintEvaluator::getCost (constraint_evaluator.cpp:80-114); returns satisfied */
static int oc_cost(const struct oc_eval* o, const double* R, double* cost)
{
    double x, y, z, w, M[9], res[9], roll, pitch, yaw;
    kdl_get_quaternion(R, &x, &y, &z, &w);
    bt_from_quat(x, y, z, w, M);
    if (!o->body_fixed) bt_mul(M, o->ninv, res);
    else bt_mul(o->ninv, M, res);
    bt_get_rpy(res, &roll, &pitch, &yaw, o->libm);
    roll = fabs(roll);
    pitch = fabs(pitch);
    yaw = fabs(yaw);
    *cost = o->weight * (o->rw * roll + o->pw * pitch + o->yw * yaw);
    return !(roll > o->tol[0] || pitch > o->tol[1] || yaw > o->tol[2]);
}

/* ---------------------------------------------------------------- distance field
 * distance_field::PropagationDistanceField::getDistanceGradient (3rd party; call site
 * stomp_collision_space.h:187-191): nearest cell = round((p - origin) * (1/res)) (VoxelGrid
 * keeps the reciprocal resolution); cells with an index < 1 or >= n-1 (or a non-finite
 * position) read distance 0. */
double so_sdf_distance(const so_problem* P, double x, double y, double z)
{
    const so_sdf* g = &P->cfg.sdf;
    const double inv = 1.0 / g->resolution;
    double fx = round((x - g->origin[0]) * inv);
    double fy = round((y - g->origin[1]) * inv);
    double fz = round((z - g->origin[2]) * inv);
    if (!(fx >= 1.0 && fy >= 1.0 && fz >= 1.0 && fx < (double)(g->nx - 1) && fy < (double)(g->ny - 1) &&
          fz < (double)(g->nz - 1)))
        return 0.0;
    long ix = (long)fx, iy = (long)fy, iz = (long)fz;
    /* PropagationDistanceField::getDistance: sqrt_table_[distance_square_], the table made as
     * sqrt(double(i)) * resolution */
    const unsigned d2 = g->data[((size_t)ix * g->ny + (size_t)iy) * g->nz + (size_t)iz];
    return sqrt((double)d2) * g->resolution;
}

/* stomp_collision_space.h:193-228 (gradient is CHOMP-only and not computed) */
static int potential_of(const so_problem* P, int j, const double* pos, double* pot)
{
    double dist = so_sdf_distance(P, pos[0], pos[1], pos[2]);
    double r = P->sph[j].radius, c = P->sph[j].clearance;
    double d = dist - r;
    if (d >= c) {
        *pot = 0.0;
    } else if (d >= 0.0) {
        double diff = d - c;
        double gm = diff * P->inv_clear[j];
        *pot = 0.5 * gm * diff;
    } else {
        *pot = -d + 0.5 * c;
    }
    return dist <= r;
}

int so_potential(const so_problem* P, int sphere, const double* pos, double* potential)
{
    return potential_of(P, sphere, pos, potential);
}

int so_sphere_positions(const so_problem* P, const double* q, double* out)
{
    frame_t* fr = (frame_t*)malloc(sizeof(frame_t) * (size_t)P->nseg);
    fk_spheres(P, q, fr, out);
    free(fr);
    return 0;
}

/* ---------------------------------------------------------------- setup */

static double* dalloc(size_t n) { return (double*)calloc(n ? n : 1, sizeof(double)); }

void so_destroy(so_problem* P)
{
    if (!P) return;
    free(P->segs); free(P->sph); free(P->inv_clear); free(P->joints);
    for (int i = 0; i < SO_NUM_DIFF_RULES; ++i) free(P->Dpol[i]);
    free(P->Rall); free(P->Rinv); free(P->L); free(P->M); free(P->Qinv); free(P->theta); free(P->pad_pos);
    free(P->r_params); free(P->r_noise); free(P->r_nproj); free(P->r_ctrl); free(P->r_prob); free(P->r_state);
    free(P->x_params); free(P->x_noise); free(P->x_nproj); free(P->x_ctrl); free(P->x_state);
    free(P->tmp_params); free(P->tmp_noise); free(P->tmp_nproj); free(P->tmp_ctrl); free(P->tmp_prob);
    free(P->tmp_state);
    free(P->last_traj); free(P->best_traj);
    free(P->chain); free(P->rb_m); free(P->rb_h); free(P->rb_I); free(P->oc);
    free(P->rank_log);
    free((void*)P->cfg.noise_stddev); free((void*)P->cfg.noise_decay);
    free((void*)P->cfg.start); free((void*)P->cfg.goal);
    free(P);
}

static double* dup_d(const double* a, int n)
{
    double* b = dalloc((size_t)n);
    memcpy(b, a, sizeof(double) * (size_t)n);
    return b;
}

so_problem* so_create(const so_config* cfg)
{
    if (cfg->num_joints <= 0 || cfg->num_time_steps <= 0 || cfg->num_rollouts <= 0 || cfg->num_spheres < 0 ||
        cfg->num_segments <= 0) {
        set_err("invalid sizes");
        return NULL;
    }
    if (cfg->num_reused_rollouts >= cfg->num_rollouts) {   /* policy_improvement.cpp:102-106 */
        set_err("Number of reused rollouts must be strictly less than number of rollouts.");
        return NULL;
    }
    if (cfg->num_joints > SO_MAX_J) {
        set_err("at most 32 joints");
        return NULL;
    }
    if (cfg->num_orientation_constraints < 0 || (cfg->num_orientation_constraints > 0 && !cfg->orientation_constraints)) {
        set_err("invalid orientation constraints");
        return NULL;
    }
    so_problem* P = (so_problem*)calloc(1, sizeof(so_problem));
    P->cfg = *cfg;
    int J = P->J = cfg->num_joints;
    int N = P->N = cfg->num_time_steps;
    int Nall = P->Nall = N + 2 * SO_PAD;
    P->K = cfg->num_rollouts;
    P->Kr = cfg->num_reused_rollouts;
    P->S = cfg->num_spheres;
    P->nseg = cfg->num_segments;
    P->B = cfg->sum_block > 0 ? cfg->sum_block : 64;
    if (cfg->ref_arith) P->B = cfg->num_rollouts;   /* one block: the reference's sequential sums */
    P->cfg.noise_stddev = dup_d(cfg->noise_stddev, J);
    P->cfg.noise_decay = dup_d(cfg->noise_decay, J);
    P->cfg.start = dup_d(cfg->start, J);
    P->cfg.goal = dup_d(cfg->goal, J);
    P->segs = (so_segment*)malloc(sizeof(so_segment) * (size_t)P->nseg);
    memcpy(P->segs, cfg->segments, sizeof(so_segment) * (size_t)P->nseg);
    P->sph = (so_sphere*)malloc(sizeof(so_sphere) * (size_t)(P->S ? P->S : 1));
    if (P->S) memcpy(P->sph, cfg->spheres, sizeof(so_sphere) * (size_t)P->S);
    P->inv_clear = dalloc((size_t)P->S);
    for (int j = 0; j < P->S; ++j) P->inv_clear[j] = 1.0 / P->sph[j].clearance;  /* stomp_collision_point.cpp:50 */
    P->joints = (so_joint*)malloc(sizeof(so_joint) * (size_t)J);
    memcpy(P->joints, cfg->joints, sizeof(so_joint) * (size_t)J);
    for (int s = 0; s < P->nseg; ++s) {
        if (P->segs[s].parent >= s || P->segs[s].q_index >= J) {
            set_err("segments must be in DFS order with valid joint indices");
            so_destroy(P);
            return NULL;
        }
    }
    for (int j = 0; j < P->S; ++j)
        if (P->sph[j].segment < 0 || P->sph[j].segment >= P->nseg) {
            set_err("sphere segment out of range");
            so_destroy(P);
            return NULL;
        }

    /* the inverse-dynamics chain (stomp_robot_model.cpp:185-189): segments below torque_root
     * up to torque_tip; its joints must be the group's, in order */
    P->torque = cfg->torque_cost_weight > 1e-9;
    /* built whenever the inertias describe a valid chain: the term runs only with the weight
     * on, the final torque statistics of optimize() always (stomp_optimizer.cpp:384-398) */
    {
        const char* why = NULL;
        int path[SO_MAX_CHAIN], n = 0;
        if (!cfg->inertias) why = "torque term needs segment inertias";
        else if (cfg->torque_root < 0 || cfg->torque_root >= P->nseg || cfg->torque_tip < 0 || cfg->torque_tip >= P->nseg)
            why = "torque chain root/tip out of range";
        else {
            for (int sgi = cfg->torque_tip; sgi != cfg->torque_root; sgi = P->segs[sgi].parent) {
                if (sgi < 0 || n == SO_MAX_CHAIN) { why = "torque tip is not below the torque root (or chain too long)"; break; }
                path[n++] = sgi;
            }
        }
        if (!why) {
            int nj = 0;
            for (int i = n - 1; i >= 0; --i)
                if (P->segs[path[i]].q_index >= 0 && P->segs[path[i]].q_index != nj++) why = "torque chain joints must be the group joints in order";
            if (!why && nj != J) why = "torque chain joints must be the group joints in order";
        }
        if (why && P->torque) {
            set_err(why);
            so_destroy(P);
            return NULL;
        }
        if (!why) {
            P->nchain = n;
            P->chain = (int*)malloc(sizeof(int) * (size_t)n);
            P->rb_m = dalloc((size_t)n);
            P->rb_h = dalloc((size_t)n * 3);
            P->rb_I = dalloc((size_t)n * 9);
            for (int i = 0; i < n; ++i) {
                P->chain[i] = path[n - 1 - i];
                rb_inertia(&cfg->inertias[P->chain[i]], &P->rb_m[i], P->rb_h + 3 * i, P->rb_I + 9 * i);
            }
        }
    }

    /* constraint_evaluators_ (stomp_optimizer.cpp:195-201) */
    P->noc = cfg->num_orientation_constraints;
    P->oc = (struct oc_eval*)calloc((size_t)(P->noc ? P->noc : 1), sizeof(struct oc_eval));
    for (int c = 0; c < P->noc; ++c) {
        if (cfg->orientation_constraints[c].segment < 0 || cfg->orientation_constraints[c].segment >= P->nseg) {
            set_err("orientation constraint segment out of range");
            so_destroy(P);
            return NULL;
        }
        oc_init(&cfg->orientation_constraints[c], &P->oc[c]);
        P->oc[c].libm = cfg->ref_arith >= 3;
    }
    P->cfg.orientation_constraints = NULL;

    P->disc = cfg->discretization;
    /* group trajectory duration (N_all-1)*disc, truncated by getDuration() -> int
     * (stomp_trajectory.cpp:86, stomp_trajectory.h:255-258); movement_dt_ =
     * duration / (num_time_steps + 1) (covariant_trajectory_policy.cpp:152) */
    int duration = (int)((double)(Nall - 1) * P->disc);
    P->dt = (double)duration / (double)(N + 1);

    /* createDifferentiationMatrices (covariant_trajectory_policy.cpp:204-226) */
    double mult = 1.0;
    for (int d = 0; d < SO_NUM_DIFF_RULES; ++d) {
        mult /= P->dt;
        P->Dpol[d] = dalloc((size_t)Nall * Nall);
        for (int i = 0; i < Nall; ++i)
            for (int j = -SO_DIFF_RULE_LENGTH / 2; j <= SO_DIFF_RULE_LENGTH / 2; ++j) {
                int idx = i + j;
                if (idx < 0 || idx >= Nall) continue;
                P->Dpol[d][(size_t)i * Nall + idx] = mult * DIFF_RULES[d][j + SO_DIFF_RULE_LENGTH / 2];
            }
    }
    /* initializeCosts (covariant_trajectory_policy.cpp:168-191): identical for every
     * dimension, so it is built once */
    P->Rall = dalloc((size_t)Nall * Nall);
    double* G = dalloc((size_t)Nall * Nall);
    for (int i = 0; i < Nall; ++i) P->Rall[(size_t)i * Nall + i] = 1.0 * cfg->ridge_factor;
    for (int d = 0; d < SO_NUM_DIFF_RULES; ++d) {
        gram(P->Dpol[d], Nall, G);
        for (size_t k = 0; k < (size_t)Nall * Nall; ++k) P->Rall[k] += cfg->smoothness_costs[d] * G[k];
    }
    double* Rfree = dalloc((size_t)N * N);
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) Rfree[(size_t)i * N + j] = P->Rall[(size_t)(i + SO_PAD) * Nall + (j + SO_PAD)];
    P->Rinv = dalloc((size_t)N * N);
    P->L = dalloc((size_t)N * N);
    P->M = dalloc((size_t)N * N);
    if (!spd_inverse(Rfree, N, P->Rinv) || !chol_lower(P->Rinv, N, P->L)) {
        set_err("control cost matrix is not positive definite");
        free(G); free(Rfree);
        so_destroy(P);
        return NULL;
    }
    /* preComputeProjectionMatrices (policy_improvement.cpp:421-441) */
    for (int p = 0; p < N; ++p) {
        double cmax = P->Rinv[p];
        for (int p2 = 1; p2 < N; ++p2)
            if (P->Rinv[(size_t)p2 * N + p] > cmax) cmax = P->Rinv[(size_t)p2 * N + p];
        double sc = 1.0 / ((double)N * cmax);
        for (int i = 0; i < N; ++i) P->M[(size_t)i * N + p] = P->Rinv[(size_t)i * N + p] * sc;
    }

    /* StompCost (stomp_cost.cpp:47-74) + scaling (stomp_optimizer.cpp:100-125) */
    P->Qinv = dalloc((size_t)J * N * N);
    {
        double* Draw = dalloc((size_t)Nall * Nall);
        double* Qfull = dalloc((size_t)Nall * Nall);
        double* Qfree = dalloc((size_t)N * N);
        double max_scale = 0.0;
        for (int jt = 0; jt < J; ++jt) {
            memset(Qfull, 0, sizeof(double) * (size_t)Nall * Nall);
            double m2 = 1.0;
            for (int d = 0; d < SO_NUM_DIFF_RULES; ++d) {
                m2 *= P->disc;
                memset(Draw, 0, sizeof(double) * (size_t)Nall * Nall);
                for (int i = 0; i < Nall; ++i)
                    for (int j = -SO_DIFF_RULE_LENGTH / 2; j <= SO_DIFF_RULE_LENGTH / 2; ++j) {
                        int idx = i + j;
                        if (idx < 0 || idx >= Nall) continue;
                        Draw[(size_t)i * Nall + idx] = DIFF_RULES[d][j + SO_DIFF_RULE_LENGTH / 2];
                    }
                gram(Draw, Nall, G);
                double w = P->joints[jt].joint_cost * cfg->smoothness_costs[d];
                double f = w * m2;
                for (size_t k = 0; k < (size_t)Nall * Nall; ++k) Qfull[k] += f * G[k];
            }
            for (int i = 0; i < Nall; ++i) Qfull[(size_t)i * Nall + i] += 1.0 * cfg->ridge_factor;
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) Qfree[(size_t)i * N + j] = Qfull[(size_t)(i + SO_PAD) * Nall + (j + SO_PAD)];
            double* Qi = P->Qinv + (size_t)jt * N * N;
            if (!spd_inverse(Qfree, N, Qi)) {
                set_err("joint cost matrix is not positive definite");
                free(Draw); free(Qfull); free(Qfree); free(G); free(Rfree);
                so_destroy(P);
                return NULL;
            }
            double mx = Qi[0];
            for (size_t k = 1; k < (size_t)N * N; ++k) if (Qi[k] > mx) mx = Qi[k];
            if (max_scale < mx) max_scale = mx;
        }
        double inv_scale = 1.0 / max_scale;
        for (size_t k = 0; k < (size_t)J * N * N; ++k) P->Qinv[k] *= inv_scale;
        free(Draw); free(Qfull); free(Qfree);
    }
    free(G);
    free(Rfree);

    /* setToMinControlCost (covariant_trajectory_policy.cpp:102-148) */
    P->theta = dalloc((size_t)J * N);
    {
        double* lin = dalloc((size_t)N);
        for (int d = 0; d < J; ++d) {
            for (int c = 0; c < N; ++c) {
                double a = 0.0;
                for (int i = 0; i < SO_PAD; ++i) a += cfg->start[d] * P->Rall[(size_t)i * Nall + (c + SO_PAD)];
                double b = 0.0;
                for (int i = 0; i < SO_PAD; ++i)
                    b += cfg->goal[d] * P->Rall[(size_t)(N + SO_PAD + i) * Nall + (c + SO_PAD)];
                lin[c] = (a + b) * 2.0;
            }
            for (int i = 0; i < N; ++i) {
                double s = 0.0;
                for (int k = 0; k < N; ++k) s += (-0.5 * P->Rinv[(size_t)i * N + k]) * lin[k];
                P->theta[(size_t)d * N + i] = s;
            }
        }
        free(lin);
    }

    /* padding-point sphere positions: iteration-0 full FK of start/goal
     * (stomp_optimizer.cpp:626-630, stomp_trajectory.cpp:94-107) */
    P->pad_pos = dalloc((size_t)2 * SO_PAD * (P->S ? P->S : 1) * 3);
    {
        frame_t* fr = (frame_t*)malloc(sizeof(frame_t) * (size_t)P->nseg);
        double* tmp = dalloc((size_t)(P->S ? P->S : 1) * 3);
        P->pad_collision = 0;
        for (int side = 0; side < 2; ++side) {
            fk_spheres(P, side ? cfg->goal : cfg->start, fr, tmp);
            for (int j = 0; j < P->S; ++j) {
                double pot;
                if (potential_of(P, j, tmp + 3 * j, &pot)) P->pad_collision = 1;
            }
            for (int i = 0; i < SO_PAD; ++i)
                memcpy(P->pad_pos + ((size_t)(side * SO_PAD + i) * P->S) * 3, tmp, sizeof(double) * 3 * (size_t)P->S);
        }
        free(fr);
        free(tmp);
    }

    size_t KJN = (size_t)P->K * J * N;
    P->r_params = dalloc(KJN); P->r_noise = dalloc(KJN); P->r_nproj = dalloc(KJN);
    P->r_ctrl = dalloc(KJN); P->r_prob = dalloc(KJN); P->r_state = dalloc((size_t)P->K * N);
    size_t RJN = (size_t)(P->Kr ? P->Kr : 1) * J * N;
    P->tmp_params = dalloc(RJN); P->tmp_noise = dalloc(RJN); P->tmp_nproj = dalloc(RJN);
    P->tmp_ctrl = dalloc(RJN); P->tmp_prob = dalloc(RJN); P->tmp_state = dalloc((size_t)(P->Kr ? P->Kr : 1) * N);
    P->x_params = dalloc((size_t)J * N); P->x_noise = dalloc((size_t)J * N); P->x_nproj = dalloc((size_t)J * N);
    P->x_ctrl = dalloc((size_t)J * N); P->x_state = dalloc((size_t)N);
    P->last_traj = dalloc((size_t)J * N);
    P->best_traj = dalloc((size_t)J * N);
    memcpy(P->last_traj, P->theta, sizeof(double) * (size_t)J * N);
    memcpy(P->best_traj, P->theta, sizeof(double) * (size_t)J * N);
    return P;
}

int so_get_matrix(const so_problem* P, const char* which, int joint, double* out)
{
    size_t NN = (size_t)P->N * P->N, AA = (size_t)P->Nall * P->Nall;
    if (!strcmp(which, "Rinv")) memcpy(out, P->Rinv, NN * 8);
    else if (!strcmp(which, "L")) memcpy(out, P->L, NN * 8);
    else if (!strcmp(which, "M")) memcpy(out, P->M, NN * 8);
    else if (!strcmp(which, "Qinv")) memcpy(out, P->Qinv + (size_t)joint * NN, NN * 8);
    else if (!strcmp(which, "Rall")) memcpy(out, P->Rall, AA * 8);
    else if (!strcmp(which, "D0")) memcpy(out, P->Dpol[0], AA * 8);
    else if (!strcmp(which, "D1")) memcpy(out, P->Dpol[1], AA * 8);
    else if (!strcmp(which, "D2")) memcpy(out, P->Dpol[2], AA * 8);
    else { set_err("unknown matrix"); return -1; }
    return 0;
}

int so_get_theta(const so_problem* P, double* theta)
{
    memcpy(theta, P->theta, sizeof(double) * (size_t)P->J * P->N);
    return 0;
}

int so_set_theta(so_problem* P, const double* theta)
{
    memcpy(P->theta, theta, sizeof(double) * (size_t)P->J * P->N);
    return 0;
}

int so_get_pad_positions(const so_problem* P, double* out)
{
    memcpy(out, P->pad_pos, sizeof(double) * (size_t)2 * SO_PAD * P->S * 3);
    return 0;
}

/* ---------------------------------------------------------------- Task::execute */

typedef struct {
    double* traj;     /* Nall x J group trajectory */
    double* pos;      /* Nall x S x 3 */
    double* pot;      /* Nall x S */
    double* q;        /* J */
    frame_t* frames;  /* nseg */
    double* con;      /* N: constraint cost per free waypoint */
} exec_scratch;

static void scratch_init(const so_problem* P, exec_scratch* s)
{
    s->traj = dalloc((size_t)P->Nall * P->J);
    s->pos = dalloc((size_t)P->Nall * (P->S ? P->S : 1) * 3);
    s->pot = dalloc((size_t)P->Nall * (P->S ? P->S : 1));
    s->q = dalloc((size_t)P->J);
    s->frames = (frame_t*)malloc(sizeof(frame_t) * (size_t)P->nseg);
    s->con = dalloc((size_t)P->N);
}

static void scratch_free(exec_scratch* s)
{
    free(s->traj); free(s->pos); free(s->pot); free(s->q); free(s->frames); free(s->con);
}

/* StompOptimizer::handleJointLimits (stomp_optimizer.cpp:562-616) */
static void handle_joint_limits(const so_problem* P, double* traj)
{
    const int J = P->J, N = P->N;
    for (int jt = 0; jt < J; ++jt) {
        if (!P->joints[jt].has_limits) continue;
        double jmax = P->joints[jt].max, jmin = P->joints[jt].min;
        const double* Qi = P->Qinv + (size_t)jt * N * N;
        int count = 0;
        int violation;
        do {
            double max_abs = 1e-6, max_v = 0.0;
            int max_idx = 0;
            violation = 0;
            for (int i = SO_PAD; i < SO_PAD + N; ++i) {
                double amount = 0.0, absamt = 0.0;
                double v = traj[(size_t)i * J + jt];
                if (v > jmax) {
                    amount = jmax - v;
                    absamt = fabs(amount);
                } else if (v < jmin) {
                    amount = jmin - v;
                    absamt = fabs(amount);
                }
                if (absamt > max_abs) {
                    max_abs = absamt;
                    max_v = amount;
                    max_idx = i;
                    violation = 1;
                }
            }
            if (violation) {
                int k = max_idx - SO_PAD;
                double m = max_v / Qi[(size_t)k * N + k];
                for (int i = 0; i < N; ++i) traj[(size_t)(i + SO_PAD) * J + jt] += m * Qi[(size_t)i * N + k];
            }
            if (++count > 10) break;
        } while (violation);
    }
}

static double vec_sum(const so_problem* P, const double* x, int n);

static void execute_one(const so_problem* P, exec_scratch* sc, const double* params, double* costs,
                        int* collision_free, double* traj_out, int iteration_member, double* total, int* cons_ok)
{
    const int J = P->J, N = P->N, Nall = P->Nall, S = P->S;
    double* traj = sc->traj;
    /* group trajectory: padding = start/goal, free block = parameters (stomp_optimizer.cpp:1068-1071) */
    for (int i = 0; i < Nall; ++i)
        for (int d = 0; d < J; ++d) {
            double v;
            if (i < SO_PAD) v = P->cfg.start[d];
            else if (i >= SO_PAD + N) v = P->cfg.goal[d];
            else v = params[(size_t)d * N + (i - SO_PAD)];
            traj[(size_t)i * J + d] = v;
        }
    handle_joint_limits(P, traj);
    if (traj_out)
        for (int d = 0; d < J; ++d)
            for (int i = 0; i < N; ++i) traj_out[(size_t)d * N + i] = traj[(size_t)(i + SO_PAD) * J + d];

    /* performForwardKinematics (stomp_optimizer.cpp:618-709) */
    int cf = !(iteration_member == 0 && P->pad_collision);
    int cs = 1;   /* last_trajectory_constraints_satisfied_ (:1082) */
    memcpy(sc->pos, P->pad_pos, sizeof(double) * SO_PAD * S * 3);
    memcpy(sc->pos + (size_t)(SO_PAD + N) * S * 3, P->pad_pos + (size_t)SO_PAD * S * 3, sizeof(double) * SO_PAD * S * 3);
    for (int i = SO_PAD; i < SO_PAD + N; ++i) {
        for (int d = 0; d < J; ++d) sc->q[d] = traj[(size_t)i * J + d];
        fk_spheres(P, sc->q, sc->frames, sc->pos + (size_t)i * S * 3);
        for (int j = 0; j < S; ++j)
            if (potential_of(P, j, sc->pos + ((size_t)i * S + j) * 3, &sc->pot[(size_t)i * S + j])) cf = 0;
        /* constraint evaluators on the waypoint's segment frames (stomp_optimizer.cpp:1107-1115) */
        double con = 0.0;
        for (int c = 0; c < P->noc; ++c) {
            double cc;
            if (!oc_cost(&P->oc[c], sc->frames[P->oc[c].seg].R, &cc)) cs = 0;
            con += cc;
        }
        sc->con[i - SO_PAD] = con;
    }
    const double invTime = 1.0 / P->disc;
    double sum = 0.0;
    for (int i = SO_PAD; i < SO_PAD + N; ++i) {
        double state = 0.0, cum = 0.0;
        for (int j = 0; j < S; ++j) {
            double v[3] = {0.0, 0.0, 0.0};
            for (int k = -SO_DIFF_RULE_LENGTH / 2; k <= SO_DIFF_RULE_LENGTH / 2; ++k) {
                double c = invTime * DIFF_RULES[0][k + SO_DIFF_RULE_LENGTH / 2];
                const double* p = sc->pos + ((size_t)(i + k) * S + j) * 3;
                v[0] += c * p[0];
                v[1] += c * p[1];
                v[2] += c * p[2];
            }
            double vmag = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            /* stomp_optimizer.cpp:1100-1105 */
            cum += sc->pot[(size_t)i * S + j] * vmag;
            state += cum;
        }
        /* stomp_optimizer.cpp:1117-1151 */
        const double tq = P->torque ? torque_cost_at(P, traj, i) : 0.0;
        double c = P->cfg.obstacle_cost_weight * state + P->cfg.constraint_cost_weight * sc->con[i - SO_PAD] +
                   P->cfg.torque_cost_weight * tq;
        costs[i - SO_PAD] = c;
    }
    sum = vec_sum(P, costs, N);   /* costs.sum() :1155 */
    *collision_free = cf;
    if (cons_ok) *cons_ok = cs;
    if (total) *total = sum;
}

int so_execute(so_problem* P, const double* params, double* costs, int* collision_free, double* traj_out,
               int iteration_member, int* constraints_ok)
{
    exec_scratch sc;
    scratch_init(P, &sc);
    double tot;
    execute_one(P, &sc, params, costs, collision_free, traj_out, iteration_member, &tot, constraints_ok);
    scratch_free(&sc);
    return 0;
}

/* ---------------------------------------------------------------- PolicyImprovement */

/* CovariantTrajectoryPolicy::computeControlCosts, per-rollout overload
 * (covariant_trajectory_policy.cpp:228-255); x_free = parameters + noise_projected */
static void control_costs(const so_problem* P, const double* params, const double* nproj, double weight,
                          double* out, double* xall, double* call)
{
    const int J = P->J, N = P->N, Nall = P->Nall;
    for (int d = 0; d < J; ++d) {
        for (int i = 0; i < Nall; ++i) {
            if (i < SO_PAD) xall[i] = P->cfg.start[d];
            else if (i >= SO_PAD + N) xall[i] = P->cfg.goal[d];
            else xall[i] = params[(size_t)d * N + i - SO_PAD] + nproj[(size_t)d * N + i - SO_PAD];
            call[i] = 0.0;
        }
        for (int r = 0; r < SO_NUM_DIFF_RULES; ++r) {
            const double* D = P->Dpol[r];
            double wr = weight * P->cfg.smoothness_costs[r];
            for (int i = 0; i < Nall; ++i) {
                double acc = 0.0;
                if (P->cfg.dense) {
                    for (int c = 0; c < Nall; ++c) acc += D[(size_t)i * Nall + c] * xall[c];
                } else {
                    int c0 = i - 3 < 0 ? 0 : i - 3, c1 = i + 3 >= Nall ? Nall - 1 : i + 3;
                    for (int c = c0; c <= c1; ++c) acc += D[(size_t)i * Nall + c] * xall[c];
                }
                call[i] += wr * (acc * acc);
            }
        }
        double* o = out + (size_t)d * N;
        for (int t = 0; t < N; ++t) o[t] = call[t + SO_PAD];
        for (int i = 0; i < SO_PAD; ++i) {
            o[0] += call[i];
            o[N - 1] += call[Nall - (i + 1)];
        }
    }
}

/* The noise path's dense products (L z in MultivariateGaussian::sample and M eps in
 * computeProjectedNoise): k ascending, one rounding per multiply-add (fma) -- the engine's
 * contract for these two products, which it evaluates on the fp64 matrix cores (a
 * v_mfma_f64_16x16x4_f64 chain is exactly this fma chain; tools/probes/mfma_f64_probe.hip).
 * Hardware fma when the host has it, libm's correctly rounded fma otherwise (same bits). */
__attribute__((target("fma"))) static void matvec_fma_hw(const double* A, int n, const double* x, double* y,
                                                          int lower_only)
{
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        int kend = lower_only ? i + 1 : n;
        for (int k = 0; k < kend; ++k) s = __builtin_fma(A[(size_t)i * n + k], x[k], s);
        y[i] = s;
    }
}

static void matvec_fma(const double* A, int n, const double* x, double* y, int lower_only)
{
    static int hw = -1;
    if (hw < 0) hw = __builtin_cpu_supports("fma") ? 1 : 0;
    if (hw) {
        matvec_fma_hw(A, n, x, y, lower_only);
        return;
    }
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        int kend = lower_only ? i + 1 : n;
        for (int k = 0; k < kend; ++k) s = fma(A[(size_t)i * n + k], x[k], s);
        y[i] = s;
    }
}

static void matvec(const double* A, int n, const double* x, double* y, int lower_only);

/* the noise path's products under the configured contract: the engine's fma chain, or
 * (ref_arith) the reference's written order -- dense, k ascending, one rounding per multiply
 * and per add (Eigen 2's MatrixXd * VectorXd under SSE2 without FMA, CMakeLists.txt:34; its
 * internal blocking is third-party and not restated, parity unpinned there) */
static void noise_product(const so_problem* P, const double* A, int n, const double* x, double* y, int lower_only)
{
    if (P->cfg.ref_arith) matvec(A, n, x, y, 0);
    else matvec_fma(A, n, x, y, lower_only);
}

static void matvec(const double* A, int n, const double* x, double* y, int lower_only)
{
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        int kend = lower_only ? i + 1 : n;
        for (int k = 0; k < kend; ++k) s += A[(size_t)i * n + k] * x[k];
        y[i] = s;
    }
}

/* VectorXd::sum().  ref_arith 2: Eigen 2's SSE2 packet reduction (third party, unpinned: two
 * double lanes over the 16-byte-aligned data, lane k summing x[k], x[k + 2], ..., then lane 0 +
 * lane 1, then the odd last element); otherwise index order. */
static double vec_sum(const so_problem* P, const double* x, int n)
{
    if (P->cfg.ref_arith >= 2 && n >= 2) {
        double l0 = x[0], l1 = x[1];
        int i = 2;
        for (; i + 1 < n; i += 2) {
            l0 += x[i];
            l1 += x[i + 1];
        }
        double r = l0 + l1;
        for (; i < n; ++i) r += x[i];
        return r;
    }
    double s = x[0];
    for (int t = 1; t < n; ++t) s += x[t];
    return s;
}

/* Rollout::getCost (policy_improvement.cpp:149-156) */
static double rollout_cost(const so_problem* P, const double* state, const double* ctrl)
{
    double c = vec_sum(P, state, P->N);
    for (int d = 0; d < P->J; ++d) c += vec_sum(P, ctrl + (size_t)d * P->N, P->N);
    return c;
}

typedef struct { double cost; int idx; } cost_idx;
static int cmp_cost_idx(const void* a, const void* b)
{
    const cost_idx* x = (const cost_idx*)a;
    const cost_idx* y = (const cost_idx*)b;
    if (x->cost < y->cost) return -1;
    if (x->cost > y->cost) return 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

static void copy_rollout_out(so_problem* P, int r, int slot)
{
    size_t JN = (size_t)P->J * P->N;
    if (r >= 0) {
        memcpy(P->tmp_params + slot * JN, P->r_params + r * JN, JN * 8);
        memcpy(P->tmp_noise + slot * JN, P->r_noise + r * JN, JN * 8);
        memcpy(P->tmp_nproj + slot * JN, P->r_nproj + r * JN, JN * 8);
        memcpy(P->tmp_ctrl + slot * JN, P->r_ctrl + r * JN, JN * 8);
        memcpy(P->tmp_prob + slot * JN, P->r_prob + r * JN, JN * 8);
        memcpy(P->tmp_state + (size_t)slot * P->N, P->r_state + (size_t)r * P->N, (size_t)P->N * 8);
    } else {
        memcpy(P->tmp_params + slot * JN, P->x_params, JN * 8);
        memcpy(P->tmp_noise + slot * JN, P->x_noise, JN * 8);
        memcpy(P->tmp_nproj + slot * JN, P->x_nproj, JN * 8);
        memcpy(P->tmp_ctrl + slot * JN, P->x_ctrl, JN * 8);
        memset(P->tmp_prob + slot * JN, 0, JN * 8);
        memcpy(P->tmp_state + (size_t)slot * P->N, P->x_state, (size_t)P->N * 8);
    }
}

static void copy_rollout_in(so_problem* P, int slot, int r)
{
    size_t JN = (size_t)P->J * P->N;
    memcpy(P->r_params + r * JN, P->tmp_params + slot * JN, JN * 8);
    memcpy(P->r_noise + r * JN, P->tmp_noise + slot * JN, JN * 8);
    memcpy(P->r_nproj + r * JN, P->tmp_nproj + slot * JN, JN * 8);
    memcpy(P->r_ctrl + r * JN, P->tmp_ctrl + slot * JN, JN * 8);
    memcpy(P->r_prob + r * JN, P->tmp_prob + slot * JN, JN * 8);
    memcpy(P->r_state + (size_t)r * P->N, P->tmp_state + (size_t)slot * P->N, (size_t)P->N * 8);
}

/* PolicyImprovement::generateRollouts (policy_improvement.cpp:158-239) */
static void generate_rollouts(so_problem* P, int iteration_number, const double* sigma)
{
    const int J = P->J, N = P->N, K = P->K, Kr = P->Kr;
    size_t JN = (size_t)J * N;
    P->K_gen = K - Kr;
    if (!P->reused_next) {
        P->K_gen = K;
        if (Kr > 0) P->reused_next = 1;
    } else {
        int n = K + (P->extra_added ? 1 : 0);
        cost_idx* v = (cost_idx*)malloc(sizeof(cost_idx) * (size_t)n);
        for (int r = 0; r < K; ++r) {
            v[r].cost = rollout_cost(P, P->r_state + (size_t)r * N, P->r_ctrl + r * JN);
            v[r].idx = r;
        }
        if (P->extra_added) {
            v[K].cost = rollout_cost(P, P->x_state, P->x_ctrl);
            v[K].idx = -1;
            P->extra_added = 0;
        }
        qsort(v, (size_t)n, sizeof(cost_idx), cmp_cost_idx);
        if (P->rank_n + Kr > P->rank_cap) {
            int cap = P->rank_cap ? 2 * P->rank_cap : 64 * (Kr > 0 ? Kr : 1);
            while (cap < P->rank_n + Kr) cap *= 2;
            int* nl = (int*)realloc(P->rank_log, sizeof(int) * (size_t)cap);
            if (nl) {
                P->rank_log = nl;
                P->rank_cap = cap;
            }
        }
        if (P->rank_n + Kr <= P->rank_cap)
            for (int r = 0; r < Kr; ++r) P->rank_log[P->rank_n++] = v[r].idx;
        for (int r = 0; r < Kr; ++r) copy_rollout_out(P, v[r].idx, r);
        for (int r = 0; r < Kr; ++r) {
            int dst = P->K_gen + r;
            copy_rollout_in(P, r, dst);
            for (int d = 0; d < J; ++d)
                for (int t = 0; t < N; ++t)
                    P->r_noise[dst * JN + (size_t)d * N + t] =
                        P->r_params[dst * JN + (size_t)d * N + t] - P->theta[(size_t)d * N + t];
        }
        free(v);
    }
    /* d outer, r inner in the reference; the (d, r) samples are independent (counter-based
     * normals), so the threads of a multi-core run may take them in any order */
    const int K_gen = P->K_gen;
    int nthreads = P->cfg.threads > 0 ? P->cfg.threads : 1;
    (void)nthreads;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
        double* z = dalloc((size_t)N);
        double* tmp = dalloc((size_t)N);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int dr = 0; dr < J * K_gen; ++dr) {
            const int d = dr / K_gen, r = dr % K_gen;
            so_normals(P->cfg.seed, iteration_number, d, r, N, z);
            /* MultivariateGaussian::sample: output = mean + L * z (multivariate_gaussian.h:88-94) */
            noise_product(P, P->L, N, z, tmp, !P->cfg.dense);
            double* nz = P->r_noise + r * JN + (size_t)d * N;
            double* pr = P->r_params + r * JN + (size_t)d * N;
            for (int t = 0; t < N; ++t) {
                nz[t] = sigma[d] * (0.0 + tmp[t]);
                pr[t] = P->theta[(size_t)d * N + t] + nz[t];
            }
        }
        free(z);
        free(tmp);
    }
}

/* fixed-order blocked sum over rollouts; returns sum_r vals[r*stride] */
static double blocked_sum(const double* vals, size_t stride, int K, int B)
{
    double total = 0.0;
    for (int b0 = 0; b0 < K; b0 += B) {
        double part = 0.0;
        int b1 = b0 + B < K ? b0 + B : K;
        for (int r = b0; r < b1; ++r) part += vals[(size_t)r * stride];
        total += part;
    }
    return total;
}

int so_iterate(so_problem* P, int iteration_number, so_iter_out* out)
{
    const int J = P->J, N = P->N, K = P->K, Nall = P->Nall;
    size_t JN = (size_t)J * N;
    int iteration_member = iteration_number - 1;
    /* noise schedule (policy_improvement_loop.cpp:155-160) */
    double* sigma = dalloc((size_t)J);
    for (int d = 0; d < J; ++d) sigma[d] = P->cfg.noise_stddev[d] * pow(P->cfg.noise_decay[d], iteration_number - 1);
    generate_rollouts(P, iteration_number, sigma);
    free(sigma);
    int nthreads = P->cfg.threads > 0 ? P->cfg.threads : 1;
    (void)nthreads;
    /* computeProjectedNoise for all K (policy_improvement.cpp:283-290, 473-482); rows independent */
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (int r = 0; r < K; ++r)
        for (int d = 0; d < J; ++d)
            noise_product(P, P->M, N, P->r_noise + r * JN + (size_t)d * N, P->r_nproj + r * JN + (size_t)d * N, 0);

    /* Task::execute for each generated rollout (policy_improvement_loop.cpp:165-170) */
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
        exec_scratch sc;
        scratch_init(P, &sc);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int r = 0; r < P->K_gen; ++r) {
            int cf;
            execute_one(P, &sc, P->r_params + r * JN, P->r_state + (size_t)r * N, &cf, NULL, iteration_member, NULL, NULL);
        }
        scratch_free(&sc);
    }

    /* setRolloutCosts -> computeRolloutControlCosts for all K (policy_improvement.cpp:262-281) */
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
        double* xall = dalloc((size_t)Nall);
        double* call = dalloc((size_t)Nall);
        double w = 0.5 * P->cfg.smoothness_cost_weight;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int r = 0; r < K; ++r) control_costs(P, P->r_params + r * JN, P->r_nproj + r * JN, w, P->r_ctrl + r * JN, xall, call);
        free(xall);
        free(call);
    }

    /* improvePolicy (policy_improvement.cpp:385-401) */
    {
        double* cum = dalloc((size_t)K * JN);   /* [K][J][N] cumulative costs */
        for (int r = 0; r < K; ++r)
            for (int d = 0; d < J; ++d) {
                double* c = cum + r * JN + (size_t)d * N;
                for (int t = 0; t < N; ++t) c[t] = P->r_state[(size_t)r * N + t] + P->r_ctrl[r * JN + (size_t)d * N + t];
                if (P->cfg.use_cumulative_costs)
                    for (int t = N - 2; t >= 0; --t) c[t] += c[t + 1];
            }
        double* upd = dalloc((size_t)N);
        double* del = dalloc((size_t)N);
        double* tmp = dalloc((size_t)K);
        for (int d = 0; d < J; ++d) {
            for (int t = 0; t < N; ++t) {
                size_t off = (size_t)d * N + t;
                double mn = cum[off], mx = mn;
                for (int r = 1; r < K; ++r) {
                    double c = cum[r * JN + off];
                    if (c < mn) mn = c;
                    if (c > mx) mx = c;
                }
                double denom = mx - mn;
                if (denom < 1e-8) denom = 1e-8;
                for (int r = 0; r < K; ++r)
                    P->r_prob[r * JN + off] = P->cfg.ref_arith >= 3 ? exp(-10.0 * (cum[r * JN + off] - mn) / denom)
                                                                    : dm_exp(-10.0 * (cum[r * JN + off] - mn) / denom);
                double psum = blocked_sum(P->r_prob + off, JN, K, P->B);
                for (int r = 0; r < K; ++r) P->r_prob[r * JN + off] /= psum;
                /* computeParameterUpdates (policy_improvement.cpp:370-383) */
                for (int r = 0; r < K; ++r) tmp[r] = P->r_noise[r * JN + off] * P->r_prob[r * JN + off];
                upd[t] = blocked_sum(tmp, 1, K, P->B);
            }
            matvec(P->M, N, upd, del, 0);
            /* updateParameters (covariant_trajectory_policy.cpp:306-342) */
            for (int t = 0; t < N; ++t) P->theta[(size_t)d * N + t] += 1.0 * del[t];
        }
        free(cum); free(upd); free(del); free(tmp);
    }

    /* noiseless rollout (policy_improvement_loop.cpp:180-192) */
    {
        exec_scratch sc;
        scratch_init(P, &sc);
        execute_one(P, &sc, P->theta, P->x_state, &P->last_cf, P->last_traj, iteration_member, &P->last_cost,
                    &P->last_cs);
        scratch_free(&sc);
        /* addExtraRollouts (policy_improvement.cpp:443-462) */
        memcpy(P->x_params, P->theta, JN * 8);
        for (size_t k = 0; k < JN; ++k) P->x_noise[k] = P->x_params[k] - P->theta[k];
        for (int d = 0; d < J; ++d) noise_product(P, P->M, N, P->x_noise + (size_t)d * N, P->x_nproj + (size_t)d * N, 0);
        double* xall = dalloc((size_t)Nall);
        double* call = dalloc((size_t)Nall);
        control_costs(P, P->x_params, P->x_nproj, 0.5 * P->cfg.smoothness_cost_weight, P->x_ctrl, xall, call);
        free(xall);
        free(call);
        P->extra_added = 1;
    }
    if (out) {
        out->cost = P->last_cost;
        out->collision_free = P->last_cf;
        out->constraints_satisfied = P->last_cs;
    }
    return 0;
}

/* StompOptimizer::optimize loop (stomp_optimizer.cpp:249-359) */
int so_optimize(so_problem* P, so_stats* st, double* costs_per_it)
{
    const size_t JN = (size_t)P->J * P->N;
    so_stats s;
    s.collision_success_iteration = -1;
    s.success_iteration = -1;
    s.success = 0;
    s.last_improvement_iteration = -1;
    int cfi = 0;
    double best_cost = 0.0;
    int it;
    for (it = 0; it < P->cfg.max_iterations; it++) {
        so_iter_out o;
        so_iterate(P, it + 1, &o);
        /* stomp_optimizer.cpp:301-339 */
        const int ok = o.collision_free && o.constraints_satisfied;
        if (ok) cfi++;
        else cfi = 0;
        if (o.collision_free && s.collision_success_iteration == -1) s.collision_success_iteration = it;
        if (ok && s.success_iteration == -1) {
            s.success_iteration = it;
            s.success = 1;
        }
        double cost = o.cost;
        if (costs_per_it) costs_per_it[it] = cost;
        if (it == 0) {
            memcpy(P->best_traj, P->last_traj, JN * 8);
            best_cost = cost;
        } else if (cost < best_cost && ok) {
            memcpy(P->best_traj, P->last_traj, JN * 8);
            best_cost = cost;
            s.last_improvement_iteration = it;
        }
        if (cfi >= P->cfg.max_iterations_after_collision_free) {
            it++;
            break;
        }
    }
    s.iterations = it;
    s.best_cost = best_cost;
    if (st) *st = s;
    return 0;
}

/* STOMPStatistics.torques (stomp_optimizer.cpp:384-398): group_trajectory_ = best, then per free
 * waypoint sum_j |tau_j| of getTorques */
int so_get_best_torques(const so_problem* P, double* out)
{
    if (!P->chain) { set_err("no torque chain (segment inertias not given)"); return -1; }
    const int J = P->J, N = P->N, Nall = P->Nall;
    double* traj = dalloc((size_t)Nall * J);
    for (int i = 0; i < Nall; ++i)
        for (int d = 0; d < J; ++d)
            traj[(size_t)i * J + d] = i < SO_PAD ? P->cfg.start[d]
                                    : (i >= SO_PAD + N ? P->cfg.goal[d] : P->best_traj[(size_t)d * N + (i - SO_PAD)]);
    for (int t = 0; t < N; ++t) out[t] = torque_cost_at(P, traj, t + SO_PAD);
    free(traj);
    return 0;
}

int so_get_best_trajectory(const so_problem* P, double* traj)
{
    memcpy(traj, P->best_traj, sizeof(double) * (size_t)P->J * P->N);
    return 0;
}

int so_get_last_trajectory(const so_problem* P, double* traj)
{
    memcpy(traj, P->last_traj, sizeof(double) * (size_t)P->J * P->N);
    return 0;
}

int so_reuse_log(const so_problem* P, int* out, int cap)
{
    const int n = P->rank_n < cap ? P->rank_n : cap;
    if (out && n > 0) memcpy(out, P->rank_log, sizeof(int) * (size_t)n);
    return P->rank_n;
}

int so_get_rollouts(const so_problem* P, const char* which, double* out)
{
    size_t KJN = (size_t)P->K * P->J * P->N;
    if (!strcmp(which, "params")) memcpy(out, P->r_params, KJN * 8);
    else if (!strcmp(which, "noise")) memcpy(out, P->r_noise, KJN * 8);
    else if (!strcmp(which, "noise_projected")) memcpy(out, P->r_nproj, KJN * 8);
    else if (!strcmp(which, "control_costs")) memcpy(out, P->r_ctrl, KJN * 8);
    else if (!strcmp(which, "probabilities")) memcpy(out, P->r_prob, KJN * 8);
    else if (!strcmp(which, "state_costs")) memcpy(out, P->r_state, (size_t)P->K * P->N * 8);
    else if (!strcmp(which, "x_params")) memcpy(out, P->x_params, (size_t)P->J * P->N * 8);
    else if (!strcmp(which, "x_noise")) memcpy(out, P->x_noise, (size_t)P->J * P->N * 8);
    else if (!strcmp(which, "x_noise_projected")) memcpy(out, P->x_nproj, (size_t)P->J * P->N * 8);
    else if (!strcmp(which, "x_control_costs")) memcpy(out, P->x_ctrl, (size_t)P->J * P->N * 8);
    else if (!strcmp(which, "x_state_costs")) memcpy(out, P->x_state, (size_t)P->N * 8);
    else { set_err("unknown rollout field"); return -1; }
    return 0;
}
