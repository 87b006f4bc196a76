// kernels.hip -- gfx950 kernels of the STOMP noisy-rollout cost engine.
//
// Floating-point contract (shared with the CPU oracle): fp64, one
// rounding per operation (-ffp-contract=off, no FMA contraction), every sum
// sequential in the reference's index order, sums over rollouts in fixed
// 64-rollout blocks.  Under that contract the kernels reproduce the oracle bit
// for bit; none of them uses MFMA (no dense contraction in fp64 with non-fused
// rounding).
#include "kernels.h"
#include "stomp_math.h"

namespace stomp {

// ============================================================== noise / projection / control cost
// PolicyImprovement::generateRollouts (policy_improvement.cpp:228-236: eps = sigma * L z,
// params = theta + eps), computeProjectedNoise (:473-482: M eps) and
// CovariantTrajectoryPolicy::computeControlCosts (covariant_trajectory_policy.cpp:228-255),
// fused: one workgroup per (RT rollouts, joint); lane i owns time step i; L and M are
// read transposed so a wave's loads are 512 contiguous bytes; z, eps and the padded
// trajectory live in LDS.
template <int BLOCK, int RT>
__global__ __launch_bounds__(BLOCK) void k_noise(NoiseArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int N = a.N, Nall = a.Nall, J = a.J;
    double* zs = lds;             // RT*N
    double* eps = zs + RT * N;    // RT*N
    double* xs = eps + RT * N;    // RT*Nall
    double* cs = xs + RT * Nall;  // RT*Nall
    const int d = blockIdx.y;
    const int r0 = blockIdx.x * RT;
    const int tid = threadIdx.x;
    const double sig = a.sigma.v[d];

    bool gen[RT];
#pragma unroll
    for (int rr = 0; rr < RT; ++rr) {
        const int r = r0 + rr;
        const int g = a.first_global + r;
        gen[rr] = (r < a.K_loc) && !a.zero_noise && g < a.K_gen_global;
        if (r >= a.K_loc) {
            for (int t = tid; t < N; t += BLOCK) { zs[rr * N + t] = 0.0; eps[rr * N + t] = 0.0; }
        } else if (gen[rr]) {
            for (int p = tid; 2 * p < N; p += BLOCK) {
                double z0, z1;
                normal_pair(a.seed, a.iteration, d, g, p, &z0, &z1);
                zs[rr * N + 2 * p] = z0;
                if (2 * p + 1 < N) zs[rr * N + 2 * p + 1] = z1;
            }
        } else if (a.zero_noise) {
            // addExtraRollouts: noise = parameters - theta (policy_improvement.cpp:464-471) with
            // parameters == theta, i.e. +0.0 exactly
            for (int t = tid; t < N; t += BLOCK) {
                eps[rr * N + t] = 0.0;
                a.noise[((size_t)r * J + d) * N + t] = 0.0;
            }
        } else {
            // reused rollout: its noise was re-based on the new theta by the reuse kernel
            for (int t = tid; t < N; t += BLOCK) eps[rr * N + t] = a.noise[((size_t)r * J + d) * N + t];
        }
    }
    __syncthreads();

    const int i = tid;
    bool any_gen = false;
#pragma unroll
    for (int rr = 0; rr < RT; ++rr) any_gen |= gen[rr];
    if (any_gen && i < N) {
        double acc[RT];
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) acc[rr] = 0.0;
        for (int k = 0; k <= i; ++k) {
            const double lk = a.LT[(size_t)k * N + i];
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) acc[rr] += lk * zs[rr * N + k];
        }
        const double th = a.theta[(size_t)d * N + i];
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            if (!gen[rr]) continue;
            const int r = r0 + rr;
            const double e = sig * (0.0 + acc[rr]);
            const double p = th + e;
            a.noise[((size_t)r * J + d) * N + i] = e;
            a.params[((size_t)r * J + d) * N + i] = p;
            eps[rr * N + i] = e;
        }
    }
    __syncthreads();

    if (i < N) {
        double acc[RT];
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) acc[rr] = 0.0;
        for (int k = 0; k < N; ++k) {
            const double mk = a.MT[(size_t)k * N + i];
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) acc[rr] += mk * eps[rr * N + k];
        }
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            const int r = r0 + rr;
            double p = 0.0;
            if (r < a.K_loc) p = a.params[((size_t)r * J + d) * N + i];
            xs[rr * Nall + i + 6] = p + acc[rr];
        }
    }
    for (int idx = tid; idx < RT * 12; idx += BLOCK) {
        const int rr = idx / 12, row = idx % 12;
        xs[rr * Nall + (row < 6 ? row : N + row)] = row < 6 ? a.start[d] : a.goal[d];
    }
    __syncthreads();

    for (int ii = tid; ii < Nall; ii += BLOCK) {
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            double call = 0.0;
#pragma unroll
            for (int rule = 0; rule < 3; ++rule) {
                const double wr = a.wr[rule];
                if (wr == 0.0) continue;   // adds +0.0 in the reference: exact to skip
                double acc = 0.0;
                const int c0 = ii - 3 < 0 ? 0 : ii - 3;
                const int c1 = ii + 3 >= Nall ? Nall - 1 : ii + 3;
                for (int c = c0; c <= c1; ++c) acc += a.dcoef[rule][c - ii + 3] * xs[rr * Nall + c];
                call += wr * (acc * acc);
            }
            cs[rr * Nall + ii] = call;
        }
    }
    __syncthreads();

    if (i < N) {
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            const int r = r0 + rr;
            if (r >= a.K_loc) continue;
            const double* c = cs + rr * Nall;
            double o = c[i + 6];
            if (N == 1) {
                for (int q = 0; q < 6; ++q) { o += c[q]; o += c[Nall - 1 - q]; }
            } else if (i == 0) {
                for (int q = 0; q < 6; ++q) o += c[q];
            } else if (i == N - 1) {
                for (int q = 0; q < 6; ++q) o += c[Nall - 1 - q];
            }
            a.control[((size_t)r * J + d) * N + i] = o;
        }
    }
}

void launch_noise(const NoiseArgs& a, int rt, hipStream_t s)
{
    const int block = a.Nall <= 128 ? 128 : 256;
    const size_t lds_per = (size_t)(2 * a.N + 2 * a.Nall) * sizeof(double);
    if (rt == 1) {
        dim3 grid((a.K_loc + 0) / 1, a.J);
        if (block == 128) hipLaunchKernelGGL((k_noise<128, 1>), grid, dim3(128), lds_per, s, a);
        else hipLaunchKernelGGL((k_noise<256, 1>), grid, dim3(256), lds_per, s, a);
    } else {
        dim3 grid((a.K_loc + 3) / 4, a.J);
        if (block == 128) hipLaunchKernelGGL((k_noise<128, 4>), grid, dim3(128), 4 * lds_per, s, a);
        else hipLaunchKernelGGL((k_noise<256, 4>), grid, dim3(256), 4 * lds_per, s, a);
    }
}

// ============================================================== rollout cost (Task::execute)
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

// frame = parent * Frame(rot, trans) * Frame(Rot2(axis, q), 0)   (KDL Rotation::Rot2 formula)
__device__ __forceinline__ void compose(const DevSegment& sg, const Frame* parent, double q, Frame& out)
{
    Frame pose;
    if (sg.q_index >= 0) {
        double st, ct;
        det_sincos(q, &st, &ct);
        const double* a = sg.axis;
        double vt = 1.0 - ct;
        double m_vt_0 = vt * a[0], m_vt_1 = vt * a[1], m_vt_2 = vt * a[2];
        double m_st_0 = a[0] * st, m_st_1 = a[1] * st, m_st_2 = a[2] * st;
        double m_vt_0_1 = m_vt_0 * a[1], m_vt_0_2 = m_vt_0 * a[2], m_vt_1_2 = m_vt_1 * a[2];
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
        rotmul(sg.rot, Rq, pose.R);
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
    rotmul(parent->R, pose.R, out.R);
#pragma unroll
    for (int i = 0; i < 3; ++i)
        out.p[i] = parent->R[3 * i + 0] * pose.p[0] + parent->R[3 * i + 1] * pose.p[1] +
                   parent->R[3 * i + 2] * pose.p[2] + parent->p[i];
}

__device__ __forceinline__ void apply(const Frame& f, const double* v, double* o)
{
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = f.R[3 * i + 0] * v[0] + f.R[3 * i + 1] * v[1] + f.R[3 * i + 2] * v[2] + f.p[i];
}

// distance_field::getDistanceGradient cell rule (3rd party; call site stomp_collision_space.h:190)
__device__ __forceinline__ double sdf_distance(const DevModel& m, const double* p)
{
    const double fx = round((p[0] - m.ox) / m.res);
    const double fy = round((p[1] - m.oy) / m.res);
    const double fz = round((p[2] - m.oz) / m.res);
    if (!(fx >= 1.0 && fy >= 1.0 && fz >= 1.0 && fx < (double)(m.nx - 1) && fy < (double)(m.ny - 1) &&
          fz < (double)(m.nz - 1)))
        return 0.0;
    const int ix = (int)fx, iy = (int)fy, iz = (int)fz;
    return (double)m.sdf[((size_t)ix * m.ny + iy) * m.nz + iz];
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

__device__ __forceinline__ Frame slot_get(int s, const Frame& f0, const Frame& f1, const Frame& f2, const Frame& f3)
{
    return s == 0 ? f0 : (s == 1 ? f1 : (s == 2 ? f2 : f3));
}

__device__ __forceinline__ void slot_put(int s, const Frame& v, Frame& f0, Frame& f1, Frame& f2, Frame& f3)
{
    if (s == 0) f0 = v;
    else if (s == 1) f1 = v;
    else if (s == 2) f2 = v;
    else f3 = v;
}

__device__ __forceinline__ void wave_argmax(double& v, int& idx)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double ov = __shfl_xor(v, off, 64);
        const int oi = __shfl_xor(idx, off, 64);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
}

// StompOptimizer::execute (stomp_optimizer.cpp:1063-1165) for one rollout per workgroup:
// handleJointLimits (:562-616) on the LDS copy of the trajectory, then per free waypoint
// (lane t) the FK program, sphere positions, distance-field gathers, 7-tap FD velocity of
// every sphere over t-3..t+3 (:683-698) and the sphere-ordered cumulative cost (:1096-1105).
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_rollout_cost(DevModel m, const double* params, long long stride,
                                                       double* state_out, uint8_t* cf_out, double* traj_out,
                                                       double* total_out, int iteration_member)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int NW = BLOCK / 64;
    const int J = m.J, N = m.N, Nall = m.Nall, S = m.S;
    double* traj = lds;                              // J*N
    double* buf = traj + J * N;                      // kRunMax*Nall*3
    double* red_v = buf + kRunMax * Nall * 3;        // NW
    int* red_i = (int*)(red_v + NW);                 // NW
    int* flag = red_i + NW;                          // 1
    const int e = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const double* prm = params + (long long)e * stride;
    for (int idx = tid; idx < J * N; idx += BLOCK) traj[idx] = prm[idx];
    if (tid == 0) *flag = 0;
    __syncthreads();

    // ---- handleJointLimits
    for (int j = 0; j < J; ++j) {
        if (!m.has_limits[j]) continue;
        const double jmax = m.jmax[j], jmin = m.jmin[j];
        const double* Q = m.QT + (size_t)j * N * N;
        for (int pass = 0; pass < 11; ++pass) {
            double cand = -1.0;
            int ci = 0x7fffffff;
            if (tid < N) {
                const double v = traj[j * N + tid];
                double amount = 0.0, absamt = 0.0;
                if (v > jmax) { amount = jmax - v; absamt = fabs(amount); }
                else if (v < jmin) { amount = jmin - v; absamt = fabs(amount); }
                if (absamt > 1e-6) { cand = absamt; ci = tid; }
            }
            wave_argmax(cand, ci);
            if (lane == 0) { red_v[wv] = cand; red_i[wv] = ci; }
            __syncthreads();
            double bv = red_v[0];
            int bi = red_i[0];
            for (int w = 1; w < NW; ++w) {
                const double ov = red_v[w];
                const int oi = red_i[w];
                if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
            }
            double mult = 0.0;
            if (bv >= 0.0) {
                const double v = traj[j * N + bi];
                const double amount = v > jmax ? jmax - v : jmin - v;
                mult = amount / Q[(size_t)bi * N + bi];
            }
            __syncthreads();       // red_v/red_i and traj[j][bi] consumed by every wave
            if (bv < 0.0) break;   // no violation: uniform across the block
            if (tid < N) traj[j * N + tid] += mult * Q[(size_t)bi * N + tid];
            __syncthreads();
        }
    }
    if (traj_out)
        for (int idx = tid; idx < J * N; idx += BLOCK) traj_out[(long long)e * J * N + idx] = traj[idx];

    // ---- forward kinematics + collision cost
    const int t = tid;
    const bool act = t < N;
    double cum = 0.0, state = 0.0;
    bool col = false;
    Frame f0, f1, f2, f3, cur;
    for (int op = 0; op < m.nops; ++op) {
        const FkOp o = m.ops[op];
        if (act) {
            if (o.seg >= 0) {
                const DevSegment& sg = m.segs[o.seg];
                const double q = sg.q_index >= 0 ? traj[sg.q_index * N + t] : 0.0;
                Frame nf;
                if (o.from < 0) {
                    compose(sg, nullptr, q, nf);
                } else {
                    const Frame par = slot_get(o.from, f0, f1, f2, f3);
                    compose(sg, &par, q, nf);
                }
                slot_put(o.to, nf, f0, f1, f2, f3);
            }
            cur = slot_get(o.to, f0, f1, f2, f3);
        }
        const int nb = o.sph_end - o.sph_begin;
        if (nb == 0) continue;   // uniform: frame-only step
        double dist[kRunMax];
#pragma unroll
        for (int q = 0; q < kRunMax; ++q) {
            dist[q] = 0.0;
            if (q < nb && act) {
                const DevSphere& sp = m.sph[o.sph_begin + q];
                double p[3];
                apply(cur, sp.pos, p);
                double* b = buf + ((size_t)q * Nall + t + 6) * 3;
                b[0] = p[0]; b[1] = p[1]; b[2] = p[2];
                dist[q] = sdf_distance(m, p);
            }
        }
        for (int idx = tid; idx < nb * 12; idx += BLOCK) {
            const int q = idx / 12, row = idx % 12;
            const int prow = row < 6 ? row : N + row;
            const double* src = m.pad_pos + ((size_t)row * S + o.sph_begin + q) * 3;
            double* b = buf + ((size_t)q * Nall + prow) * 3;
            b[0] = src[0]; b[1] = src[1]; b[2] = src[2];
        }
        __syncthreads();
        if (act) {
#pragma unroll
            for (int q = 0; q < kRunMax; ++q) {
                if (q < nb) {
                    const DevSphere& sp = m.sph[o.sph_begin + q];
                    double v0 = 0.0, v1 = 0.0, v2 = 0.0;
#pragma unroll
                    for (int k = 0; k < 7; ++k) {
                        const double c = m.vel_coef[k];
                        const double* b = buf + ((size_t)q * Nall + t + 3 + k) * 3;
                        v0 += c * b[0];
                        v1 += c * b[1];
                        v2 += c * b[2];
                    }
                    const double vmag = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
                    const double pot = potential(sp, dist[q]);
                    col |= dist[q] <= sp.radius;
                    cum += pot * vmag;
                    state += cum;
                }
            }
        }
        __syncthreads();
    }
    if (col) *flag = 1;   // benign race: every writer stores 1
    double cost = 0.0;
    if (act) {
        cost = m.w_obs * state + m.w_con * 0.0 + m.w_tq * 0.0;
        state_out[(long long)e * N + t] = cost;
        buf[t] = cost;
    }
    __syncthreads();
    if (tid == 0) {
        const bool cf = !(*flag) && !(iteration_member == 0 && m.pad_collision);
        if (cf_out) cf_out[e] = cf ? 1 : 0;
        if (total_out) {
            double s = buf[0];
            for (int k = 1; k < N; ++k) s += buf[k];
            total_out[e] = s;
        }
    }
}

void launch_rollout_cost(const DevModel& m, const double* params, long long stride, int num, double* state_out,
                         uint8_t* cf_out, double* traj_out, double* total_out, int iteration_member, hipStream_t s)
{
    if (num <= 0) return;
    const int block = m.N <= 64 ? 64 : (m.N <= 128 ? 128 : 256);
    const size_t lds = ((size_t)m.J * m.N + (size_t)kRunMax * m.Nall * 3 + 4) * sizeof(double) + 4 * 4 * sizeof(int) + 16;
    if (block == 64)
        hipLaunchKernelGGL((k_rollout_cost<64>), dim3(num), dim3(64), lds, s, m, params, stride, state_out, cf_out,
                           traj_out, total_out, iteration_member);
    else if (block == 128)
        hipLaunchKernelGGL((k_rollout_cost<128>), dim3(num), dim3(128), lds, s, m, params, stride, state_out, cf_out,
                           traj_out, total_out, iteration_member);
    else
        hipLaunchKernelGGL((k_rollout_cost<256>), dim3(num), dim3(256), lds, s, m, params, stride, state_out, cf_out,
                           traj_out, total_out, iteration_member);
}

// padding-point sphere positions: iteration-0 full FK of start (rows 0..5) and goal (rows 6..11)
__global__ void k_pad_fk(DevModel m, const double* start, const double* goal, double* pad_pos, int* pad_cf)
{
    const int side = threadIdx.x;
    if (side > 1) return;
    const double* q = side ? goal : start;
    Frame f0, f1, f2, f3, cur;
    bool col = false;
    for (int op = 0; op < m.nops; ++op) {
        const FkOp o = m.ops[op];
        if (o.seg >= 0) {
            const DevSegment& sg = m.segs[o.seg];
            const double qv = sg.q_index >= 0 ? q[sg.q_index] : 0.0;
            Frame nf;
            if (o.from < 0) {
                compose(sg, nullptr, qv, nf);
            } else {
                const Frame par = slot_get(o.from, f0, f1, f2, f3);
                compose(sg, &par, qv, nf);
            }
            slot_put(o.to, nf, f0, f1, f2, f3);
        }
        cur = slot_get(o.to, f0, f1, f2, f3);
        for (int s = o.sph_begin; s < o.sph_end; ++s) {
            double p[3];
            apply(cur, m.sph[s].pos, p);
            if (sdf_distance(m, p) <= m.sph[s].radius) col = true;
            for (int row = 0; row < 6; ++row)
                for (int c = 0; c < 3; ++c) pad_pos[((size_t)(side * 6 + row) * m.S + s) * 3 + c] = p[c];
        }
    }
    if (col) atomicOr(pad_cf, 1);
}

void launch_pad_fk(const DevModel& m, const double* start, const double* goal, double* pad_pos, int* pad_cf,
                   hipStream_t s)
{
    hipLaunchKernelGGL(k_pad_fk, dim3(1), dim3(64), 0, s, m, start, goal, pad_pos, pad_cf);
}

// ============================================================== weights
// computeRolloutCumulativeCosts (policy_improvement.cpp:301-320)
__global__ void k_cumulative(WeightArgs a)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.K_loc * a.J) return;
    const int r = idx / a.J, d = idx % a.J;
    const int N = a.N;
    double* c = a.cum + ((size_t)r * a.J + d) * N;
    const double* st = a.state + (size_t)r * N;
    const double* ct = a.control + ((size_t)r * a.J + d) * N;
    for (int t = 0; t < N; ++t) c[t] = st[t] + ct[t];
    if (a.use_cumulative)
        for (int t = N - 2; t >= 0; --t) c[t] += c[t + 1];
}

void launch_cumulative(const WeightArgs& a, hipStream_t s)
{
    const int n = a.K_loc * a.J;
    hipLaunchKernelGGL(k_cumulative, dim3((n + 255) / 256), dim3(256), 0, s, a);
}

// computeRolloutProbabilities (:322-368) + computeParameterUpdates (:370-383) before the
// projection.  Lane = time step of one joint column, waves split the 64-rollout blocks;
// min/max are order-free, the two sums use the canonical blocked order.
__global__ __launch_bounds__(256) void k_weights(WeightArgs a)
{
    __shared__ double mnl[4][64], mxl[4][64];
    __shared__ double part[64][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int d = blockIdx.y, t = blockIdx.x * 64 + lane;
    const int N = a.N, J = a.J, K = a.K_loc;
    const int nb = (K + kSumBlock - 1) / kSumBlock;
    const bool act = t < N;
    const size_t col = (size_t)d * N + t;
    const size_t JN = (size_t)J * N;
    auto cost = [&](int r) -> double {
        if (a.cum) return a.cum[(size_t)r * JN + col];
        return a.state[(size_t)r * N + t] + a.control[(size_t)r * JN + col];
    };
    double mn = 0.0, mx = 0.0;
    bool have = false;
    if (act) {
        for (int b = w; b < nb; b += 4) {
            const int r1 = min(K, (b + 1) * kSumBlock);
            for (int r = b * kSumBlock; r < r1; ++r) {
                const double c = cost(r);
                if (!have) { mn = c; mx = c; have = true; }
                else { if (c < mn) mn = c; if (c > mx) mx = c; }
            }
        }
    }
    mnl[w][lane] = have ? mn : __builtin_inf();
    mxl[w][lane] = have ? mx : -__builtin_inf();
    __syncthreads();
    mn = mnl[0][lane];
    mx = mxl[0][lane];
    for (int q = 1; q < 4; ++q) {
        if (mnl[q][lane] < mn) mn = mnl[q][lane];
        if (mxl[q][lane] > mx) mx = mxl[q][lane];
    }
    double denom = mx - mn;
    if (denom < 1e-8) denom = 1e-8;
    if (act) {
        for (int b = w; b < nb; b += 4) {
            const int r1 = min(K, (b + 1) * kSumBlock);
            double ps = 0.0;
            for (int r = b * kSumBlock; r < r1; ++r) {
                const double p = det_exp(-10.0 * (cost(r) - mn) / denom);
                a.prob[(size_t)r * JN + col] = p;
                ps += p;
            }
            part[b][lane] = ps;
        }
    }
    __syncthreads();
    double psum = 0.0;
    for (int b = 0; b < nb; ++b) psum += part[b][lane];
    __syncthreads();
    if (act) {
        for (int b = w; b < nb; b += 4) {
            const int r1 = min(K, (b + 1) * kSumBlock);
            double us = 0.0;
            for (int r = b * kSumBlock; r < r1; ++r) {
                const double pn = a.prob[(size_t)r * JN + col] / psum;
                a.prob[(size_t)r * JN + col] = pn;
                us += a.noise[(size_t)r * JN + col] * pn;
            }
            part[b][lane] = us;
        }
    }
    __syncthreads();
    if (w == 0 && act) {
        double u = 0.0;
        for (int b = 0; b < nb; ++b) u += part[b][lane];
        a.u[col] = u;
    }
}

void launch_weights(const WeightArgs& a, hipStream_t s)
{
    dim3 grid((a.N + 63) / 64, a.J);
    hipLaunchKernelGGL(k_weights, grid, dim3(256), 0, s, a);
}

// delta = M u (policy_improvement.cpp:380), theta += 1.0 * delta (covariant_trajectory_policy.cpp:318-323)
__global__ __launch_bounds__(256) void k_update(int J, int N, const double* MT, const double* u, double* theta)
{
    __shared__ double us[256];
    const int d = blockIdx.x, i = threadIdx.x;
    if (i < N) us[i] = u[(size_t)d * N + i];
    __syncthreads();
    if (i >= N) return;
    double s = 0.0;
    for (int k = 0; k < N; ++k) s += MT[(size_t)k * N + i] * us[k];
    theta[(size_t)d * N + i] += 1.0 * s;
}

void launch_update(int J, int N, const double* MT, const double* u, double* theta, hipStream_t s)
{
    hipLaunchKernelGGL(k_update, dim3(J), dim3(256), 0, s, J, N, MT, u, theta);
}

// ============================================================== rollout reuse
// PolicyImprovement::generateRollouts reuse branch (policy_improvement.cpp:176-225): rank the
// K previous rollouts and the extra (noiseless) rollout by Rollout::getCost (:149-156),
// lexicographic on (cost, index) with the extra rollout at index -1 (std::sort of pairs), copy
// the best K_r into rows K_gen.. and re-base their noise on the current theta.
__global__ __launch_bounds__(256) void k_reuse(int K, int J, int N, int Kr, int K_gen, int with_extra, double* params,
                                               double* noise, double* state, const double* control,
                                               const double* x_params, const double* x_state,
                                               const double* x_control, const double* theta, double* tmp_params,
                                               double* tmp_state)
{
    extern __shared__ __attribute__((aligned(16))) double sh[];
    const int n = K + with_extra;
    double* costs = sh;
    int* sel = (int*)(sh + n);
    const int tid = threadIdx.x, bs = blockDim.x;
    const size_t JN = (size_t)J * N;
    for (int c = tid; c < n; c += bs) {
        const double* st = c < K ? state + (size_t)c * N : x_state;
        const double* ct = c < K ? control + (size_t)c * JN : x_control;
        double s = st[0];
        for (int t = 1; t < N; ++t) s += st[t];
        for (int d = 0; d < J; ++d) {
            double x = ct[(size_t)d * N];
            for (int t = 1; t < N; ++t) x += ct[(size_t)d * N + t];
            s += x;
        }
        costs[c] = s;
    }
    __syncthreads();
    for (int c = tid; c < n; c += bs) {
        const int ic = c < K ? c : -1;
        const double cc = costs[c];
        int rank = 0;
        for (int c2 = 0; c2 < n; ++c2) {
            const int ic2 = c2 < K ? c2 : -1;
            const double x = costs[c2];
            if (x < cc || (x == cc && ic2 < ic)) ++rank;
        }
        if (rank < Kr) sel[rank] = c;
    }
    __syncthreads();
    for (size_t idx = tid; idx < (size_t)Kr * JN; idx += bs) {
        const int r = (int)(idx / JN);
        const size_t off = idx % JN;
        const int src = sel[r];
        tmp_params[idx] = src < K ? params[(size_t)src * JN + off] : x_params[off];
    }
    for (size_t idx = tid; idx < (size_t)Kr * N; idx += bs) {
        const int r = (int)(idx / N);
        const int t = (int)(idx % N);
        const int src = sel[r];
        tmp_state[idx] = src < K ? state[(size_t)src * N + t] : x_state[t];
    }
    __syncthreads();
    for (size_t idx = tid; idx < (size_t)Kr * JN; idx += bs) {
        const int r = (int)(idx / JN);
        const size_t off = idx % JN;
        const size_t dst = (size_t)(K_gen + r) * JN + off;
        const double p = tmp_params[idx];
        params[dst] = p;
        noise[dst] = p - theta[off];
    }
    for (size_t idx = tid; idx < (size_t)Kr * N; idx += bs) {
        const int r = (int)(idx / N);
        const int t = (int)(idx % N);
        state[(size_t)(K_gen + r) * N + t] = tmp_state[idx];
    }
}

void launch_reuse(int K, int J, int N, int Kr, int K_gen, int with_extra, double* params, double* noise,
                  double* state, const double* control, const double* x_params, const double* x_state,
                  const double* x_control, const double* theta, double* tmp_params, double* tmp_state,
                  hipStream_t s)
{
    const size_t lds = (size_t)(K + 1) * sizeof(double) + (size_t)(Kr + 1) * sizeof(int) + 16;
    hipLaunchKernelGGL(k_reuse, dim3(1), dim3(256), lds, s, K, J, N, Kr, K_gen, with_extra, params, noise, state,
                       control, x_params, x_state, x_control, theta, tmp_params, tmp_state);
}

// ============================================================== distance field construction
__global__ void k_sdf_build(int nx, int ny, int nz, int cap2, double res, const int* boxes, int nb,
                            const long long* cyl_d2, const int* cyl_z, int nc, float* out)
{
    const long long total = (long long)nx * ny * nz;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int z = (int)(idx % nz);
        const int y = (int)((idx / nz) % ny);
        const int x = (int)(idx / ((long long)nz * ny));
        long long d2 = cap2;
        for (int b = 0; b < nb; ++b) {
            const int* r = boxes + 6 * b;
            long long dx = max(max(r[0] - x, 0), x - r[1]);
            long long dy = max(max(r[2] - y, 0), y - r[3]);
            long long dz = max(max(r[4] - z, 0), z - r[5]);
            long long v = dx * dx + dy * dy + dz * dz;
            if (v < d2) d2 = v;
        }
        for (int c = 0; c < nc; ++c) {
            const long long dxy = cyl_d2[((size_t)c * nx + x) * ny + y];
            long long dz = max(max(cyl_z[2 * c] - z, 0), z - cyl_z[2 * c + 1]);
            long long v = dxy + dz * dz;
            if (v < d2) d2 = v;
        }
        out[idx] = (float)(sqrt((double)d2) * res);
    }
}

void launch_sdf_build(int nx, int ny, int nz, int cap2, double res, const int* boxes, int nb, const long long* cyl_d2,
                      const int* cyl_z, int nc, float* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_sdf_build, dim3(2048), dim3(256), 0, s, nx, ny, nz, cap2, res, boxes, nb, cyl_d2, cyl_z, nc,
                       out);
}

}  // namespace stomp
