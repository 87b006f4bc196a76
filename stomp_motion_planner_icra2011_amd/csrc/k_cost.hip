// k_cost.hip -- StompOptimizer::execute (stomp_optimizer.cpp:1063-1165) as two launches.
//
// k_fk (one workgroup per rollout, lane t = free waypoint t):
//   handleJointLimits (:562-616) on the LDS copy of the trajectory (block-wide "any
//   violation" vote, then one wave per limited joint: wave argmax with first-index tie
//   break and a Q^-1 column axpy, <= 11 passes); sin/cos of every joint angle; the FK program
//   (treefksolverjointposaxis_partial.cpp:108-140 restated: one running frame plus <= 2
//   saved branch frames in registers) and the frame of every sphere-carrying segment
//   written to `frames` as [rollout][slot][component][t] (a wave's store = 512 contiguous B).
// k_pairs (one workgroup per rollout, one lane per (frame slot, waypoint) over 256 lanes):
//   sphere position (stomp_collision_point.h:138-141), distance-field gather and hinge
//   potential (stomp_optimizer.cpp:659-674, stomp_collision_space.h:193-228); where the
//   potential is non-zero the 7-tap velocity (:683-698; the t-3, t-2, t+3 taps are zero,
//   padding rows come from the iteration-0 FK of start/goal) -> a = pot * |v| (pot == +0
//   gives +0 exactly, as the reference's product does); then lane t folds a over the
//   spheres in list order into cum / state (:1096-1105) and writes the state cost.
// The extra workgroup (index num_noisy) evaluates the noiseless rollout of theta that the
// previous iteration deferred (policy_improvement_loop.cpp:180-182).
#include "device_fk.h"
#include "stamps.h"

namespace stomp {

namespace {
constexpr int kMaxOps = 64;
constexpr int kMaxSeg = 64;
#ifndef KGATHER
#define KGATHER 8
#endif
constexpr int kGather = KGATHER;   // distance-field gathers in flight per lane
constexpr int kPairsBlock = 256;
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_fk(DevModel m, CostArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ FkOp ops_s[kMaxOps];
    __shared__ DevSegment seg_s[kMaxSeg];
    __shared__ double jlim_s[2 * kMaxJoints];
    __shared__ int hl_s[kMaxJoints];
    constexpr int NW = BLOCK / 64;
    const int J = m.J, N = m.N;
    double* traj = lds;                          // J*N
    double* sc = traj + J * N;                   // J*N*2 (sin, cos)

    STAMP(0);
    const int e = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool extra = e == a.num_noisy;
    const double* prm = extra ? a.x_params : a.params + (long long)e * a.stride;
    for (int idx = tid; idx < J * N; idx += BLOCK) traj[idx] = prm[idx];
    for (int idx = tid; idx < m.nops; idx += BLOCK) ops_s[idx] = m.ops[idx];
    for (int idx = tid; idx < m.nseg; idx += BLOCK) seg_s[idx] = m.segs[idx];
    for (int idx = tid; idx < J; idx += BLOCK) {
        hl_s[idx] = m.has_limits[idx];
        jlim_s[2 * idx] = m.jmin[idx];
        jlim_s[2 * idx + 1] = m.jmax[idx];
    }
    __syncthreads();
    STAMP(1);

    // ---- handleJointLimits
    int any = 0;
    for (int idx = tid; idx < J * N; idx += BLOCK) {
        const int j = idx / N;
        if (!hl_s[j]) continue;
        const double v = traj[idx], jmin = jlim_s[2 * j], jmax = jlim_s[2 * j + 1];
        double absamt = 0.0;
        if (v > jmax) absamt = fabs(jmax - v);
        else if (v < jmin) absamt = fabs(jmin - v);
        any |= absamt > 1e-6;
    }
    // Joints are independent, so each wave owns joints wv, wv + NW, ...: the argmax is a
    // wave butterfly (every lane ends with the same (max, first index)) and a pass needs
    // no block barrier.  LDS accesses of one wave execute in program order.
    if (__syncthreads_or(any)) {
        for (int j = wv; j < J; j += NW) {
            if (!hl_s[j]) continue;
            const double jmin = jlim_s[2 * j], jmax = jlim_s[2 * j + 1];
            const double* Q = m.QT + (size_t)j * N * N;
            double* tj = traj + j * N;
            for (int pass = 0; pass < 11; ++pass) {
                double cand = -1.0;
                int ci = 0x7fffffff;
                for (int t = lane; t < N; t += 64) {
                    const double v = tj[t];
                    double absamt = 0.0;
                    if (v > jmax) absamt = fabs(jmax - v);
                    else if (v < jmin) absamt = fabs(jmin - v);
                    if (absamt > 1e-6 && absamt > cand) { cand = absamt; ci = t; }   // t ascending per lane
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const double ov = __shfl_xor(cand, off, 64);
                    const int oi = __shfl_xor(ci, off, 64);
                    if (ov > cand || (ov == cand && oi < ci)) { cand = ov; ci = oi; }
                }
                if (cand < 0.0) break;   // wave-uniform
                const double v = tj[ci];
                const double amount = v > jmax ? jmax - v : jmin - v;
                const double mult = amount / Q[(size_t)ci * N + ci];
                for (int t = lane; t < N; t += 64) tj[t] += mult * Q[(size_t)ci * N + t];
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
    }
    STAMP(2);
    double* tout = extra ? a.x_traj : (a.traj_out ? a.traj_out + (long long)e * J * N : nullptr);
    if (tout)
        for (int idx = tid; idx < J * N; idx += BLOCK) tout[idx] = traj[idx];
    for (int idx = tid; idx < J * N; idx += BLOCK) det_sincos(traj[idx], &sc[2 * idx], &sc[2 * idx + 1]);
    __syncthreads();
    STAMP(3);

    if (tid < N) {
        const int t = tid;
        double* fout = a.frames + (size_t)e * m.nslots * 12 * N;
        Frame C, S0, S1;
        for (int op = 0; op < m.nops; ++op) {
            const FkOp o = ops_s[op];
            if (o.seg < 0) continue;   // emit-only step: same frame as the step before
            const DevSegment& sg = seg_s[o.seg];
            double st = 0.0, ct = 1.0;
            if (sg.q_index >= 0) {
                st = sc[2 * (sg.q_index * N + t)];
                ct = sc[2 * (sg.q_index * N + t) + 1];
            }
            fk_op(sg, o.base, o.save, st, ct, C, S0, S1);
            if (o.slot >= 0) {
                double* f = fout + (size_t)o.slot * 12 * N + t;
#pragma unroll
                for (int k = 0; k < 9; ++k) f[k * N] = C.R[k];
#pragma unroll
                for (int k = 0; k < 3; ++k) f[(9 + k) * N] = C.p[k];
            }
        }
    }
    STAMP(4);
}

__device__ __forceinline__ void load_frame(const double* fr, int N, int tt, double* R, double* P)
{
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = fr[k * N + tt];
#pragma unroll
    for (int k = 0; k < 3; ++k) P[k] = fr[(9 + k) * N + tt];
}

// One lane per (frame slot g, waypoint t): the slot's frame at t is loaded once and serves
// every sphere of that segment; the neighbour frames needed by the velocity stencil are
// loaded only when one of those spheres has a non-zero potential.  All loads are
// unconditional (clamped addresses) so a lane's loads are in flight together.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_pairs(DevModel m, CostArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double lds2[];
    __shared__ int flag;
    __shared__ int slot_sph_s[kMaxSeg + 1];
    const int N = m.N, S = m.S, G = m.nslots;
    const int SC = m.sph_chunk;                         // spheres per LDS chunk
    double* av = lds2;                                  // SC*N: pot, then a = pot*|v|
    double* pad = av + SC * N;                          // [12][S][3] padding-row positions
    DevSphere* sph = (DevSphere*)(pad + 36 * S);        // S
    STAMP(100);
    const int e = blockIdx.x, tid = threadIdx.x;
    const bool extra = e == a.num_noisy;
    const int member = extra ? a.x_member : a.member;
    const double* frames = a.frames + (size_t)e * G * 12 * N;
    for (int idx = tid; idx < S; idx += BLOCK) sph[idx] = m.sph[idx];
    for (int idx = tid; idx < 36 * S; idx += BLOCK) pad[idx] = m.pad_pos[idx];
    for (int idx = tid; idx <= G; idx += BLOCK) slot_sph_s[idx] = m.slot_sph[idx];
    if (tid == 0) flag = 0;
    __syncthreads();

    double cum = 0.0, state = 0.0;
    bool col = false;
    for (int g0 = 0; g0 < G;) {
        // chunk of whole slots whose spheres fit in av (uniform)
        int g1 = g0 + 1;
        while (g1 < G && slot_sph_s[g1 + 1] - slot_sph_s[g0] <= SC) ++g1;
        const int s0 = slot_sph_s[g0];
        const int ns = slot_sph_s[g1] - s0;
        const int items = (g1 - g0) * N;
        for (int it = tid; it < items; it += BLOCK) {
            const int g = g0 + it / N, t = it - (it / N) * N;
            const int sb = slot_sph_s[g], se = slot_sph_s[g + 1];
            const double* fr = frames + (size_t)g * 12 * N;
            constexpr int NT = kVelTap1 - kVelTap0 + 1, TC = 3 - kVelTap0;   // TC: centre tap
            double v[NT][12];
            load_frame(fr, N, t, v[TC], v[TC] + 9);
            bool any = false;
            for (int q0 = sb; q0 < se; q0 += kGather) {
                float dv[kGather];
#pragma unroll
                for (int k = 0; k < kGather; ++k) {
                    const int s = min(q0 + k, se - 1);
                    double x[3];
                    apply(v[TC], v[TC] + 9, sph[s].pos, x);
#ifdef PAIRS_NOGATHER
                    dv[k] = (float)(x[0] + x[1]);
#else
                    dv[k] = sdf_distance(m, x);
#endif
                }
#pragma unroll
                for (int k = 0; k < kGather; ++k) {
                    const int s = q0 + k;
                    if (s >= se) continue;
                    const double dd = (double)dv[k];
                    col |= dd <= sph[s].radius;
                    const double pot = potential(sph[s], dd);
                    any |= pot != 0.0;
                    av[(s - s0) * N + t] = pot;   // a = pot * |v| is +0 exactly when pot == +0
                }
            }
#ifdef PAIRS_NOVEL
            any = false;
#endif
            if (any) {
                // frames at the other velocity taps t-1, t+1, t+2 (kVelTap0..kVelTap1; the
                // remaining taps are zero, checked on the host), clamped rows
#pragma unroll
                for (int q = 0; q < NT; ++q) {
                    if (q == TC) continue;
                    const int tt = min(max(t + q - TC, 0), N - 1);
                    load_frame(fr, N, tt, v[q], v[q] + 9);
                }
                for (int s = sb; s < se; ++s) {
                    const double pot = av[(s - s0) * N + t];
                    if (pot == 0.0) continue;
                    double v0 = 0.0, v1 = 0.0, v2 = 0.0;
#pragma unroll
                    for (int q = 0; q < NT; ++q) {
                        const double c = m.vel_coef[kVelTap0 + q];
                        if (c == 0.0) continue;   // 0 * p adds a signed zero: |v| unchanged
                        const int tt = t + q - TC;
                        double y[3];
                        if (tt >= 0 && tt < N) {
                            apply(v[q], v[q] + 9, sph[s].pos, y);
                        } else {
                            const int row = tt < 0 ? tt + 6 : tt - N + 6;   // padding row 0..11
                            const double* src = pad + (row * S + s) * 3;
                            y[0] = src[0]; y[1] = src[1]; y[2] = src[2];
                        }
                        v0 += c * y[0];
                        v1 += c * y[1];
                        v2 += c * y[2];
                    }
                    av[(s - s0) * N + t] = pot * sqrt(v0 * v0 + v1 * v1 + v2 * v2);
                }
            }
        }
        __syncthreads();
        STAMP(102);
        if (tid < N)
            for (int q = 0; q < ns; ++q) {
                cum += av[q * N + tid];
                state += cum;
            }
        __syncthreads();
        g0 = g1;
    }
    STAMP(103);
    if (col) flag = 1;   // every writer stores 1
    if (tid < N) {
        const double cost = m.w_obs * state + m.w_con * 0.0 + m.w_tq * 0.0;   // :1148-1151
        double* so = extra ? a.x_state : a.state_out + (long long)e * N;
        so[tid] = cost;
        av[tid] = cost;
    }
    __syncthreads();
    if (tid == 0) {
        const bool cf = !flag && !(member == 0 && m.pad_collision);
        uint8_t* cfo = extra ? a.x_cf : (a.cf_out ? a.cf_out + e : nullptr);
        double* to = extra ? a.x_total : (a.total_out ? a.total_out + e : nullptr);
        if (cfo) *cfo = cf ? 1 : 0;
        if (to) {
            double s = av[0];
            for (int k = 1; k < N; ++k) s += av[k];   // costs.sum() (:1155)
            *to = s;
        }
    }
    STAMP(104);
}

STOMP_STAMP_ACCESSORS(cost)

bool cost_supported(const DevModel& m) { return m.nops <= kMaxOps && m.nseg <= kMaxSeg && m.J <= kMaxJoints; }

size_t pairs_lds_bytes(int chunk, int S, int N)
{
    return (size_t)chunk * N * sizeof(double) + (size_t)S * (36 * sizeof(double) + sizeof(DevSphere));
}

int pairs_sphere_chunk(int S, int N)
{
    // one double per (sphere, waypoint); chunk + sphere tables within 64 KB of LDS
    int sc = (int)((64 * 1024 - pairs_lds_bytes(0, S, N)) / (8 * (size_t)N));
    if (sc > S) sc = S;
    return sc < 1 ? 1 : sc;
}

void launch_cost(const DevModel& m, const CostArgs& a, hipStream_t s)
{
    const int blocks = a.num_noisy + (a.x_params ? 1 : 0);
    if (blocks <= 0) return;
    const size_t lds1 = (size_t)m.J * m.N * 3 * sizeof(double);
    // 256 lanes: four waves share the limited joints in handleJointLimits; the FK program
    // runs on lanes t < N (N <= 256)
    hipLaunchKernelGGL((k_fk<256>), dim3(blocks), dim3(256), lds1, s, m, a);
    const size_t lds2 = pairs_lds_bytes(m.sph_chunk, m.S, m.N);
    hipLaunchKernelGGL((k_pairs<kPairsBlock>), dim3(blocks), dim3(kPairsBlock), lds2, s, m, a);
}

}  // namespace stomp
