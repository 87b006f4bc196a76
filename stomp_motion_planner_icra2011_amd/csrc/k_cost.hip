// k_cost.hip -- StompOptimizer::execute (stomp_optimizer.cpp:1063-1165), one workgroup per rollout.
//
// k_rollout<256>, everything in LDS, nothing but the inputs and the state costs touches HBM:
//   1. handleJointLimits (:562-616) on the LDS copy of the trajectory: block-wide "any
//      violation" vote, then one wave per limited joint (wave argmax with first-index tie
//      break, Q^-1 column axpy, <= 11 passes).
//   2. The FK program (treefksolverjointposaxis_partial.cpp:108-140 restated: one running
//      frame in the registers of lanes t < N, <= 2 saved branch frames in LDS) walks the
//      segments in DFS order.  Each sphere-carrying segment ("slot") is published to an LDS
//      frame buffer [12][N]; then lane (t, g) reads the frame at t once and takes spheres
//      g, g + G, ... of the slot (G = 256 / N groups): sphere position
//      (stomp_collision_point.h:138-141), distance-field gathers of the voxel's squared cell
//      distance d2 (branch-free, all in flight per lane); the hinge potential is zero and the
//      collision flag set by per-sphere thresholds on d2 (stomp_optimizer.cpp:659-674,
//      stomp_collision_space.h:193-228); where the potential is non-zero, the distance
//      sqrt(d2) res, the potential, the 7-tap velocity (:683-698) from the neighbouring frames
//      in LDS (padding rows: iteration-0 FK of start/goal) and a = pot * |v|; then lanes t
//      fold a over the slot's spheres,
//      in list order, into cum / state (:1096-1105).  Slots are numbered in sphere order,
//      so slot-by-slot folding is the reference's order.
//   3. costs(t) = w_obs * state (:1148-1151), the collision flag and the total (:1155).
// The extra workgroup (index num_noisy) evaluates the noiseless rollout of theta that the
// previous iteration deferred (policy_improvement_loop.cpp:180-182).
#include <algorithm>
#include <cassert>
#include <cstdlib>

#include "device_fk.h"
#include "limits_device.h"
#include "noise_device.h"
#include "stamps.h"

namespace stomp {

namespace {
constexpr int kMaxOps = 64;
constexpr int kMaxSeg = 64;
#ifndef ROLLOUT_BLOCK
#define ROLLOUT_BLOCK 256
#endif
constexpr int kBlock = ROLLOUT_BLOCK;
#ifndef ROLLOUT_MIN_WAVES
#define ROLLOUT_MIN_WAVES (ROLLOUT_BLOCK > 256 ? 4 : 3)
#endif
// the wide rollout workgroup: when a launch's rollouts fit one per CU (the K-sharded ranks,
// the deferred noiseless rollout, small K) no CU runs two of them, so a rollout gets 512
// lanes (twice the pair lanes per slot round, half the gather rounds per lane) and the
// register budget of two waves per SIMD
#ifndef ROLLOUT_WIDE_BLOCK
#define ROLLOUT_WIDE_BLOCK 512
#endif
constexpr int kWideBlock = ROLLOUT_WIDE_BLOCK;
// the waypoint-split rollout: workgroup size, most pieces per rollout
#ifndef ROLLOUT_SPLIT_BLOCK
#define ROLLOUT_SPLIT_BLOCK 512
#endif
constexpr int kSplitBlock = ROLLOUT_SPLIT_BLOCK;
// pieces per rollout at most: cfg1 (11 rollouts) 25.6k it/s at 4, 26.4-26.9k at 5-7 (6: 26.7k, 25.1k
// in the driver's window against 24.6k; profiles/ab/r5_split_pieces.txt)
constexpr int kSplitMaxDefault = 6;
template <int BLOCK>
constexpr int rollout_min_waves()
{
    return BLOCK == kBlock ? ROLLOUT_MIN_WAVES : (BLOCK > 512 ? 4 : 2);
}
// spheres of one run a pair lane takes: run_max(N) / (BLOCK / N) <= 16 / 2 (N <= 128) or 8 / 1
constexpr int kLaneSpheres = 8;
static_assert(kRunMaxSmall / 2 <= kLaneSpheres && kRunMaxLarge <= kLaneSpheres && kBlock >= 256,
              "a pair lane's spheres of one run must fit kLaneSpheres");
}

// The lean layout's tables in HBM, typed in the constant address space: the kernel never writes
// them, so a load through them with a wave-uniform index is a scalar load, which waits on the
// scalar counter, not behind the vector memory counter of the gathers in flight.  The loaders copy
// a record member by member into registers.
using CSegment = const __attribute__((address_space(4))) DevSegment;
using COp = const __attribute__((address_space(4))) FkOp;
using CSphere = const __attribute__((address_space(4))) DevSphere;
using CInt = const __attribute__((address_space(4))) int;
using CDouble = const __attribute__((address_space(4))) double;
__device__ __forceinline__ DevSegment load_seg(CSegment* p)
{
    DevSegment r;
    r.parent = p->parent;
    r.q_index = p->q_index;
    r.rot_identity = p->rot_identity;
    r.pad_ = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) r.rot[k] = p->rot[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        r.trans[k] = p->trans[k];
        r.axis[k] = p->axis[k];
    }
    return r;
}
__device__ __forceinline__ FkOp load_op(COp* p)
{
    FkOp r;
    r.seg = p->seg;
    r.base = p->base;
    r.save = p->save;
    r.sph_begin = p->sph_begin;
    r.sph_end = p->sph_end;
    r.slot = p->slot;
    return r;
}
__device__ __forceinline__ DevSphere load_sph(CSphere* p)
{
    DevSphere r;
    r.slot = p->slot;
    r.zero_lim = p->zero_lim;
    r.col_lim = p->col_lim;
    r.pad_ = 0;
    r.radius = p->radius;
    r.clearance = p->clearance;
    r.inv_clearance = p->inv_clearance;
#pragma unroll
    for (int k = 0; k < 3; ++k) r.pos[k] = p->pos[k];
    return r;
}
// a pointer into HBM marked global (no flat instructions, which would wait on the LDS counter too)
__device__ __forceinline__ double* global_ptr(double* p)
{
    return (double*)(__attribute__((address_space(1))) double*)p;
}

__device__ __forceinline__ void apply_lds(const double* fb, int N, int t, const double* pos, double* x)
{
#pragma unroll
    for (int i = 0; i < 3; ++i)
        x[i] = fb[(3 * i + 0) * N + t] * pos[0] + fb[(3 * i + 1) * N + t] * pos[1] +
               fb[(3 * i + 2) * N + t] * pos[2] + fb[(9 + i) * N + t];
}

// The ordered fold of one waypoint's a values a[q * stride], q ascending over n: cum += a_q,
// state += cum (stomp_optimizer.cpp:1099-1104), in the same order as a plain loop.  Whole batches
// of 16 run unrolled.  The rest (n mod 16 terms) is loaded reversed (w[j] = a[rest - 1 - j]) and
// entered by a switch on its length, so every register index is static: with an early exit
// inside an unrolled loop the compiler indexed the batch's registers at run time
// (s_set_gpr_idx_on / off around every term).
__device__ __forceinline__ void fold_avalues(const double* av, int stride, int n, double& cum, double& state)
{
    int q0 = 0;
    for (; q0 + 16 <= n; q0 += 16) {
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = av[(q0 + q) * stride];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            cum += v[q];
            state += cum;
        }
    }
    const int rest = n - q0;
    if (rest <= 0) return;
    double w[15];
#pragma unroll
    for (int j = 0; j < 15; ++j) w[j] = av[(q0 + max(rest - 1 - j, 0)) * stride];
#define STOMP_FOLD_STEP(j) \
    cum += w[j];           \
    state += cum;
    switch (rest) {
    case 15: STOMP_FOLD_STEP(14) [[fallthrough]];
    case 14: STOMP_FOLD_STEP(13) [[fallthrough]];
    case 13: STOMP_FOLD_STEP(12) [[fallthrough]];
    case 12: STOMP_FOLD_STEP(11) [[fallthrough]];
    case 11: STOMP_FOLD_STEP(10) [[fallthrough]];
    case 10: STOMP_FOLD_STEP(9) [[fallthrough]];
    case 9: STOMP_FOLD_STEP(8) [[fallthrough]];
    case 8: STOMP_FOLD_STEP(7) [[fallthrough]];
    case 7: STOMP_FOLD_STEP(6) [[fallthrough]];
    case 6: STOMP_FOLD_STEP(5) [[fallthrough]];
    case 5: STOMP_FOLD_STEP(4) [[fallthrough]];
    case 4: STOMP_FOLD_STEP(3) [[fallthrough]];
    case 3: STOMP_FOLD_STEP(2) [[fallthrough]];
    case 2: STOMP_FOLD_STEP(1) [[fallthrough]];
    case 1: STOMP_FOLD_STEP(0) break;
    default: break;
    }
#undef STOMP_FOLD_STEP
}

// |v| of sphere s at free waypoint t: the 7-tap velocity of its position (stomp_optimizer.cpp:683-698)
// from the slot's frames in LDS, padding rows from the iteration-0 FK of start / goal
__device__ __forceinline__ double sphere_speed(const DevModel& m, const double* fb, const double* pad,
                                               const DevSphere& sp, int s, int t)
{
    const int N = m.N;
    // every tap's free-row position and padding-row position are fetched unconditionally
    // (clamped indices, all reads in flight together) and the right one selected per tap
    double y[7][3];
#pragma unroll
    for (int kk = kVelTap0; kk <= kVelTap1; ++kk) {
        const int tt = t + kk - 3;
        double yf[3];
        apply_lds(fb, N, min(max(tt, 0), N - 1), sp.pos, yf);
        const int row = tt < 0 ? tt + 6 : (tt >= N ? tt - N + 6 : 0);   // padding row 0..11
        const double* src = pad + (row * m.S + s) * 3;
        const bool in = tt >= 0 && tt < N;
#pragma unroll
        for (int c = 0; c < 3; ++c) y[kk][c] = in ? yf[c] : src[c];
    }
    double v0 = 0.0, v1 = 0.0, v2 = 0.0;
#pragma unroll
    for (int kk = kVelTap0; kk <= kVelTap1; ++kk) {
        const double c = m.vel_coef[kk];
        if (c == 0.0) continue;   // 0 * p adds a signed zero: |v| unchanged
        v0 += c * y[kk][0];
        v1 += c * y[kk][1];
        v2 += c * y[kk][2];
    }
    return sqrt(v0 * v0 + v1 * v1 + v2 * v2);
}

// handleJointLimits (stomp_optimizer.cpp:562-616) of the row in traj [J][N] (LDS) by the NW waves
// of a workgroup; the caller publishes traj before and synchronises after.
// Joints are independent: the limited joints are dealt round-robin over the waves and a wave
// runs the passes of two of its joints in lockstep (pass p of one beside pass p of the other,
// each joint still stopping on its own), so the two Q^-1 column loads of a step are in flight
// together.  The argmax is a wave butterfly (every lane ends with the same (max, first
// index)) and a pass needs no block barrier: LDS accesses of one wave execute in program order.
// A joint without violations costs its wave one argmax.
template <int NW, typename IntTable, typename DoubleTable>
__device__ __forceinline__ void joint_limit_passes(const DevModel& m, double* traj, IntTable hl_s,
                                                   DoubleTable jlim_s, int lane, int wv)
{
    const int J = m.J, N = m.N;
    // A wave keeps its joints' rows in registers through the passes (lane l: waypoints l,
    // l + 64, ...; N <= 256), so a pass is the argmax, the column load and the update with
    // no LDS round trip; the rows go back to traj after the last pass.
    // the violated waypoint a pass corrects (wave-uniform, -1 when none is left) and the
    // correction (limits_device.h)
    auto jl_argmax = [&](const double* v, double jmin, double jmax) -> int {
        return stomp::jl_argmax(v, N, lane, jmin, jmax);
    };
    auto jl_apply = [&](double* v, int cm, double jmin, double jmax, const double* qv, double qd) {
        stomp::jl_apply(v, N, lane, cm, jmin, jmax, qv, qd);
    };
    auto jl_pair = [&](int ja, int jb) {
        const bool hb = jb >= 0;
        const int jb0 = hb ? jb : ja;
        const double amin = jlim_s[2 * ja], amax = jlim_s[2 * ja + 1];
        const double bmin = jlim_s[2 * jb0], bmax = jlim_s[2 * jb0 + 1];
        double va[4], vb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = min(lane + 64 * u, N - 1);
            va[u] = traj[ja * N + t];
            vb[u] = traj[jb0 * N + t];
        }
        bool la = true, lb = hb;
        for (int pass = 0; pass < 11 && (la || lb); ++pass) {
            int ca = -1, cb = -1;
            if (la) { ca = jl_argmax(va, amin, amax); la = ca >= 0; }
            if (lb) { cb = jl_argmax(vb, bmin, bmax); lb = cb >= 0; }
            if (!la && !lb) break;
            // both columns and diagonals in flight (unconditional loads, clamped; N <= 256)
            const double* Qa = m.QT + ((size_t)ja * N + (size_t)max(ca, 0)) * N;
            const double* Qb = m.QT + ((size_t)jb0 * N + (size_t)max(cb, 0)) * N;
            double qa[4], qb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                qa[u] = Qa[min(lane + 64 * u, N - 1)];
                qb[u] = Qb[min(lane + 64 * u, N - 1)];
            }
            const double qda = Qa[max(ca, 0)], qdb = Qb[max(cb, 0)];
            if (la) jl_apply(va, ca, amin, amax, qa, qda);
            if (lb) jl_apply(vb, cb, bmin, bmax, qb, qdb);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = lane + 64 * u;
            if (t < N) {
                traj[ja * N + t] = va[u];
                if (hb) traj[jb * N + t] = vb[u];
            }
        }
    };
    int mine = -1, k = 0;
    for (int j = 0; j < J; ++j) {
        if (!hl_s[j]) continue;
        if (k++ % NW != wv) continue;
        if (mine < 0) {
            mine = j;
        } else {
            jl_pair(mine, j);
            mine = -1;
        }
    }
    if (mine >= 0) jl_pair(mine, -1);
}

// a rollout launch's block past its rollouts: pregen row r of the next iteration (normals,
// sigma L z, M eps), left at the default wave priority while the rollout waves raise theirs, so
// it takes the issue slots the latency-bound rollout waves leave idle and the CUs the
// early-finishing rollouts free; no stop check (the rows stay valid for pre_it).  First, unless
// its rollout prices it (own), this iteration's row r (ctl_by_pre).  pA / pB: LDS buffers of the
// noise phase
template <int BLOCK>
__device__ __forceinline__ void pregen_block(const CostArgs& a, int r, bool own, double* pA, double* pB)
{
    const NoiseArgs& pa = a.pre_next;
    if (a.ctl_by_pre && r < a.ctl_rows && !own && !(a.stop && *a.stop)) {
        // this iteration's row r priced here instead of on its rollout's critical path
        pre_row_control<BLOCK>(a.nz, r, pA, pB, threadIdx.x);
        __syncthreads();   // pA / pB are the normals' buffers next
    }
    rollout_normals<BLOCK>(pa, r, pA, pB, threadIdx.x);
    if (pa.J <= 8) {
        pregen_eps_ng<BLOCK, 2>(pa, r, pA, pB, threadIdx.x);
        pregen_meps_ng<BLOCK, 2>(pa, r, pB, threadIdx.x);
    } else {
        pregen_eps_ng<BLOCK, 4>(pa, r, pA, pB, threadIdx.x);
        pregen_meps_ng<BLOCK, 4>(pa, r, pB, threadIdx.x);
    }
}

// a rollout launch's block past its pregen blocks: the total of reuse candidate c (the previous
// iteration's row c, candidate_total) for launch_reuse_rows; stage: (J + 1) N doubles of LDS
template <int BLOCK>
__device__ __forceinline__ void totals_block(const CostArgs& a, int J, int N, int c, double* stage)
{
    if (a.stop && *a.stop) return;
    const double t = candidate_total<BLOCK>(a.tot_state + (size_t)c * N, a.tot_control + (size_t)c * J * N, J, N,
                                            stage, threadIdx.x);
    if (threadIdx.x == 0) a.tot_out[c] = t;
}

// a split rollout launch's block past its totals blocks: reuse candidate c priced ahead of the
// ranking (price_candidate into the spec rows; c = spec_rows - 1 is the extra rollout, params
// theta); lds: the workgroup's whole dynamic LDS (at least price_candidate_lds_bytes).  Only the
// split kernel carries these blocks (rollout_split_pieces): inlined into the slot-loop kernels the
// pricing code pushed them into scratch.
template <int BLOCK>
__device__ __forceinline__ void spec_block(const CostArgs& a, int c, double* lds)
{
    if (a.stop && *a.stop) return;
    const size_t JN = (size_t)a.nz.J * a.nz.N;
    const double* psrc = c < a.spec_rows - 1 ? a.spec_src + c * JN : nullptr;
    if (a.nz.J <= 2 * kNoiseJT)
        price_candidate<BLOCK, 2>(a.nz, psrc, a.spec_params + c * JN, a.spec_noise + c * JN, a.spec_ctl + c * JN, lds,
                                  threadIdx.x);
    else
        price_candidate<BLOCK, 4>(a.nz, psrc, a.spec_params + c * JN, a.spec_noise + c * JN, a.spec_ctl + c * JN, lds,
                                  threadIdx.x);
}

// a split launch's last block (CostArgs::x_ctl_block): the extra rollout's rows of addExtraRollouts
// (theta copied, noise 0, the control costs of theta + 0), which its first piece made ahead of its
// row before; zA / zB: the block's LDS
template <int BLOCK>
__device__ __forceinline__ void x_ctl_rows_block(const CostArgs& a, int Nall, double* zA, double* zB)
{
    if (a.stop && *a.stop) return;
    const int J = a.nz.J, N = a.nz.N, tid = threadIdx.x;
    for (int idx0 = 0; idx0 < J * N; idx0 += 4 * BLOCK) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = a.x_params[min(idx0 + tid + u * BLOCK, J * N - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = idx0 + tid + u * BLOCK;
            if (idx < J * N) {
                a.x_prm[idx] = v[u];
                a.x_nse[idx] = 0.0;
                const int d = idx / N, i = idx - d * N;
                zA[d * Nall + i + 6] = v[u] + 0.0;
            }
        }
    }
    rollout_control<BLOCK>(a.nz, 0, zA, zB, tid, a.x_ctl);
}

// the rollout kernel's workgroup `bid` of one engine's launch (k_rollout: bid = blockIdx.x;
// k_rollout_group: the engines of a group share one launch)
// FK_OVERLAP: the slot loop's FK lanes advance the program to the next sphere segment while the
// slot's gathers are in flight (the running frame then stays live across the pair phases); off,
// they advance after the fold from the frame reloaded from fb (fewer live registers; every launch
// now overlaps)
// LEAN (DevModel::lean, slot loop only): the saved branch-point frames in HBM (the workgroup's
// block of sv_glob), no (sin, cos) pre-pass, the FK / joint-limit tables (and with LEAN 2 the sphere
// table) read from the image in HBM through the constant address space, so their wave-uniform
// loads are scalar loads that do not wait behind the vector memory counter of the gathers in flight
template <int BLOCK, bool BRICK, bool PHASED = false, bool FK_OVERLAP = true, int LEAN = 0>
__device__ __forceinline__ void rollout_body(const DevModel& m, const CostArgs& a, const int bid)
{
    static_assert(!LEAN || (!PHASED && FK_OVERLAP), "the lean layout is the slot loop's");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    __shared__ int flag;
    __shared__ int nz_count;
    const int J = m.J, N = m.N, S = m.S;
    const RolloutLds L = rollout_lds(J, N, S, m.sph_chunk, m.nsaves, m.nseg, m.nops, m.nslots, LEAN ? 0 : m.pad_lds,
                                     PHASED, LEAN);
    {
        // blocks past the rollouts: the next iteration's pregen rows (normals, sigma L z,
        // M eps), left at the default wave priority while the rollout waves raise theirs, so
        // they take the issue slots the latency-bound rollout waves leave idle and the CUs
        // the early-finishing rollouts free; no stop check (the rows stay valid for pre_it)
        const int nro = a.num_noisy + (a.x_params ? 1 : 0);
        if (bid >= nro) {
            const int r = bid - nro;
            if (r >= a.pre_rows) {   // the reuse candidates' totals (nzA, nzB: contiguous)
                totals_block<BLOCK>(a, J, N, r - a.pre_rows, (double*)(lds_raw + L.nzA));
                return;
            }
            // a phased launch's rollouts price their own rows (the FK-idle waves)
            const bool own = PHASED && r >= a.row0 && r < a.row0 + a.num_noisy;
            pregen_block<BLOCK>(a, r, own, (double*)(lds_raw + L.nzA), (double*)(lds_raw + L.nzB));
            return;
        }
    }
    if (a.pre_rows > 0 || a.tot_rows > 0) __builtin_amdgcn_s_setprio(2);
    if (a.stop && *a.stop) return;
    double* traj = (double*)(lds_raw + L.traj);   // J*N
    double* fb = (double*)(lds_raw + L.fb);       // 12*N frame of the current slot
    // nsaves*12*N saved branch-point frames (LEAN: this workgroup's block of sv_glob in HBM)
    double* sv = LEAN ? global_ptr(m.sv_glob) + (size_t)bid * m.nsaves * 12 * N : (double*)(lds_raw + L.sv);
    double* av = (double*)(lds_raw + L.av);       // max_slot*N: pot, then pot * |v|
    unsigned short* nzl = (unsigned short*)(lds_raw + L.nzl);   // pairs q*N+t with a non-zero potential
    // the tables: LDS copies of the image, or (LEAN) the image in HBM (offsets relative to .sph)
    const unsigned char* gimg = (const unsigned char*)m.img;
    const DevSphere* sph = (const DevSphere*)(lds_raw + L.sph);   // not with LEAN 2
    const DevSegment* seg_s = (const DevSegment*)(lds_raw + L.seg);   // not with LEAN
    const FkOp* ops_s = (const FkOp*)(lds_raw + L.ops);
    const int* hl_s = (const int*)(lds_raw + L.hl);
    const double* jlim_s = (const double*)(lds_raw + L.jlim);
    CSphere* csph = (CSphere*)gimg;
    CSegment* cseg = (CSegment*)(gimg + (L.seg - L.sph));
    COp* cops = (COp*)(gimg + (L.ops - L.sph));
    CInt* chl = (CInt*)(gimg + (L.hl - L.sph));
    CDouble* cjlim = (CDouble*)(gimg + (L.jlim - L.sph));
    // the FK program's op i
    auto op_at = [&](int i) -> FkOp {
        if constexpr (LEAN != 0) return load_op(cops + i);
        else return ops_s[i];
    };
    // [12][S][3] padding-row sphere positions: LDS copy when it fits, else HBM
    const double* pad = !LEAN && m.pad_lds ? (const double*)(lds_raw + L.pad) : m.pad_pos;
    // every (sin, cos) made ahead of the FK program (the cosines in the saved-frame area)
    const bool sincos_pre = !LEAN && m.sincos_pre;

    STAMP(0);
    BLOCK_BEGIN();
    const int e = bid, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int NW = BLOCK / 64;
    const bool extra = e == a.num_noisy;
    const int member = extra ? a.x_member : a.member;
    // the table image: every lane's loads go out together and land while the normals are
    // drawn (or the trajectory is loaded); they are stored to LDS after that
    double* zA = (double*)(lds_raw + L.nzA);
    double* zB = (double*)(lds_raw + L.nzB);
    const bool gen = a.fused_noise == 1 && !extra;
    const bool pre = a.fused_noise == 2 && !extra;
    constexpr int kCopyBatch = 12 * 256 / BLOCK;   // table-image words per lane per copy pass
    unsigned long long img[kCopyBatch];
    // LEAN 1 copies the sphere table only, LEAN 2 nothing
    const int nw = LEAN == 0 ? m.img_words : LEAN == 1 ? (int)(S * sizeof(DevSphere) / 8) : 0;
    if constexpr (LEAN != 2) {
#pragma unroll
        for (int u = 0; u < kCopyBatch; ++u) img[u] = m.img[min(tid + u * BLOCK, nw - 1)];
    }
    // the pregen row's first chunk goes out with the image loads (one memory latency for both)
    PreChunk pc0;
    // a row priced by its pregen block (ctl_by_pre) needs no M eps here
    const bool priced = !PHASED && a.ctl_by_pre;
    const int pr = e + a.row0;   // the row in the pregen buffers
    if (pre) {
        if (priced) pre_chunk_load<BLOCK, false>(a.nz, pr, 0, tid, pc0);
        else pre_chunk_load<BLOCK>(a.nz, pr, 0, tid, pc0);
    }
    if (gen) {
        rollout_normals<BLOCK>(a.nz, e, zA, zB, tid);
    } else if (!pre) {
        const double* prm = extra ? a.x_params : a.params + (long long)e * a.stride;
        const bool xc = extra && a.x_ctl;   // the extra rollout's rows too (addExtraRollouts)
        for (int idx0 = 0; idx0 < J * N; idx0 += 4 * BLOCK) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = prm[min(idx0 + tid + u * BLOCK, J * N - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int idx = idx0 + tid + u * BLOCK;
                if (idx < J * N) {
                    traj[idx] = v[u];
                    if (xc) {
                        // k_noise's zero-noise row: noise +0.0, x = params + (M 0 = +0.0)
                        a.x_prm[idx] = v[u];
                        a.x_nse[idx] = 0.0;
                        const int d = idx / N, i = idx - d * N;
                        zA[d * m.Nall + i + 6] = v[u] + 0.0;
                    }
                }
            }
        }
        if (xc) rollout_control<BLOCK>(a.nz, 0, zA, zB, tid, a.x_ctl);
    }
    if constexpr (LEAN != 2) {
        unsigned long long* dst = (unsigned long long*)(lds_raw + L.sph);
#pragma unroll
        for (int u = 0; u < kCopyBatch; ++u)
            if (tid + u * BLOCK < nw) dst[tid + u * BLOCK] = img[u];
        for (int w = tid + kCopyBatch * BLOCK; w < nw; w += BLOCK) dst[w] = m.img[w];
    }
    STAMP(6);
    // phased with x in the a-value buffers: the control costs are made during the FK program
    const bool defer = PHASED && L.nzA == L.av && (gen || pre);
    if (gen) {
        if (defer) rollout_project<BLOCK, true>(a.nz, e, traj, zA, zB, tid);
        else rollout_project<BLOCK>(a.nz, e, traj, zA, zB, tid);
    } else if (pre) {
        // the control costs are left to the pregen block of this row (ctl_by_pre) or, in the
        // phased body, to the FK-idle waves (defer)
        if (priced) rollout_from_pre<BLOCK, true, false>(a.nz, pr, e == 0, traj, zA, zB, tid, pc0);
        else if (defer) rollout_from_pre<BLOCK, true>(a.nz, pr, e == 0, traj, zA, zB, tid, pc0);
        else rollout_from_pre<BLOCK>(a.nz, pr, e == 0, traj, zA, zB, tid, pc0);
    }
    if (tid == 0) flag = 0;
    __syncthreads();
    STAMP(1);
    BLOCK_MARK(4);

    // ---- handleJointLimits (no block-wide pre-scan: the barrier above already published traj)
    {
        __builtin_amdgcn_s_setprio(3);   // a dependent chain per joint (critical path)
        if constexpr (LEAN != 0) joint_limit_passes<NW>(m, traj, chl, cjlim, lane, wv);
        else joint_limit_passes<NW>(m, traj, hl_s, jlim_s, lane, wv);
        __builtin_amdgcn_s_setprio(2);
        __syncthreads();
    }
    STAMP(2);
    BLOCK_MARK(5);
    double* tout = extra ? a.x_traj : (a.traj_out ? a.traj_out + (long long)e * J * N : nullptr);
    if (tout)
        for (int idx = tid; idx < J * N; idx += BLOCK) tout[idx] = traj[idx];
    __syncthreads();
    STAMP(3);

    // ---- FK program, slot by slot, with the slot's pairs in between
    // FK / fold lane: waypoint t_own (< N).  Odd workgroups run the FK program on waves 2-3
    // (N <= 128): two workgroups share a CU, and their waves 0-1 would otherwise share SIMDs
    // while the FK-idle waves leave the other two SIMDs empty
    const int t_own = tid - ((N <= 128 && (e & 1)) ? 128 : 0);
    const bool fk_lane = t_own >= 0 && t_own < N;
    const int G = BLOCK / N, pg = tid / N, pt = tid - pg * N;   // pair lanes: (group, waypoint)
    // C: running frame in the registers of lanes t < N; branch-point frames saved in LDS
    // (column t of sv).  Lanes t < N are also pair lanes (0, t).
    Frame C;
    double cum = 0.0, state = 0.0;
    bool col = false;
    // one FK program step (stomp_optimizer.cpp via treefksolverjointposaxis_partial.cpp:108-140)
    auto fk_step = [&](const FkOp& o, const DevSegment& sg) {
        double st = 0.0, ct = 1.0;
        if (sg.q_index >= 0) {
            if (sincos_pre) {
                st = traj[sg.q_index * N + t_own];
                ct = sv[sg.q_index * N + t_own];
            } else {
                det_sincos(traj[sg.q_index * N + t_own], &st, &ct);
            }
        }
        Frame nf;
        if (o.base == kBaseChain) {
            compose(sg, &C, st, ct, nf);
        } else if (o.base == kBaseRoot) {
            compose(sg, nullptr, st, ct, nf);
        } else {
            Frame pf;
            const double* src = sv + (size_t)o.base * 12 * N + t_own;
#pragma unroll
            for (int k = 0; k < 9; ++k) pf.R[k] = src[k * N];
#pragma unroll
            for (int k = 0; k < 3; ++k) pf.p[k] = src[(9 + k) * N];
            compose(sg, &pf, st, ct, nf);
        }
        C = nf;
        if (o.save >= 0) {
            double* dst = sv + (size_t)o.save * 12 * N + t_own;
#pragma unroll
            for (int k = 0; k < 9; ++k) dst[k * N] = C.R[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) dst[(9 + k) * N] = C.p[k];
        }
    };
    auto fk_op = [&](const FkOp& o) {
        if (o.seg < 0 || !fk_lane) return;
        if constexpr (LEAN != 0) {
            const DevSegment sg = load_seg(cseg + o.seg);
            fk_step(o, sg);
        } else {
            fk_step(o, seg_s[o.seg]);
        }
    };
    // run the program from op up to and including the next sphere-carrying segment; its
    // index (or nops) is uniform
    auto fk_advance = [&](int op) -> int {
        for (; op < m.nops; ++op) {
            const FkOp o = op_at(op);
            fk_op(o);
            if (o.sph_end > o.sph_begin) return op;   // a run of spheres on C
        }
        return m.nops;
    };
    if (sincos_pre) {
        // every joint angle's (sin, cos) by all lanes, three independent chains per lane, so the
        // FK lanes' chain is frame products only
        // (each element is read and overwritten by one lane; a clamped read past the end may see a
        // sine already stored there, and its result is discarded)
        const int JN = J * N;
        for (int i0 = tid; i0 - tid < JN; i0 += 3 * BLOCK) {
            double q[3], sn[3], cs[3];
#pragma unroll
            for (int u = 0; u < 3; ++u) q[u] = traj[min(i0 + u * BLOCK, JN - 1)];
#pragma unroll
            for (int u = 0; u < 3; ++u) det_sincos(q[u], &sn[u], &cs[u]);
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                if (i0 + u * BLOCK < JN) {
                    traj[i0 + u * BLOCK] = sn[u];
                    sv[i0 + u * BLOCK] = cs[u];
                }
            }
        }
        __syncthreads();
    }
    if constexpr (PHASED) {
        // ---- the phased evaluation (one workgroup per CU): the FK lanes run the whole program
        // and leave every sphere slot's frame in LDS; then every (sphere, waypoint) pair at once
        // (one round of gathers), the velocities of the non-zero pairs, and the fold over all
        // spheres in list order.  Same expressions, same order per waypoint as the slot loop.
        __builtin_amdgcn_s_setprio(3);
        // the waves without FK lanes price the row (deferred control costs), one joint per wave
        const int fk_off = t_own - tid;   // -128 or 0
        const int fk_w0 = -fk_off / 64, fk_w1 = (N - 1 - fk_off) / 64;
        // N <= 256 (cost_supported) puts the FK lanes on at most four of the eight waves
        static_assert(!PHASED || BLOCK >= 512, "the phased body prices rows on its non-FK waves");
        if (defer && (wv < fk_w0 || wv > fk_w1)) {
            const int nfk = fk_w1 - fk_w0 + 1;
            const int cw = wv < fk_w0 ? wv : wv - nfk;
            for (int d = cw; d < J; d += NW - nfk)
                wave_control(a.nz, (size_t)pr * J * N, zA, zB, d, lane);
        }
        if (fk_lane) {
            for (int op = 0; op < m.nops; ++op) {
                const FkOp o = ops_s[op];
                fk_op(o);
                if (o.slot >= 0) {
                    double* dst = fb + (size_t)o.slot * 12 * N + t_own;
#pragma unroll
                    for (int k = 0; k < 9; ++k) dst[k * N] = C.R[k];
#pragma unroll
                    for (int k = 0; k < 3; ++k) dst[(9 + k) * N] = C.p[k];
                }
                if (op < 40) STAMP(100 + op);
            }
        }
        __builtin_amdgcn_s_setprio(2);
        if (tid == 0) nz_count = 0;
        __syncthreads();   // every slot's frame published
        STAMP(10);
        // lane (g, t): spheres [g CPL, (g + 1) CPL) at waypoint t, contiguous so that a lane's
        // spheres mostly share a frame; kLaneSpheres lookups with their gathers in flight at once
        const int CPL = (S + G - 1) / G;
        if (pg < G) {
            double F[12];
            int fslot = -1;
            for (int u0 = 0; u0 < CPL; u0 += kLaneSpheres) {   // uniform
                unsigned dv[kLaneSpheres];
#pragma unroll
                for (int u = 0; u < kLaneSpheres; ++u) {
                    if (u0 + u >= CPL) break;   // uniform
                    const int sc = min(pg * CPL + u0 + u, S - 1);
                    const DevSphere& sp = sph[sc];
                    if (sp.slot != fslot) {
                        fslot = sp.slot;
                        const double* src = fb + (size_t)fslot * 12 * N + pt;
#pragma unroll
                        for (int k = 0; k < 12; ++k) F[k] = src[k * N];
                    }
                    double x[3];
#pragma unroll
                    for (int i = 0; i < 3; ++i)
                        x[i] = F[3 * i] * sp.pos[0] + F[3 * i + 1] * sp.pos[1] + F[3 * i + 2] * sp.pos[2] + F[9 + i];
                    dv[u] = sdf_d2<BRICK>(m, x);
                }
#pragma unroll
                for (int u = 0; u < kLaneSpheres; ++u) {
                    if (u0 + u >= CPL) break;   // uniform
                    const int sq = pg * CPL + u0 + u;
                    const bool in = sq < S;
                    bool nz = false;
                    if (in) {
                        const DevSphere& sp = sph[sq];
                        const int d2 = (int)dv[u];
                        col |= d2 < sp.col_lim;
                        nz = d2 < sp.zero_lim;
                        // a non-zero pair keeps its d2 until the velocity phase prices it; a = pot * |v|
                        // is +0 exactly when pot == +0
                        av[sq * N + pt] = nz ? (double)d2 : 0.0;
                    }
                    const unsigned long long mask = __ballot(nz);
                    if (mask) {
                        const int lane_id = tid & 63;
                        const int leader = __ffsll((long long)mask) - 1;
                        int base = 0;
                        if (lane_id == leader) base = atomicAdd(&nz_count, __popcll(mask));
                        base = __shfl(base, leader, 64);
                        if (nz) nzl[base + __popcll(mask & ((1ull << lane_id) - 1ull))] = (unsigned short)(sq * N + pt);
                    }
                }
            }
        }
        __syncthreads();   // pots and the non-zero list complete
        STAMP(11);
        __builtin_amdgcn_s_setprio(3);
        for (int i = tid; i < nz_count; i += BLOCK) {
            const int it = nzl[i];
            const int qi = it / N, ti = it - qi * N;
            const DevSphere& sp = sph[qi];
            const double pot = potential(sp, sdf_metres(m, (unsigned)av[it]));
            av[it] = pot * sphere_speed(m, fb + (size_t)sp.slot * 12 * N, pad, sp, qi, ti);
        }
        __syncthreads();   // every a value complete
        STAMP(12);
        if (fk_lane) fold_avalues(av + t_own, N, S, cum, state);   // in sphere order
        __builtin_amdgcn_s_setprio(2);
        STAMP(13);
    } else {
    // the FK chain and the ordered fold run on two waves while the other waves wait at the
    // next barrier: they are this workgroup's critical path, so they take issue priority (3)
    // over the co-resident workgroup's wide, VALU-heavy pair and velocity phases (2) and the
    // pregen blocks (0)
    __builtin_amdgcn_s_setprio(3);
    int op = fk_advance(0);
    __builtin_amdgcn_s_setprio(2);
    int run = 0;   // sphere runs done (stamp index only)
    STAMP(7);
    while (op < m.nops) {
        const FkOp o = op_at(op);
        if (fk_lane) {
#pragma unroll
            for (int k = 0; k < 9; ++k) fb[k * N + t_own] = C.R[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) fb[(9 + k) * N + t_own] = C.p[k];
        }
        if (tid == 0) nz_count = 0;
        __syncthreads();   // frame published; every lane's previous fold is done
        STAMP(10 + 4 * run);
        // one run of the slot's spheres (all of them, or run_max(N) at a time: the a-value
        // buffer and the pair list hold one run); runs of a slot follow in sphere order and
        // re-publish the same frame
        const int sb = o.sph_begin, se = o.sph_end;
        const int ns = se - sb;
        // lane (g, t) = (tid / N, tid % N): its frame column is read once (all 12 LDS reads in
        // flight) and serves spheres g, g + G, ... of the slot
        // Every sphere of the run this lane takes (at most kLaneSpheres: a run holds <= 16
        // spheres and G >= 2 when N <= 128; <= 8 spheres and G >= 1 otherwise) is looked up with
        // all its gathers in flight at once, and they stay in flight through the FK advance
        // below: no branch around the loads (every lane runs them; past the run's spheres, and
        // on the lanes past the pair lanes, a lookup repeats a valid one and is not used) and the
        // out-of-grid select at the use, since the compiler waits for a load whose register
        // leaves a divergent region or is copied
        unsigned dv[kLaneSpheres];
        unsigned okm = 0;
        {
            double F[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) F[k] = fb[k * N + pt];
#pragma unroll
            for (int u = 0; u < kLaneSpheres; ++u) {
                if (u * G >= ns) break;   // uniform: no lane takes a u-th sphere of this run
                double pos[3];
                if constexpr (LEAN == 2) {   // G = 1: sphere u on every lane, a uniform index (scalar loads)
#pragma unroll
                    for (int i = 0; i < 3; ++i) pos[i] = csph[sb + u].pos[i];
                } else {
                    const double* ps = sph[sb + min(pg + u * G, ns - 1)].pos;
#pragma unroll
                    for (int i = 0; i < 3; ++i) pos[i] = ps[i];
                }
                double x[3];
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    x[i] = F[3 * i] * pos[0] + F[3 * i + 1] * pos[1] + F[3 * i + 2] * pos[2] + F[9 + i];
                bool ok;
                const unsigned idx = sdf_cell<BRICK>(m, x, ok);
                dv[u] = m.sdf[idx];
                okm |= (unsigned)ok << u;
            }
        }
        STAMP(40 + run);
        // while the gathers are in flight the FK lanes run the program on to the next sphere
        // segment (C in registers; fb keeps this slot's frame for the velocities, and the next
        // frame is published after the fold)
        int next_op = op;
        if constexpr (FK_OVERLAP) {
            __builtin_amdgcn_s_setprio(3);
            next_op = fk_advance(op + 1);
            __builtin_amdgcn_s_setprio(2);
        }
        if (pg < G) {
            // the potentials and the pair list
#pragma unroll
            for (int u = 0; u < kLaneSpheres; ++u) {
                if (u * G >= ns) break;   // uniform
                const int q = LEAN == 2 ? u : pg + u * G;   // LEAN 2: G = 1 and pg = 0 here
                const bool in = q < ns;
                bool nz = false;
                if (in) {
                    int zl, cl;
                    if constexpr (LEAN == 2) {
                        zl = csph[sb + q].zero_lim;
                        cl = csph[sb + q].col_lim;
                    } else {
                        zl = sph[sb + q].zero_lim;
                        cl = sph[sb + q].col_lim;
                    }
                    const int d2 = (okm >> u) & 1u ? (int)dv[u] : 0;
                    col |= d2 < cl;
                    nz = d2 < zl;
                    // a non-zero pair keeps its d2 until the velocity phase prices it; a = pot * |v|
                    // is +0 exactly when pot == +0
                    av[q * N + pt] = nz ? (double)d2 : 0.0;
                }
                const unsigned long long mask = __ballot(nz);
                if (mask) {
                    const int lane_id = tid & 63;
                    const int leader = __ffsll((long long)mask) - 1;
                    int base = 0;
                    if (lane_id == leader) base = atomicAdd(&nz_count, __popcll(mask));
                    base = __shfl(base, leader, 64);
                    if (nz) nzl[base + __popcll(mask & ((1ull << lane_id) - 1ull))] = (unsigned short)(q * N + pt);
                }
            }
        }
        __syncthreads();   // pots and the non-zero list complete
        STAMP(11 + 4 * run);
        // velocities only for the listed pairs, spread densely over the block: usually fewer
        // pairs than lanes, one latency chain each, so at the critical-path priority too
        __builtin_amdgcn_s_setprio(3);
        for (int i = tid; i < nz_count; i += BLOCK) {
            const int it = nzl[i];
            const int qi = it / N, ti = it - qi * N;
            if constexpr (LEAN == 2) {
                const DevSphere sp = load_sph(csph + sb + qi);
                const double pot = potential(sp, sdf_metres(m, (unsigned)av[it]));
                av[it] = pot * sphere_speed(m, fb, pad, sp, sb + qi, ti);
            } else {
                const DevSphere& sp = sph[sb + qi];
                const double pot = potential(sp, sdf_metres(m, (unsigned)av[it]));
                av[it] = pot * sphere_speed(m, fb, pad, sp, sb + qi, ti);
            }
        }
        if constexpr (!FK_OVERLAP) {
            // C is reloaded from fb (not kept live across the pairs)
            if (fk_lane) {
#pragma unroll
                for (int k = 0; k < 9; ++k) C.R[k] = fb[k * N + t_own];
#pragma unroll
                for (int k = 0; k < 3; ++k) C.p[k] = fb[(9 + k) * N + t_own];
            }
        }
        __syncthreads();   // the slot's a values complete; fb free for the next slot
        STAMP(12 + 4 * run);
        __builtin_amdgcn_s_setprio(3);
        if (fk_lane) fold_avalues(av + t_own, N, se - sb, cum, state);   // in sphere order
        // the program's control flow is uniform, so every lane has the same next op
        if constexpr (FK_OVERLAP) op = next_op;
        else op = fk_advance(op + 1);
        __builtin_amdgcn_s_setprio(2);
        STAMP(13 + 4 * run);
        ++run;
    }
    }
    STAMP(4);
    if (col) flag = 1;   // every writer stores 1
    // lane t's cost into av[t], which only lane t's fold reads: one barrier covers the flag and
    // the costs, and the state-cost stores come after it (a global store before a barrier makes
    // the barrier wait for its completion)
    double cost = 0.0;
    if (fk_lane) {
        cost = m.w_obs * state + m.w_con * 0.0 + m.w_tq * 0.0;   // :1148-1151
        av[t_own] = cost;
    }
    __syncthreads();
    if (fk_lane) {
        double* so = extra ? a.x_state : a.state_out + (long long)e * N;
        so[t_own] = cost;
    }
    if (tid == 0) {
        const bool cf = !flag && !(member == 0 && m.pad_collision);
        uint8_t* cfo = extra ? a.x_cf : (a.cf_out ? a.cf_out + e : nullptr);
        double* to = extra ? a.x_total : (a.total_out ? a.total_out + e : nullptr);
        if (cfo) *cfo = cf ? 1 : 0;
        if (to) {
            // costs.sum() (:1155), sequential; the reads are independent so they pipeline
            double s = 0.0;
            int k = 0;
            for (; k + 8 <= N; k += 8) {
                double v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = av[k + q];
#pragma unroll
                for (int q = 0; q < 8; ++q) s += v[q];
            }
            for (; k < N; ++k) s += av[k];
            *to = s;
        }
    }
    STAMP(5);
    BLOCK_END();
}

template <int BLOCK, bool BRICK, int LEAN = 0>
__global__ __launch_bounds__(BLOCK, rollout_min_waves<BLOCK>()) void k_rollout(DevModel m, CostArgs a)
{
    rollout_body<BLOCK, BRICK, false, true, LEAN>(m, a, blockIdx.x);
}

// the phased evaluation for launches whose rollouts run one per CU (LDS: rollout_lds phased)
template <bool BRICK>
__global__ __launch_bounds__(kWideBlock, kWideBlock > 512 ? 4 : 2) void k_rollout_phased(DevModel m, CostArgs a)
{
    rollout_body<kWideBlock, BRICK, true>(m, a, blockIdx.x);
}

// one launch for the rollouts of a group of engines of one shape (stomp_group_run): every
// engine's rollout workgroups first (engine p's nro of them at p nro), then every engine's
// pregen blocks (npre each, at the default priority behind them all); models and arguments
// live in device memory, one entry per engine
template <int BLOCK, bool BRICK>
__global__ __launch_bounds__(BLOCK, rollout_min_waves<BLOCK>()) void k_rollout_group(const DevModel* ms, const CostArgs* as,
                                                                           int engines, int nro, int npre)
{
    const int b = blockIdx.x;
    int p, bid;
    if (b < engines * nro) {
        p = b / nro;
        bid = b - p * nro;
    } else {
        const int j = b - engines * nro;
        p = j / npre;
        bid = nro + (j - p * npre);
    }
    // the per-engine models and arguments read through the constant address space: wave-uniform
    // scalar loads the compiler may repeat, as it does for a kernel argument
    using CModel = const __attribute__((address_space(4))) DevModel;
    using CArgs = const __attribute__((address_space(4))) CostArgs;
    // the FK advance overlaps the gathers here too: with the arguments in the constant address space
    // the grouped kernel fits it in 162 VGPRs without spilling (it had spilled 104 B per lane with
    // the generic-pointer arguments, round 3)
    rollout_body<BLOCK, BRICK, false, true>(*(const DevModel*)((CModel*)ms + p), *(const CostArgs*)((CArgs*)as + p), bid);
}

// ---- the waypoint-split rollout (k_rollout_split): when a launch's rollouts fit P >= 2 to a CU
// (the K-sharded ranks, cfg1, the deferred noiseless rollout) rollout e runs on P workgroups,
// piece p owning the free waypoints [t0, t1) = [p N / P, (p + 1) N / P).  Everything but the
// joint-limit passes is per waypoint or needs a halo of the velocity stencil's taps
// (stomp_optimizer.cpp:618-709, 1096-1105): each piece makes the whole row and runs
// handleJointLimits on it (as the one-workgroup rollout does), then the FK program on the
// waypoints [x0, x1) = [t0 - 1, t1 + 2) clamped to [0, N) (one lane per waypoint, every slot's
// frame kept in LDS), the (sphere, waypoint) pairs of its own waypoints, their velocities and the
// fold.  The last piece of a rollout to finish (a per-rollout counter, agent-scope release /
// acquire, no waiting) reads the N costs back and makes costs.sum() (:1155) and the collision
// flag.  Same expressions, same order per waypoint: bit-identical to the other bodies.
namespace {
constexpr int kSplitHaloL = 3 - kVelTap0;   // velocity taps reach t - 1 .. t + 2
constexpr int kSplitHaloR = kVelTap1 - 3;
}

struct SplitLds {
    size_t traj, ps, sv, fb, av, nzl, zA, zB, img, total;
};

// W: FK waypoints of the widest piece, Wo: its own waypoints
__host__ __device__ inline SplitLds split_lds(int J, int N, int S, int nsaves, int nslots, int W, int Wo,
                                              size_t img_bytes)
{
    SplitLds l;
    l.traj = 0;
    l.ps = l.traj + (size_t)J * N * sizeof(double);                // pose rotations [J][9][W]
    l.sv = l.ps + (size_t)J * 9 * W * sizeof(double);              // saved frames [nsaves][12][W]
    l.fb = l.sv + (size_t)nsaves * 12 * W * sizeof(double);        // slot frames [nslots][12][W]
    l.av = l.fb + (size_t)nslots * 12 * W * sizeof(double);        // a values [S][Wo]
    l.nzl = l.av + (size_t)S * Wo * sizeof(double);                // non-zero pairs
    // the noise phase's buffers alias the pair buffers (dead until the pairs)
    const size_t nzw = (size_t)(N + kBandBatch) * noise_jp(J) > (size_t)J * (N + 12)
                           ? (size_t)(N + kBandBatch) * noise_jp(J) : (size_t)J * (N + 12);
    l.zA = l.av;
    l.zB = l.zA + nzw * sizeof(double);
    size_t end = l.nzl + (size_t)S * Wo * sizeof(unsigned short);
    if (l.zB + nzw * sizeof(double) > end) end = l.zB + nzw * sizeof(double);
    l.img = align16(end);
    l.total = l.img + img_bytes;
    return l;
}

__host__ __device__ inline void split_range(int N, int P, int p, int& t0, int& t1, int& x0, int& x1)
{
    t0 = p * N / P;
    t1 = (p + 1) * N / P;
    x0 = t0 - kSplitHaloL < 0 ? 0 : t0 - kSplitHaloL;
    x1 = t1 + kSplitHaloR > N ? N : t1 + kSplitHaloR;
}

// sphere_speed with the frames of waypoints [x0, x0 + W) in fb ([12][W])
__device__ __forceinline__ double sphere_speed_w(const DevModel& m, const double* fb, int W, int x0,
                                                 const double* pad, const DevSphere& sp, int s, int t)
{
    const int N = m.N;
    double y[7][3];
#pragma unroll
    for (int kk = kVelTap0; kk <= kVelTap1; ++kk) {
        const int tt = t + kk - 3;
        double yf[3];
        apply_lds(fb, W, min(max(tt, 0), N - 1) - x0, sp.pos, yf);
        const int row = tt < 0 ? tt + 6 : (tt >= N ? tt - N + 6 : 0);
        const double* src = pad + (row * m.S + s) * 3;
        const bool in = tt >= 0 && tt < N;
#pragma unroll
        for (int c = 0; c < 3; ++c) y[kk][c] = in ? yf[c] : src[c];
    }
    double v0 = 0.0, v1 = 0.0, v2 = 0.0;
#pragma unroll
    for (int kk = kVelTap0; kk <= kVelTap1; ++kk) {
        const double c = m.vel_coef[kk];
        if (c == 0.0) continue;
        v0 += c * y[kk][0];
        v1 += c * y[kk][1];
        v2 += c * y[kk][2];
    }
    return sqrt(v0 * v0 + v1 * v1 + v2 * v2);
}

template <int BLOCK, bool BRICK>
__global__ __launch_bounds__(BLOCK, BLOCK > 256 ? 2 : 3) void k_rollout_split(DevModel m, CostArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    __shared__ int flag, nz_count, last;
    const int J = m.J, N = m.N, S = m.S, P = a.split;
    const int nro = a.num_noisy + (a.x_params ? 1 : 0);
    const int Wmax = (N + P - 1) / P + kSplitHaloL + kSplitHaloR, Womax = (N + P - 1) / P;
    const RolloutLds R = rollout_lds(J, N, S, m.sph_chunk, m.nsaves, m.nseg, m.nops, m.nslots, m.pad_lds);
    const int nw = (int)((R.pad - R.sph) / 8);   // the table image without the padding positions
    const SplitLds L = split_lds(J, N, S, m.nsaves, m.nslots, Wmax, Womax, (size_t)nw * 8);
    const int bid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int NW = BLOCK / 64;
    double* zA = (double*)(lds_raw + L.zA);
    double* zB = (double*)(lds_raw + L.zB);
    if (bid >= nro * P) {
        const int r = bid - nro * P;
        if (r >= a.pre_rows + a.tot_rows + a.spec_rows) x_ctl_rows_block<BLOCK>(a, m.Nall, zA, zB);
        else if (r >= a.pre_rows + a.tot_rows) spec_block<BLOCK>(a, r - a.pre_rows - a.tot_rows, (double*)lds_raw);
        else if (r >= a.pre_rows) totals_block<BLOCK>(a, J, N, r - a.pre_rows, zA);   // zA, zB: contiguous
        else pregen_block<BLOCK>(a, r, false, zA, zB);
        return;
    }
    if (a.pre_rows > 0 || a.tot_rows > 0) __builtin_amdgcn_s_setprio(2);
    if (a.stop && *a.stop) return;
    STAMP(200);
    BLOCK_BEGIN();
    const int e = bid / P, piece = bid - e * P;
    int t0, t1, x0, x1;
    split_range(N, P, piece, t0, t1, x0, x1);
    const int W = x1 - x0, Wo = t1 - t0;
    // the table image's parts at their offsets relative to its start (RolloutLds from .sph); the
    // padding-row positions (read by the velocities at the trajectory's ends only) stay in HBM
    unsigned char* img0 = lds_raw + L.img - R.sph;
    const DevSphere* sph = (const DevSphere*)(img0 + R.sph);
    const DevSegment* seg_s = (const DevSegment*)(img0 + R.seg);
    const FkOp* ops_s = (const FkOp*)(img0 + R.ops);
    const int* hl_s = (const int*)(img0 + R.hl);
    const double* jlim_s = (const double*)(img0 + R.jlim);
    const double* pad = m.pad_pos;
    double* traj = (double*)(lds_raw + L.traj);
    double* ps = (double*)(lds_raw + L.ps);
    double* sv = (double*)(lds_raw + L.sv);
    double* fb = (double*)(lds_raw + L.fb);
    double* av = (double*)(lds_raw + L.av);
    unsigned short* nzl = (unsigned short*)(lds_raw + L.nzl);

    // ---- the row (as rollout_body), the table image copied meanwhile
    const bool extra = e == a.num_noisy;
    const int member = extra ? a.x_member : a.member;
    const bool gen = a.fused_noise == 1 && !extra;
    const bool pre = a.fused_noise == 2 && !extra;
    const bool priced = a.ctl_by_pre;
    const int pr = e + a.row0;
    constexpr int kCopyBatch = 12 * 256 / BLOCK;
    unsigned long long img[kCopyBatch];
#pragma unroll
    for (int u = 0; u < kCopyBatch; ++u) img[u] = m.img[min(tid + u * BLOCK, nw - 1)];
    PreChunk pc0;
    if (pre) {
        if (priced) pre_chunk_load<BLOCK, false>(a.nz, pr, 0, tid, pc0);
        else pre_chunk_load<BLOCK>(a.nz, pr, 0, tid, pc0);
    }
    // the row's noise / params / control stores: every piece computes the same values; the
    // control rows are dealt over the pieces by joint (defer), the rest is stored by all
    if (gen) {
        rollout_normals<BLOCK>(a.nz, e, zA, zB, tid);
    } else if (!pre) {
        const double* prm = extra ? a.x_params : a.params + (long long)e * a.stride;
        // the extra rollout's rows (addExtraRollouts), unless the launch's last block makes them
        const bool xc = extra && a.x_ctl && piece == 0 && !a.x_ctl_block;
        for (int idx0 = 0; idx0 < J * N; idx0 += 4 * BLOCK) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = prm[min(idx0 + tid + u * BLOCK, J * N - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int idx = idx0 + tid + u * BLOCK;
                if (idx < J * N) {
                    traj[idx] = v[u];
                    if (xc) {
                        a.x_prm[idx] = v[u];
                        a.x_nse[idx] = 0.0;
                        const int d = idx / N, i = idx - d * N;
                        zA[d * m.Nall + i + 6] = v[u] + 0.0;
                    }
                }
            }
        }
        if (xc) rollout_control<BLOCK>(a.nz, 0, zA, zB, tid, a.x_ctl);
    }
    {
        unsigned long long* dst = (unsigned long long*)(lds_raw + L.img);
#pragma unroll
        for (int u = 0; u < kCopyBatch; ++u)
            if (tid + u * BLOCK < nw) dst[tid + u * BLOCK] = img[u];
        for (int w = tid + kCopyBatch * BLOCK; w < nw; w += BLOCK) dst[w] = m.img[w];
    }
    STAMP(201);
    const bool defer = gen || (pre && !priced);
    if (gen) rollout_project<BLOCK, true>(a.nz, e, traj, zA, zB, tid);
    else if (pre) {
        if (priced) rollout_from_pre<BLOCK, true, false>(a.nz, pr, e == 0, traj, zA, zB, tid, pc0);
        else rollout_from_pre<BLOCK, true>(a.nz, pr, e == 0, traj, zA, zB, tid, pc0);
    }
    if (tid == 0) { flag = 0; nz_count = 0; }
    __syncthreads();
    STAMP(202);
    BLOCK_MARK(4);

    // ---- handleJointLimits on the whole row (every piece: the passes couple the waypoints)
    __builtin_amdgcn_s_setprio(3);
    joint_limit_passes<NW>(m, traj, hl_s, jlim_s, lane, wv);
    __builtin_amdgcn_s_setprio(2);
    __syncthreads();
    STAMP(203);
    BLOCK_MARK(5);
    double* tout = extra ? a.x_traj : (a.traj_out ? a.traj_out + (long long)e * J * N : nullptr);
    if (tout)
        for (int idx = tid; idx < J * Wo; idx += BLOCK) {
            const int d = idx / Wo, t = t0 + idx - d * Wo;
            tout[d * N + t] = traj[d * N + t];
        }
    // the joint segments' pose rotations at the piece's FK waypoints (rot * Rot2(axis, q), as
    // compose makes them), one (segment, waypoint) per lane, into ps [q][9][W]
    __syncthreads();
    for (int idx = tid; idx < m.nseg * W; idx += BLOCK) {
        const int g = idx / W, l = idx - g * W;
        const DevSegment& sg = seg_s[g];
        if (sg.q_index < 0) continue;
        double st, ct, R[9];
        det_sincos(traj[sg.q_index * N + x0 + l], &st, &ct);
        pose_rotation(sg, st, ct, R);
        double* dst = ps + (size_t)sg.q_index * 9 * W + l;
#pragma unroll
        for (int k = 0; k < 9; ++k) dst[k * W] = R[k];
    }
    __syncthreads();
    STAMP(204);

    // ---- FK program, row-parallel: frame row r (R[r][0..2], p[r]) depends only on the parent's
    // row r and the pose (compose's products, element by element), so wave fk0 + r runs row r of
    // every frame (lane l: waypoint x0 + l) and writes it to the saved / slot frames; the other
    // waves price the control rows this piece is dealt (joints piece, piece + P, ...)
    const int fk0 = NW >= 8 ? ((bid & 1) ? 5 : 0) : (bid & 1);
    const int r = wv - fk0;
    if (r >= 0 && r < 3) {
        __builtin_amdgcn_s_setprio(3);
        if (lane < W) {
            double c0 = 0.0, c1 = 0.0, c2 = 0.0, cp = 0.0;   // row r of the running frame
            for (int op = 0; op < m.nops; ++op) {
                const FkOp o = ops_s[op];
                if (o.seg >= 0) {
                    const DevSegment& sg = seg_s[o.seg];
                    double PR[9];
                    if (sg.q_index >= 0) {
                        const double* src = ps + (size_t)sg.q_index * 9 * W + lane;
#pragma unroll
                        for (int k = 0; k < 9; ++k) PR[k] = src[k * W];
                    } else {
#pragma unroll
                        for (int k = 0; k < 9; ++k) PR[k] = sg.rot[k];
                    }
                    double b0 = c0, b1 = c1, b2 = c2, bp = cp;
                    if (o.base >= 0) {
                        const double* src = sv + (size_t)o.base * 12 * W + lane;
                        b0 = src[(3 * r + 0) * W];
                        b1 = src[(3 * r + 1) * W];
                        b2 = src[(3 * r + 2) * W];
                        bp = src[(9 + r) * W];
                    }
                    if (o.base == kBaseRoot) {   // the pose itself (r is wave-uniform: selects, no indexing)
                        c0 = r == 0 ? PR[0] : (r == 1 ? PR[3] : PR[6]);
                        c1 = r == 0 ? PR[1] : (r == 1 ? PR[4] : PR[7]);
                        c2 = r == 0 ? PR[2] : (r == 1 ? PR[5] : PR[8]);
                        cp = sg.trans[r];
                    } else {
                        if (sg.q_index < 0 && sg.rot_identity) {   // parent * 1
                            c0 = b0; c1 = b1; c2 = b2;
                        } else {
                            c0 = b0 * PR[0] + b1 * PR[3] + b2 * PR[6];
                            c1 = b0 * PR[1] + b1 * PR[4] + b2 * PR[7];
                            c2 = b0 * PR[2] + b1 * PR[5] + b2 * PR[8];
                        }
                        cp = b0 * sg.trans[0] + b1 * sg.trans[1] + b2 * sg.trans[2] + bp;
                    }
                    if (o.save >= 0) {
                        double* dst = sv + (size_t)o.save * 12 * W + lane;
                        dst[(3 * r + 0) * W] = c0;
                        dst[(3 * r + 1) * W] = c1;
                        dst[(3 * r + 2) * W] = c2;
                        dst[(9 + r) * W] = cp;
                    }
                }
                if (o.slot >= 0) {
                    double* dst = fb + (size_t)o.slot * 12 * W + lane;
                    dst[(3 * r + 0) * W] = c0;
                    dst[(3 * r + 1) * W] = c1;
                    dst[(3 * r + 2) * W] = c2;
                    dst[(9 + r) * W] = cp;
                }
            }
        }
        __builtin_amdgcn_s_setprio(2);
    } else if (defer) {
        const int cw = wv < fk0 ? wv : wv - 3;
        for (int d = piece + P * cw; d < J; d += P * (NW - 3))
            wave_control(a.nz, (size_t)pr * J * N, zA, zB, d, lane);
    }
    __syncthreads();   // every slot's frame published (and the control rows' LDS use done)
    STAMP(205);

    // ---- pairs of the own waypoints: lane (g, tl) takes spheres [g CPL, (g + 1) CPL) at t0 + tl
    bool col = false;
    {
        const int G = BLOCK / Wo, pg = tid / Wo, pt = tid - pg * Wo;
        const int CPL = (S + G - 1) / G;
        const int fc = t0 - x0 + pt;   // the lane's frame column
        if (pg < G) {
            double F[12];
            int fslot = -1;
            for (int u0 = 0; u0 < CPL; u0 += kLaneSpheres) {   // uniform
                unsigned dv[kLaneSpheres];
#pragma unroll
                for (int u = 0; u < kLaneSpheres; ++u) {
                    if (u0 + u >= CPL) break;   // uniform
                    const int sc = min(pg * CPL + u0 + u, S - 1);
                    const DevSphere& sp = sph[sc];
                    if (sp.slot != fslot) {
                        fslot = sp.slot;
                        const double* src = fb + (size_t)fslot * 12 * W + fc;
#pragma unroll
                        for (int k = 0; k < 12; ++k) F[k] = src[k * W];
                    }
                    double x[3];
#pragma unroll
                    for (int i = 0; i < 3; ++i)
                        x[i] = F[3 * i] * sp.pos[0] + F[3 * i + 1] * sp.pos[1] + F[3 * i + 2] * sp.pos[2] + F[9 + i];
                    dv[u] = sdf_d2<BRICK>(m, x);
                }
#pragma unroll
                for (int u = 0; u < kLaneSpheres; ++u) {
                    if (u0 + u >= CPL) break;   // uniform
                    const int sq = pg * CPL + u0 + u;
                    bool nz = false;
                    if (sq < S) {
                        const DevSphere& sp = sph[sq];
                        const int d2 = (int)dv[u];
                        col |= d2 < sp.col_lim;
                        nz = d2 < sp.zero_lim;
                        av[sq * Wo + pt] = nz ? (double)d2 : 0.0;
                    }
                    const unsigned long long mask = __ballot(nz);
                    if (mask) {
                        const int leader = __ffsll((long long)mask) - 1;
                        int base = 0;
                        if (lane == leader) base = atomicAdd(&nz_count, __popcll(mask));
                        base = __shfl(base, leader, 64);
                        if (nz) nzl[base + __popcll(mask & ((1ull << lane) - 1ull))] = (unsigned short)(sq * Wo + pt);
                    }
                }
            }
        }
    }
    __syncthreads();   // pots and the non-zero list complete
    STAMP(206);
    __builtin_amdgcn_s_setprio(3);
    for (int i = tid; i < nz_count; i += BLOCK) {
        const int it = nzl[i];
        const int qi = it / Wo, tl = it - qi * Wo;
        const DevSphere& sp = sph[qi];
        const double pot = potential(sp, sdf_metres(m, (unsigned)av[it]));
        av[it] = pot * sphere_speed_w(m, fb + (size_t)sp.slot * 12 * W, W, x0, pad, sp, qi, t0 + tl);
    }
    if (col) flag = 1;   // every writer stores 1
    __syncthreads();   // every a value complete
    STAMP(207);
    double* so = extra ? a.x_state : a.state_out + (long long)e * N;
    uint8_t* cfo = extra ? a.x_cf : (a.cf_out ? a.cf_out + e : nullptr);
    double* to = extra ? a.x_total : (a.total_out ? a.total_out + e : nullptr);
    const bool combine = cfo || to;   // workgroup-uniform
    if (tid < Wo) {
        double cum = 0.0, state = 0.0;
        fold_avalues(av + tid, Wo, S, cum, state);   // in sphere order
        so[t0 + tid] = m.w_obs * state + m.w_con * 0.0 + m.w_tq * 0.0;   // :1148-1151
        if (combine) __threadfence();   // release: the costs before this piece counts itself done
    }
    __builtin_amdgcn_s_setprio(2);
    STAMP(208);
    if (!combine) return;
    __syncthreads();
    BLOCK_END();
    if (tid == 0) {
        // pieces done in the low 16 bits, pieces that saw a collision above
        const int add = 1 + (flag ? 1 << 16 : 0);
        const int old = atomicAdd(a.split_cnt + e, add);
        last = (old & 0xffff) == P - 1 ? 1 + ((old + add) >> 16 > 0 ? 2 : 0) : 0;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();   // acquire: the other pieces' costs
    if (to && tid < N) av[tid] = so[tid];
    __syncthreads();
    if (tid == 0) {
        const bool any_col = (last & 2) != 0;
        const bool cf = !any_col && !(member == 0 && m.pad_collision);
        if (cfo) *cfo = cf ? 1 : 0;
        if (to) {
            // costs.sum() (:1155), sequential
            double s = 0.0;
            int k = 0;
            for (; k + 8 <= N; k += 8) {
                double v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = av[k + q];
#pragma unroll
                for (int q = 0; q < 8; ++q) s += v[q];
            }
            for (; k < N; ++k) s += av[k];
            *to = s;
        }
        a.split_cnt[e] = 0;   // for the next launch (stream order)
    }
    STAMP(209);
}

// pieces per rollout of a launch of nro rollouts and pre_rows pregen blocks (0: the split body
// does not apply)
int split_pieces(const DevModel& m, int nro, int pre_rows)
{
    if (!m.split_cnt || nro <= 0 || nro > m.split_cap) return 0;   // one counter per rollout
    // m.split_max: STOMP_DEBUG_SPLIT_MAX at creation (1: the phased body; tests and A/B)
    const int cap = m.split_max > 0 ? m.split_max : kSplitMaxDefault;
    int P = std::min(m.cus / nro, std::min(cap, m.N));
    if (P < 2) return 0;
    // the launch's pregen blocks share it: past two workgroups per CU the split pieces take the
    // CUs those blocks need (a gather-mode rank's 65 rollouts beside 512 pregen rows: the phased
    // one-workgroup body is faster there, 40.5 against 44.2 us)
    if (nro * P + pre_rows > 2 * m.cus) return 0;
    // one FK wave per piece
    const int Pmin = (m.N + 63 - kSplitHaloL - kSplitHaloR - 1) / (64 - kSplitHaloL - kSplitHaloR);
    if (P < Pmin) return 0;
    if ((size_t)m.S * ((m.N + P - 1) / P) > 65535) return 0;   // pair ids are 16-bit
    return P;
}

size_t rollout_split_lds_bytes(const DevModel& m, int P)
{
    const int Wo = (m.N + P - 1) / P, W = Wo + kSplitHaloL + kSplitHaloR;
    const RolloutLds R = rollout_lds(m.J, m.N, m.S, m.sph_chunk, m.nsaves, m.nseg, m.nops, m.nslots, m.pad_lds);
    return split_lds(m.J, m.N, m.S, m.nsaves, m.nslots, W, Wo, R.pad - R.sph).total;
}

// the split launch's dynamic LDS: the split body's, or a pricing block's if larger
size_t rollout_split_launch_lds(const DevModel& m, int P, bool spec)
{
    const size_t ls = rollout_split_lds_bytes(m, P);
    return spec ? std::max(ls, price_candidate_lds_bytes(m.J, m.N)) : ls;
}

int rollout_split_pieces(const DevModel& m, int nro, int extra_blocks, bool spec)
{
    const int P = split_pieces(m, nro, extra_blocks);
    if (!P || rollout_split_launch_lds(m, P, spec) + 1024 > kRolloutLdsMax) return 0;
    return P;
}

STOMP_STAMP_ACCESSORS(cost)

// generateRollouts' normals and eps = sigma L z, computeProjectedNoise's M eps for one row per
// workgroup (policy_improvement.cpp:228-236, 473-482): the theta-independent half of the
// rollout kernel's noise phase, run on a side stream while the previous iteration's weights
// and update occupy the main one
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_pregen(NoiseArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_pg[];
    if (a.stop && *a.stop) return;
    const RolloutLds L = rollout_lds(a.J, a.N, 0, 0, 0, 0, 0, 0, 0);
    double* zA = (double*)lds_pg;
    double* zB = (double*)(lds_pg + (L.nzB - L.nzA));
    rollout_normals<BLOCK>(a, blockIdx.x, zA, zB, threadIdx.x);
    if (a.J <= 8) {
        pregen_eps_ng<BLOCK, 2>(a, blockIdx.x, zA, zB, threadIdx.x);
        pregen_meps_ng<BLOCK, 2>(a, blockIdx.x, zB, threadIdx.x);
    } else {
        pregen_eps_ng<BLOCK, 4>(a, blockIdx.x, zA, zB, threadIdx.x);
        pregen_meps_ng<BLOCK, 4>(a, blockIdx.x, zB, threadIdx.x);
    }
}

void launch_pregen(const NoiseArgs& a, int rows, hipStream_t s)
{
    if (rows <= 0) return;
    const RolloutLds L = rollout_lds(a.J, a.N, 0, 0, 0, 0, 0, 0, 0);
    const size_t lds = 2 * (L.nzB - L.nzA);
    hipLaunchKernelGGL((k_pregen<256>), dim3(rows), dim3(256), lds, s, a);
}

template <bool BRICK>
static void launch_cost_group_t(const DevModel& m0, const DevModel* ms, const CostArgs* as, int engines, int nro,
                                int npre, hipStream_t s)
{
    const int blocks = engines * (nro + npre);
    const size_t lds = rollout_lds_bytes(m0, m0.pad_lds);
    if (kWideBlock != kBlock && engines * nro <= m0.cus) {   // e.g. the grouped noiseless flush
        if (lds > 64 * 1024) lds_opt_in((const void*)k_rollout_group<kWideBlock, BRICK>, lds);
        hipLaunchKernelGGL((k_rollout_group<kWideBlock, BRICK>), dim3(blocks), dim3(kWideBlock), lds, s, ms, as,
                           engines, nro, npre);
        return;
    }
    if (lds > 64 * 1024) lds_opt_in((const void*)k_rollout_group<kBlock, BRICK>, lds);
    hipLaunchKernelGGL((k_rollout_group<kBlock, BRICK>), dim3(blocks), dim3(kBlock), lds, s, ms, as, engines, nro,
                       npre);
}

void launch_cost_group(const DevModel& m0, const DevModel* ms, const CostArgs* as, int engines, int nro, int npre,
                       hipStream_t s)
{
    if (engines * (nro + npre) <= 0) return;
    // the group's engines share one shape; the layout is each engine's (its own field copy when
    // bricked), and one launch takes one layout: the group is made of engines of one layout
    if (m0.brick) launch_cost_group_t<true>(m0, ms, as, engines, nro, npre, s);
    else launch_cost_group_t<false>(m0, ms, as, engines, nro, npre, s);
}

bool cost_supported(const DevModel& m)
{
    return m.nops <= kMaxOps && m.nseg <= kMaxSeg && m.nslots <= kMaxSeg && m.J <= kMaxJoints && m.N <= kBlock;
}

size_t rollout_lds_bytes(const DevModel& m, int pad_lds, int lean)
{
    return rollout_lds(m.J, m.N, m.S, m.sph_chunk, m.nsaves, m.nseg, m.nops, m.nslots, lean ? 0 : pad_lds, false,
                       lean).total;
}

size_t rollout_phased_lds_bytes(const DevModel& m)
{
    const size_t dyn = rollout_lds(m.J, m.N, m.S, m.sph_chunk, m.nsaves, m.nseg, m.nops, m.nslots, m.pad_lds, true).total;
    hipFuncAttributes attr;
    size_t stat = 2048;
    if (hipFuncGetAttributes(&attr, (const void*)k_rollout_phased<false>) == hipSuccess) stat = attr.sharedSizeBytes;
    if ((size_t)m.S * m.N > 65535 || dyn + stat > kLdsPerCu) return 0;   // pair ids are 16-bit
    return dyn;
}

size_t rollout_static_lds()
{
    hipFuncAttributes attr;
    if (hipFuncGetAttributes(&attr, (const void*)k_rollout<kBlock, false>) != hipSuccess) return 2048;
    return attr.sharedSizeBytes;
}

// resident rollout workgroups per CU for a given total LDS per workgroup: the smaller of
// the LDS limit and the register limit (4 SIMDs, 512 VGPRs per lane-slot, 8-register
// granules; MI355X_MICROARCH.md occupancy table)
bool rollout_lean_allowed(const DevModel& m, int lean)
{
    return lean == 0 || lean == 1 || (lean == 2 && m.N > kBlock / 2 && m.N <= kBlock);
}

int rollout_blocks_per_cu(size_t lds_total, int lean)
{
    hipFuncAttributes attr;
    int regs = 256;
    const void* fn = lean == 2 ? (const void*)k_rollout<kBlock, false, 2>
                   : lean == 1 ? (const void*)k_rollout<kBlock, false, 1> : (const void*)k_rollout<kBlock, false>;
    if (hipFuncGetAttributes(&attr, fn) == hipSuccess && attr.numRegs > 0)
        regs = attr.numRegs;
    const int alloc = (regs + 7) / 8 * 8;
    int waves_per_simd = 512 / alloc;
    if (waves_per_simd > 8) waves_per_simd = 8;
    const int by_regs = waves_per_simd * 4 / (kBlock / 64);
    const int by_lds = (int)(kLdsPerCu / (lds_total ? lds_total : 1));
    return by_regs < by_lds ? by_regs : by_lds;
}

template <bool BRICK>
static void launch_cost_t(const DevModel& m, const CostArgs& a, hipStream_t s)
{
    const int nro = a.num_noisy + (a.x_params ? 1 : 0);
    // pregen, then totals, then the priced candidates (split launches only)
    const int extra_blocks = (a.pre_rows > 0 ? a.pre_rows : 0) + a.tot_rows + a.spec_rows;
    const int blocks = nro + extra_blocks;
    const size_t lds = rollout_lds_bytes(m, m.pad_lds);
    if (const int P = rollout_split_pieces(m, nro, extra_blocks, a.spec_rows > 0)) {
        const size_t ls = rollout_split_launch_lds(m, P, a.spec_rows > 0);
        assert(nro <= m.split_cap);   // split_pieces keeps nro within the counters
        CostArgs b = a;
        b.split = P;
        b.split_cnt = m.split_cnt;
        // the extra rollout's control rows on a block of their own when one more fits the CUs
        b.x_ctl_block = a.x_params && a.x_ctl && !m.x_ctl_inline && nro * P + extra_blocks + 1 <= m.cus ? 1 : 0;
        lds_opt_in((const void*)k_rollout_split<kSplitBlock, BRICK>, ls);
        hipLaunchKernelGGL((k_rollout_split<kSplitBlock, BRICK>), dim3(nro * P + extra_blocks + b.x_ctl_block),
                           dim3(kSplitBlock), ls, s, m, b);
        return;
    }
    assert(a.spec_rows == 0);   // the engine asks rollout_split_pieces first
    if (kWideBlock != kBlock && nro <= m.cus && m.phased_lds > 0) {
        const size_t lp = m.phased_lds;
        lds_opt_in((const void*)k_rollout_phased<BRICK>, lp);
        hipLaunchKernelGGL(k_rollout_phased<BRICK>, dim3(blocks), dim3(kWideBlock), lp, s, m, a);
        return;
    }
    if (kWideBlock != kBlock && nro <= m.cus) {
        if (lds > 64 * 1024) lds_opt_in((const void*)k_rollout<kWideBlock, BRICK>, lds);
        hipLaunchKernelGGL((k_rollout<kWideBlock, BRICK>), dim3(blocks), dim3(kWideBlock), lds, s, m, a);
        return;
    }
    if (m.lean) {
        // the LDS-lean layout (DevModel::lean): sv_glob holds a block per rollout workgroup
        assert(nro <= m.sv_rows || m.nsaves == 0);
        const size_t ll = rollout_lds_bytes(m, 0, m.lean);
        if (m.lean == 2) {
            if (ll > 64 * 1024) lds_opt_in((const void*)k_rollout<kBlock, BRICK, 2>, ll);
            hipLaunchKernelGGL((k_rollout<kBlock, BRICK, 2>), dim3(blocks), dim3(kBlock), ll, s, m, a);
        } else {
            if (ll > 64 * 1024) lds_opt_in((const void*)k_rollout<kBlock, BRICK, 1>, ll);
            hipLaunchKernelGGL((k_rollout<kBlock, BRICK, 1>), dim3(blocks), dim3(kBlock), ll, s, m, a);
        }
        return;
    }
    if (lds > 64 * 1024) lds_opt_in((const void*)k_rollout<kBlock, BRICK>, lds);
    hipLaunchKernelGGL((k_rollout<kBlock, BRICK>), dim3(blocks), dim3(kBlock), lds, s, m, a);
}

void launch_cost(const DevModel& m, const CostArgs& a, hipStream_t s)
{
    if (a.num_noisy + (a.x_params ? 1 : 0) + (a.pre_rows > 0 ? a.pre_rows : 0) + a.tot_rows + a.spec_rows <= 0)
        return;
    if (m.brick) launch_cost_t<true>(m, a, s);
    else launch_cost_t<false>(m, a, s);
}

}  // namespace stomp
