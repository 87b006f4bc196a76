// k_misc.hip -- setup-time and bookkeeping kernels: padding-point FK, rollout reuse,
// distance-field construction.
#include "device_fk.h"
#include "stamps.h"

#include <algorithm>

#include <map>
#include <mutex>
#include <string>
#include <utility>

namespace stomp {

namespace {
thread_local std::string g_opt_in_error;   // the last failed opt-in on this host thread
}

hipError_t lds_opt_in(const void* kernel, size_t bytes)
{
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, size_t> raised;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    size_t& r = raised[{kernel, dev}];
    if (bytes <= r) return hipSuccess;
    const hipError_t st = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (st != hipSuccess) {
        // not recorded as raised: the next launch retries, and the launch error names the size
        g_opt_in_error = "dynamic LDS opt-in of " + std::to_string(bytes) + " bytes on device " + std::to_string(dev) +
                         " failed: " + hipGetErrorString(st);
        (void)hipGetLastError();
        return st;
    }
    r = bytes;
    return hipSuccess;
}

const char* lds_opt_in_error()
{
    return g_opt_in_error.c_str();
}

// padding-point sphere positions: iteration-0 full FK of start (rows 0..5) and goal (rows 6..11)
// (stomp_optimizer.cpp:626-630 with JntToCartFull; padding rows of the group trajectory hold
// start/goal, stomp_trajectory.cpp:94-107)
__global__ void k_pad_fk(DevModel m, const double* start, const double* goal, double* pad_pos, int* pad_cf)
{
    const int side = threadIdx.x;
    if (side > 1) return;
    const double* q = side ? goal : start;
    Frame C, S0, S1;
    bool col = false;
    for (int op = 0; op < m.nops; ++op) {
        const FkOp o = m.ops[op];
        if (o.seg >= 0) {
            const DevSegment& sg = m.segs[o.seg];
            double st = 0.0, ct = 1.0;
            if (sg.q_index >= 0) det_sincos(q[sg.q_index], &st, &ct);
            fk_op(sg, o.base, o.save, st, ct, C, S0, S1);
        }
        for (int s = o.sph_begin; s < o.sph_end; ++s) {
            double p[3];
            apply(C.R, C.p, m.sph[s].pos, p);
            if ((int)sdf_d2(m, p) < m.sph[s].col_lim) col = true;   // distance <= radius
            for (int row = 0; row < 6; ++row)
                for (int c = 0; c < 3; ++c) pad_pos[((size_t)(side * 6 + row) * m.S + s) * 3 + c] = p[c];
        }
    }
    if (col) atomicOr(pad_cf, 1);
}

__global__ void k_gather_max(const double* g, int world, int n, double* out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = g[i];
    for (int r = 1; r < world; ++r) {
        const double x = g[(size_t)r * n + i];
        v = x > v ? x : v;
    }
    out[i] = v;
}

void launch_gather_max(const double* gathered, int world, int n, double* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_gather_max, dim3((n + 255) / 256), dim3(256), 0, s, gathered, world, n, out);
}

void launch_pad_fk(const DevModel& m, const double* start, const double* goal, double* pad_pos, int* pad_cf,
                   hipStream_t s)
{
    hipLaunchKernelGGL(k_pad_fk, dim3(1), dim3(64), 0, s, m, start, goal, pad_pos, pad_cf);
}

// ============================================================== rollout reuse
// Rollout::getCost (policy_improvement.cpp:149-156) as the reference sums it: the state costs
// t-ascending, each joint's control costs t-ascending, then s += joint d for d ascending.  The
// J + 1 t-chains are independent, so each is one lane's (loads two 16-batches ahead of its adds)
// and only the J final adds are serial: a candidate's total costs ~N + J dependent adds instead
// of (J + 1) N dependent loads.
__device__ __forceinline__ double chain_sum(const double* __restrict__ v, int N)
{
    double x = v[0];
    int t = 1;
    double b[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) b[u] = v[min(t + u, N - 1)];
    for (; t + 16 <= N; t += 16) {
        double nb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) nb[u] = v[min(t + 16 + u, N - 1)];
#pragma unroll
        for (int u = 0; u < 16; ++u) x += b[u];
#pragma unroll
        for (int u = 0; u < 16; ++u) b[u] = nb[u];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
        if (t + u < N) x += b[u];
    return x;
}

constexpr int kReusePart = 2048;   // chain sums staged in LDS per pass (doubles)

// totals of candidates [c0, c1) (c == K: the extra rollout) into out[c - c0]; every thread of
// the block takes part, `part` is kReusePart doubles of LDS
__device__ __forceinline__ void reuse_totals_block(int c0, int c1, int K, int J, int N, const double* state,
                                                   const double* control, const double* x_state,
                                                   const double* x_control, double* out, double* part)
{
    const int L = J + 1, per = kReusePart / L;
    const size_t JN = (size_t)J * N;
    for (int a = c0; a < c1; a += per) {
        const int b = min(c1, a + per);
        for (int it = threadIdx.x; it < (b - a) * L; it += blockDim.x) {
            const int c = a + it / L, j = it % L;
            const double* v;
            if (j == 0) v = c < K ? state + (size_t)c * N : x_state;
            else v = (c < K ? control + (size_t)c * JN : x_control) + (size_t)(j - 1) * N;
            part[it] = chain_sum(v, N);
        }
        __syncthreads();
        for (int c = a + threadIdx.x; c < b; c += blockDim.x) {
            const double* q = part + (size_t)(c - a) * L;
            double s = q[0];
            for (int d = 0; d < J; ++d) s += q[1 + d];
            out[c - c0] = s != s ? __builtin_inf() : s;   // NaN ranks last: the ranks stay a permutation
        }
        __syncthreads();
    }
}

// PolicyImprovement::generateRollouts reuse branch (policy_improvement.cpp:176-225): rank the
// K previous rollouts and the extra (noiseless) rollout by Rollout::getCost (:149-156),
// lexicographic on (cost, index) with the extra rollout at index -1 (std::sort of pairs), copy
// the best K_r into rows K_gen.. and re-base their noise on the current theta.
// One 1024-lane workgroup per candidate prices it: its cost rows (state row + J control rows,
// (J + 1) N doubles) staged in LDS with every load in flight, the J + 1 t-chains out of LDS (lane
// per chain, chain_sum's order and roundings), the total to costs_g; the last workgroup to finish
// (a counter, agent-scope release / acquire, no waiting) ranks all candidates and copies the kept
// rows with all their loads in flight.
constexpr int kReuseBlock = 1024;
constexpr size_t kReuseLds = 156 * 1024;

__global__ __launch_bounds__(kReuseBlock) void k_reuse(int K, int J, int N, int Kr, int K_gen, int with_extra,
                                                       const double* src_params, const double* src_state,
                                                       const double* control, double* params, double* noise,
                                                       double* state, const double* x_params, const double* x_state,
                                                       const double* x_control, const double* theta, double* costs_g,
                                                       int* count, const int* stop, int costs_only)
{
    if (stop && *stop) return;
    extern __shared__ __attribute__((aligned(16))) double sh[];
    __shared__ double part[kMaxJoints + 1];
    __shared__ int last;
    const int n = K + with_extra;
    const int tid = threadIdx.x, c = blockIdx.x;
    const int L = J + 1, P = L * N;
    const size_t JN = (size_t)J * N;
    STAMP(0);
    {
        double* stage = sh;   // [L][N]
        constexpr int kMaxLoads = 4;
        for (int i0 = tid; i0 < P; i0 += kMaxLoads * kReuseBlock) {
            double v[kMaxLoads];
#pragma unroll
            for (int u = 0; u < kMaxLoads; ++u) {
                const int i = min(i0 + u * kReuseBlock, P - 1);
                v[u] = i < N ? (c < K ? src_state + (size_t)c * N : x_state)[i]
                             : (c < K ? control + (size_t)c * JN : x_control)[i - N];
            }
#pragma unroll
            for (int u = 0; u < kMaxLoads; ++u)
                if (i0 + u * kReuseBlock < P) stage[i0 + u * kReuseBlock] = v[u];
        }
        __syncthreads();
        STAMP(1);
        if (tid < L) {
            // chain_sum's order: x = v[0], then x += v[t] for t ascending; the next 16 values
            // are read while this 16 are added (two buffers that swap roles, no copies)
            const double* v = stage + (size_t)tid * N;
            double x = v[0];
            double b0[16], b1[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) b0[u] = v[min(1 + u, N - 1)];
            for (int t0 = 1; t0 < N; t0 += 32) {
#pragma unroll
                for (int u = 0; u < 16; ++u) b1[u] = v[min(t0 + 16 + u, N - 1)];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (t0 + u < N) x += b0[u];
                if (t0 + 16 >= N) break;
#pragma unroll
                for (int u = 0; u < 16; ++u) b0[u] = v[min(t0 + 32 + u, N - 1)];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (t0 + 16 + u < N) x += b1[u];
            }
            part[tid] = x;
        }
        __syncthreads();
        STAMP(2);
        if (tid == 0) {
            double s2 = part[0];
            for (int d = 0; d < J; ++d) s2 += part[1 + d];
            costs_g[c] = s2 != s2 ? __builtin_inf() : s2;   // NaN ranks last: the ranks stay a permutation
            if (!costs_only) {
                __threadfence();   // release: the total before the count
                last = atomicAdd(count, 1) == n - 1;
            } else {
                last = 0;   // the ranking and copies are the reused rows' kernel's (launch_reuse_rows)
            }
        }
        __syncthreads();
        STAMP(3);
    }
    if (!last) return;
    STAMP_ANY(10);
    __threadfence();   // acquire: every candidate's total
    double* costs = sh;                       // [n] (the stage is dead)
    int* sel = (int*)(costs + n);             // [Kr]
    for (int i = tid; i < n; i += kReuseBlock) costs[i] = costs_g[i];
    __syncthreads();
    STAMP_ANY(11);
    for (int cc0 = tid; cc0 < n; cc0 += kReuseBlock) {
        const int ic = cc0 < K ? cc0 : -1;
        const double cc = costs[cc0];
        int rank = 0;
        for (int c0 = 0; c0 < n; c0 += 8) {   // eight reads in flight, then the compares
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = costs[min(c0 + u, n - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int c2 = c0 + u, ic2 = c2 < K ? c2 : -1;
                if (c2 < n && (x[u] < cc || (x[u] == cc && ic2 < ic))) ++rank;
            }
        }
        if (rank < Kr) sel[rank] = cc0;
    }
    __syncthreads();
    STAMP_ANY(12);
    // the kept rows into rows K_gen.. of this iteration's set (the row sets are distinct buffers,
    // launch_reuse checks it): params row, noise = params - theta, state row; all loads of a batch
    // in flight before its stores
    const int W = (int)JN + N;
    constexpr int kCopyRows = 16;
    for (int i = tid; i < W; i += kReuseBlock) {
        const bool pr = i < (int)JN;
        const double th = pr ? theta[i] : 0.0;
        for (int r0 = 0; r0 < Kr; r0 += kCopyRows) {
            double v[kCopyRows];
#pragma unroll
            for (int u = 0; u < kCopyRows; ++u) {
                const int src = sel[min(r0 + u, Kr - 1)];
                v[u] = pr ? (src < K ? src_params + (size_t)src * JN : x_params)[i]
                          : (src < K ? src_state + (size_t)src * N : x_state)[i - (int)JN];
            }
#pragma unroll
            for (int u = 0; u < kCopyRows; ++u) {
                const int r = r0 + u;
                if (r >= Kr) break;
                if (pr) {
                    params[(size_t)(K_gen + r) * JN + i] = v[u];
                    noise[(size_t)(K_gen + r) * JN + i] = v[u] - th;
                } else {
                    state[(size_t)(K_gen + r) * N + (i - (int)JN)] = v[u];
                }
            }
        }
    }
    if (tid == 0) *count = 0;   // for the next launch (stream order)
    STAMP_ANY(13);
}

int launch_reuse(int K, int J, int N, int Kr, int K_gen, int with_extra, const double* src_params,
                 const double* src_state, const double* src_control, double* params, double* noise, double* state,
                 const double* x_params, const double* x_state, const double* x_control, const double* theta,
                 double* costs_g, int* count, const int* stop, hipStream_t s, bool costs_only)
{
    // k_reuse copies straight from the source rows into rows K_gen..: an in-place call would read
    // rows this same loop already overwrote
    if (src_params == params || src_state == state) return -1;
    const int n = K + with_extra, P = (J + 1) * N;
    const size_t rank_bytes = (size_t)n * sizeof(double) + (size_t)Kr * sizeof(int);
    const size_t lds = std::max((size_t)P * sizeof(double), rank_bytes);
    if (lds > kReuseLds) return -2;
    if (lds > 48 * 1024) lds_opt_in((const void*)k_reuse, lds);
    hipLaunchKernelGGL(k_reuse, dim3(n), dim3(kReuseBlock), lds, s, K, J, N, Kr, K_gen, with_extra, src_params,
                       src_state, src_control, params, noise, state, x_params, x_state, x_control, theta, costs_g,
                       count, stop, costs_only ? 1 : 0);
    return 0;
}

// ---- the same reuse step with the K rows sharded over ranks: every rank prices its
// own rows (Rollout::getCost, policy_improvement.cpp:149-156), the totals are all-gathered, every
// rank ranks all K + 1 candidates identically, the owners pack the chosen rows into slot r of a
// [Kr][J N + N] buffer, the slots are all-gathered and every rank unpacks the reused rows it owns
// (rows K_gen + r, noise re-based on theta, :214-223).  Same ranking, same row order, so the result
// is the single-device one bit for bit.
constexpr int kReuseTotalsPerBlock = 64;   // candidates per k_reuse_totals block (reuse_totals_block)

__global__ __launch_bounds__(256) void k_reuse_totals(int K_loc, int J, int N, const double* state,
                                                      const double* control, const double* x_state,
                                                      const double* x_control, double* tot_loc, double* tot_x,
                                                      const int* stop)
{
    if (stop && *stop) return;
    __shared__ double part[kReusePart];
    __shared__ double tot[kReuseTotalsPerBlock];
    const int c0 = blockIdx.x * kReuseTotalsPerBlock, c1 = min(K_loc + 1, c0 + kReuseTotalsPerBlock);
    reuse_totals_block(c0, c1, K_loc, J, N, state, control, x_state, x_control, tot, part);
    for (int c = c0 + threadIdx.x; c < c1; c += 256) {
        if (c < K_loc) tot_loc[c] = tot[c - c0];
        else *tot_x = tot[c - c0];
    }
}

__global__ __launch_bounds__(256) void k_reuse_select(int K, int Kr, int with_extra, const double* tot_all,
                                                      const double* tot_x, int* sel, const int* stop)
{
    if (stop && *stop) return;
    const int n = K + with_extra;
    for (int c = threadIdx.x; c < n; c += 256) {
        const int ic = c < K ? c : -1;
        const double cc = c < K ? tot_all[c] : *tot_x;
        int rank = 0;
        for (int c2 = 0; c2 < n; ++c2) {
            const int ic2 = c2 < K ? c2 : -1;
            const double x = c2 < K ? tot_all[c2] : *tot_x;
            if (x < cc || (x == cc && ic2 < ic)) ++rank;
        }
        if (rank < Kr) sel[rank] = ic;   // -1: the extra rollout
    }
}

__global__ __launch_bounds__(256) void k_reuse_pack(int Kr, int J, int N, int first, int K_loc, const int* sel,
                                                    const double* params, const double* state, double* slot,
                                                    const int* stop)
{
    if (stop && *stop) return;
    const size_t JN = (size_t)J * N, W = JN + N;
    for (size_t idx = blockIdx.x * 256 + threadIdx.x; idx < (size_t)Kr * W; idx += (size_t)gridDim.x * 256) {
        const int r = (int)(idx / W);
        const size_t off = idx % W;
        const int src = sel[r] - first;
        if (sel[r] < 0 || src < 0 || src >= K_loc) continue;   // another rank's row, or the extra
        slot[idx] = off < JN ? params[(size_t)src * JN + off] : state[(size_t)src * N + (off - JN)];
    }
}

__global__ __launch_bounds__(256) void k_reuse_unpack(int Kr, int K_gen, int J, int N, int first, int K_loc,
                                                      const int* sel, const double* slot_all, const double* x_params,
                                                      const double* x_state, const double* theta, double* params,
                                                      double* noise, double* state, const int* stop)
{
    if (stop && *stop) return;
    const size_t JN = (size_t)J * N, W = JN + N;
    for (size_t idx = blockIdx.x * 256 + threadIdx.x; idx < (size_t)Kr * W; idx += (size_t)gridDim.x * 256) {
        const int r = (int)(idx / W);
        const size_t off = idx % W;
        const int dst = K_gen + r - first;
        if (dst < 0 || dst >= K_loc) continue;
        const int src = sel[r];
        double v;
        if (src < 0) v = off < JN ? x_params[off] : x_state[off - JN];
        else v = slot_all[((size_t)(src / K_loc) * Kr + r) * W + off];
        if (off < JN) {
            params[(size_t)dst * JN + off] = v;
            noise[(size_t)dst * JN + off] = v - theta[off];
        } else {
            state[(size_t)dst * N + (off - JN)] = v;
        }
    }
}

void launch_reuse_totals(int K_loc, int J, int N, const double* state, const double* control, const double* x_state,
                         const double* x_control, double* tot_loc, double* tot_x, const int* stop, hipStream_t s)
{
    hipLaunchKernelGGL(k_reuse_totals, dim3((K_loc + 1 + kReuseTotalsPerBlock - 1) / kReuseTotalsPerBlock), dim3(256), 0,
                       s, K_loc, J, N, state, control,
                       x_state, x_control, tot_loc, tot_x, stop);
}

void launch_reuse_select(int K, int Kr, int with_extra, const double* tot_all, const double* tot_x, int* sel,
                         const int* stop, hipStream_t s)
{
    hipLaunchKernelGGL(k_reuse_select, dim3(1), dim3(256), 0, s, K, Kr, with_extra, tot_all, tot_x, sel, stop);
}

void launch_reuse_pack(int Kr, int J, int N, int first, int K_loc, const int* sel, const double* params,
                       const double* state, double* slot, const int* stop, hipStream_t s)
{
    const size_t n = (size_t)Kr * ((size_t)J * N + N);
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_reuse_pack, dim3(blocks), dim3(256), 0, s, Kr, J, N, first, K_loc, sel, params, state, slot,
                       stop);
}

void launch_reuse_unpack(int Kr, int K_gen, int J, int N, int first, int K_loc, const int* sel,
                         const double* slot_all, const double* x_params, const double* x_state, const double* theta,
                         double* params, double* noise, double* state, const int* stop, hipStream_t s)
{
    const size_t n = (size_t)Kr * ((size_t)J * N + N);
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_reuse_unpack, dim3(blocks), dim3(256), 0, s, Kr, K_gen, J, N, first, K_loc, sel, slot_all,
                       x_params, x_state, theta, params, noise, state, stop);
}

__global__ __launch_bounds__(256) void k_materialize_rows(size_t n, int JN, const double* eps, const double* theta_gen,
                                                          double* noise, double* params)
{
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const double e = eps[i];
        noise[i] = e;
        params[i] = theta_gen[i % JN] + e;   // the rollout kernel's theta + eps
    }
}

void launch_materialize_rows(int K_loc, int JN, const double* eps, const double* theta_gen, double* noise,
                             double* params, hipStream_t s)
{
    const size_t n = (size_t)K_loc * JN;
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_materialize_rows, dim3(blocks), dim3(256), 0, s, n, JN, eps, theta_gen, noise, params);
}

// StompOptimizer::optimize bookkeeping (stomp_optimizer.cpp:301-344) for iteration index `it`
// (iteration_), after its noiseless rollout: collision-free streak, success / collision-success
// iterations, the cost history, best_group_trajectory_ (copied by the whole block) and the
// break condition, which turns every later launch of the loop into a no-op.
__global__ __launch_bounds__(256) void k_track(DevTrack* tr, int it, int max_it_cf, const double* total,
                                               const uint8_t* cf, const uint8_t* cs, double* costs,
                                               const double* last_traj, double* best_traj, int JN)
{
    __shared__ int copy;
    if (tr->stop) return;   // uniform: every thread reads the same flag before any write
    __syncthreads();
    if (threadIdx.x == 0) {
        const double cost = *total;
        const bool cfree = *cf != 0;
        const bool ok = cfree && *cs != 0;
        tr->cfi = ok ? tr->cfi + 1 : 0;
        if (cfree && tr->collision_success_iteration == -1) {
            tr->collision_success_iteration = it;
            tr->t_collision_success = wall_clock64();
        }
        if (ok && tr->success_iteration == -1) {
            tr->success_iteration = it;
            tr->success = 1;
            tr->t_success = wall_clock64();
        }
        costs[it] = cost;
        copy = 0;
        if (it == 0 || (cost < tr->best && ok)) {
            tr->best = cost;
            if (it != 0) tr->last_improvement_iteration = it;
            copy = 1;
        }
        tr->iterations = it + 1;
        if (tr->cfi >= max_it_cf) tr->stop = 1;
    }
    __syncthreads();
    if (copy)
        for (int i = threadIdx.x; i < JN; i += blockDim.x) best_traj[i] = last_traj[i];
}

__global__ void k_track_start(DevTrack* tr)
{
    if (threadIdx.x == 0) tr->t0 = wall_clock64();
}

void launch_track_start(DevTrack* tr, hipStream_t s)
{
    hipLaunchKernelGGL(k_track_start, dim3(1), dim3(64), 0, s, tr);
}

void launch_track(DevTrack* tr, int it, int max_it_cf, const double* total, const uint8_t* cf, const uint8_t* cs,
                  double* costs, const double* last_traj, double* best_traj, int JN, hipStream_t s)
{
    hipLaunchKernelGGL(k_track, dim3(1), dim3(256), 0, s, tr, it, max_it_cf, total, cf, cs, costs, last_traj,
                       best_traj, JN);
}

// ============================================================== distance field construction
__global__ void k_sdf_build(int nx, int ny, int nz, int cap2, const int* boxes, int nb, const long long* cyl_d2,
                            const int* cyl_z, int nc, unsigned short* out)
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
        out[idx] = (unsigned short)d2;   // <= cap2 <= 65535
    }
}

void launch_sdf_build(int nx, int ny, int nz, int cap2, const int* boxes, int nb, const long long* cyl_d2,
                      const int* cyl_z, int nc, unsigned short* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_sdf_build, dim3(2048), dim3(256), 0, s, nx, ny, nz, cap2, boxes, nb, cyl_d2, cyl_z, nc, out);
}

STOMP_STAMP_ACCESSORS(misc)

}  // namespace stomp
