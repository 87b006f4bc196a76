// k_weights.hip -- exponentiated-cost probability weights and the weighted noise sum.
//
//   S[r,d,t]   = state[r,t] + control[r,d,t]  (or its suffix sum)   computeRolloutCumulativeCosts
//                                                                   (policy_improvement.cpp:301-320)
//   P[r,d,t]   = exp(-10 (S - min_r S) / max(max_r S - min_r S, 1e-8)) / sum_r (...)
//                                                                   computeRolloutProbabilities (:322-368)
//   u[d,t]     = sum_r eps[r,d,t] * P[r,d,t]                        computeParameterUpdates (:370-379)
//
// One workgroup owns TC time-step columns of one joint and stages the K_loc x TC cost tile
// in LDS.  min/max are order-free; both sums use the canonical order (fixed 64-rollout
// blocks summed sequentially, block partials summed in block order), which is what makes
// the K-sharded multi-GPU result bit-identical to one GPU: the W_MINMAX / W_PSUM / W_USUM
// phases emit exactly the per-block partials the fused mode sums, and RCCL moves them.
#include "kernels.h"
#include "update_device.h"
#include "noise_device.h"
#include "stomp_math.h"
#include "stamps.h"

namespace stomp {

// sum_{q < count} p[q * stride], q ascending from 0.0; the LDS reads go out 16 at a time so
// the chain waits on one LDS latency per 16 terms instead of one per term
__device__ __forceinline__ double lds_seq_sum(const double* p, int stride, int count)
{
    double s = 0.0;
    if (count == kSumBlock) {
        // a whole block: no per-term predicate, so the chain is the adds alone (a select after
        // every add made it three dependent operations per term)
#pragma unroll
        for (int q0 = 0; q0 < kSumBlock; q0 += 16) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = p[(q0 + q) * stride];
#pragma unroll
            for (int q = 0; q < 16; ++q) s += v[q];
        }
        return s;
    }
    for (int q0 = 0; q0 < count; q0 += 16) {
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = p[min(q0 + q, count - 1) * stride];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q0 + q < count) s += v[q];
    }
    return s;
}

// The rows kernel's LDS tile V: row r of column cc at r * TCW + cc, each 64-row summation
// block shifted by kVPad doubles so that the block-sum threads (one per block and column,
// reading row q of their block together) hit distinct banks: without the shift the blocks
// are 64 * TCW * 8 B apart, a multiple of the 256-B bank row, and all land on one bank.
constexpr int kVPad = 4;
__device__ __forceinline__ int vidx(int r, int cc, int tcw) { return r * tcw + cc + (r / kSumBlock) * kVPad; }
__host__ __device__ inline size_t weights_rows_v_bytes(int K_loc, int tcw)
{
    return ((size_t)K_loc * tcw + (size_t)((K_loc + kSumBlock - 1) / kSumBlock) * kVPad) * sizeof(double);
}


// EPT: cost-tile elements per lane, K_loc * TC <= EPT * 256
template <int EPT>
__global__ __launch_bounds__(256) void k_weights(WeightArgs a)
{
    constexpr int BLOCK = 256;
    extern __shared__ __attribute__((aligned(16))) double V[];   // K_loc * TC
    __shared__ double red0[BLOCK], red1[BLOCK];
    __shared__ double part[BLOCK];
    __shared__ double mn_s[16], den_s[16], ps_s[16];
    if (a.stop && *a.stop) return;
    const int TC = a.tc, N = a.N, J = a.J, K = a.K_loc;
    const int tid = threadIdx.x, c = tid % TC;
    const int d = blockIdx.y, t0 = blockIdx.x * TC, t = t0 + c;
    const bool colok = t < N;
    const size_t JN = (size_t)J * N;
    const size_t col = (size_t)d * N + t;
    const size_t colc = (size_t)d * N + min(t, N - 1);   // clamped: loads stay unconditional
    const int tcl = min(t, N - 1);
    const int nel = K * TC;
    const int nb = (K + kSumBlock - 1) / kSumBlock;
    STAMP(0);
    // the noise tile is only needed at the end; its loads go out first so they land while
    // the costs are reduced and exponentiated (MINMAX / PSUM never read it)
    double nz[EPT];
    if (a.mode == W_FUSED || a.mode == W_USUM) {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int r = min((tid + k * BLOCK) / TC, K - 1);
            nz[k] = a.noise[(size_t)r * JN + colc];
        }
    }

    if (a.mode != W_USUM) {
        double lmn = __builtin_inf(), lmx = -__builtin_inf();
        // all of a lane's loads in flight together (nel <= EPT * BLOCK by weights_tile):
        // clamped addresses, no loads under divergent branches
        double v[EPT];
        if (a.cum) {
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                const int r = min((tid + k * BLOCK) / TC, K - 1);
                v[k] = a.cum[(size_t)r * JN + colc];
            }
        } else {
            double w[EPT];
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                const int r = min((tid + k * BLOCK) / TC, K - 1);
                v[k] = a.state[(size_t)r * N + tcl];
                w[k] = a.control[(size_t)r * JN + colc];
            }
#pragma unroll
            for (int k = 0; k < EPT; ++k) v[k] += w[k];
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) v[k] = (tid + k * BLOCK < nel && colok) ? v[k] : 0.0;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int el = tid + k * BLOCK;
            if (el < nel) {
                if (colok) {
                    if (v[k] < lmn) lmn = v[k];
                    if (v[k] > lmx) lmx = v[k];
                }
                V[el] = v[k];
            }
        }
        if (a.mode == W_PSUM) {
            if (tid < TC && colok) {
                red0[tid] = -a.mm[JN + col];
                red1[tid] = a.mm[col];
            }
        } else {
            red0[tid] = lmn;
            red1[tid] = lmx;
            __syncthreads();
            if (tid < TC) {
                double mn = red0[tid], mx = red1[tid];
                for (int j0 = tid + TC; j0 < BLOCK; j0 += 16 * TC) {
                    double x0[16], x1[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int j = min(j0 + q * TC, BLOCK - TC + tid);   // stays in this column
                        x0[q] = red0[j];
                        x1[q] = red1[j];
                    }
#pragma unroll
                    for (int q = 0; q < 16; ++q) {   // order-free; the clamped repeats are harmless
                        if (x0[q] < mn) mn = x0[q];
                        if (x1[q] > mx) mx = x1[q];
                    }
                }
                red0[tid] = mn;   // only lanes < TC read these slots from here on
                red1[tid] = mx;
                if (a.mode == W_MINMAX && colok) {
                    a.mm[col] = mx;
                    a.mm[JN + col] = -mn;
                }
            }
            if (a.mode == W_MINMAX) return;
        }
        __syncthreads();
        if (tid < TC) {
            double den = red1[tid] - red0[tid];
            if (den < 1e-8) den = 1e-8;
            den_s[tid] = den;
            mn_s[tid] = red0[tid];
        }
        __syncthreads();
        STAMP(1);
        for (int el = tid; el < nel; el += BLOCK) V[el] = det_exp(-10.0 * (V[el] - mn_s[c]) / den_s[c]);
        __syncthreads();
        STAMP(2);
        if (tid < nb * TC) {
            const int b = tid / TC, cc = tid % TC;
            const int r1 = min(K, (b + 1) * kSumBlock);
            const double s = lds_seq_sum(V + (size_t)b * kSumBlock * TC + cc, TC, r1 - b * kSumBlock);
            part[tid] = s;
            if (a.mode == W_PSUM && t0 + cc < N) a.psum_part[(size_t)b * JN + (size_t)d * N + t0 + cc] = s;
        }
        if (a.mode == W_PSUM) {
            for (int el = tid; el < nel; el += BLOCK)
                if (colok) a.prob[(size_t)(el / TC) * JN + col] = V[el];
            return;
        }
        __syncthreads();
        if (tid < TC) {
            double ps = 0.0;
            for (int b = 0; b < nb; ++b) ps += part[b * TC + tid];
            ps_s[tid] = ps;
        }
    } else {
        double pv[EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) pv[k] = a.prob[(size_t)min((tid + k * BLOCK) / TC, K - 1) * JN + colc];
#pragma unroll
        for (int k = 0; k < EPT; ++k)
            if (tid + k * BLOCK < nel) V[tid + k * BLOCK] = colok ? pv[k] : 0.0;
        if (tid < TC) {
            double ps = 0.0;
            if (t0 + tid < N)
                for (int b = 0; b < a.nb_total; ++b) ps += a.psum_all[(size_t)b * JN + (size_t)d * N + t0 + tid];
            ps_s[tid] = ps;
        }
    }
    __syncthreads();
    STAMP(3);
    {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int el = tid + k * BLOCK;
            if (el >= nel) continue;
            if (!colok) { V[el] = 0.0; continue; }
            const double pn = V[el] / ps_s[c];
            a.prob[(size_t)(el / TC) * JN + col] = pn;
            V[el] = nz[k] * pn;
        }
    }
    __syncthreads();
    if (tid < nb * TC) {
        const int b = tid / TC, cc = tid % TC;
        const int r1 = min(K, (b + 1) * kSumBlock);
        const double s = lds_seq_sum(V + (size_t)b * kSumBlock * TC + cc, TC, r1 - b * kSumBlock);
        part[tid] = s;
        if (a.mode == W_USUM && t0 + cc < N) a.u_part[(size_t)b * JN + (size_t)d * N + t0 + cc] = s;
    }
    if (a.mode == W_USUM) return;
    __syncthreads();
    STAMP(4);
    if (tid < TC && colok) {
        double u = 0.0;
        for (int b = 0; b < nb; ++b) u += part[b * TC + tid];
        a.u[col] = u;
    }
    STAMP(5);
}

// Row-coalesced variant: a workgroup owns TCW consecutive flat columns c = d * N + t of the
// [K][J][N] rows, so every row of its tile is TCW * 8 contiguous bytes (a whole 128-B line at
// TCW = 16) and a wave's load covers 64 / TCW rows of it; lane (rs, cc) holds rows
// rs, rs + RS, ... of column cc in registers.  Same phases, modes and canonical sums as
// k_weights.
// the body of k_weights_rows for tile block bid of nt; V = [K_loc][TCW] dynamic LDS
template <int BLOCK, int TCW, int EPT>
__device__ __forceinline__ void weights_rows(const WeightArgs& a, int bid, int nt, double* V)
{
    constexpr int RS = BLOCK / TCW;
    // the per-wave extremes of the tile's columns, and the block partials (nb TCW <= 256, rows_tcw)
    __shared__ double red0[BLOCK / 64 * TCW], red1[BLOCK / 64 * TCW];
    __shared__ double part[256];
    __shared__ double ps_s[TCW];
    if (a.stop && *a.stop) return;
    const int N = a.N, J = a.J, K = a.K_loc;
    const int JN = J * N;
    const int tid = threadIdx.x, cc = tid % TCW, rs = tid / TCW;
    // XCD-grouped tiles: workgroups are dealt round-robin over the 8 XCDs, so block b takes
    // tile (b mod 8)-th group's (b / 8)-th tile and the tiles sharing a 128-B line of a row
    // meet in one XCD's L2 instead of each fetching the line from memory
    const int x = bid & 7, q8 = nt >> 3, r8 = nt & 7;
    const int tile = x * q8 + min(x, r8) + (bid >> 3);
    const int c0 = tile * TCW, c = c0 + cc;
    const bool colok = c < JN;
    const int cl = min(c, JN - 1);
    const int tcol = cl % N;
    const int nb = (K + kSumBlock - 1) / kSumBlock;
    STAMP(0);
    double nz[EPT];
    if (a.mode == W_FUSED || a.mode == W_USUM) {
#pragma unroll
        for (int k = 0; k < EPT; ++k) nz[k] = a.noise[(size_t)min(rs + RS * k, K - 1) * JN + cl];
    }
    double v[EPT];
    if (a.mode != W_USUM) {
        double lmn = __builtin_inf(), lmx = -__builtin_inf();
        if (a.cum) {
#pragma unroll
            for (int k = 0; k < EPT; ++k) v[k] = a.cum[(size_t)min(rs + RS * k, K - 1) * JN + cl];
        } else {
            double w[EPT];
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                const int r = min(rs + RS * k, K - 1);
                v[k] = a.state[(size_t)r * N + tcol];
                w[k] = a.control[(size_t)r * JN + cl];
            }
            // every load of the tile in flight before the first add (left alone, the scheduler
            // interleaves adds that wait on a few loads at a time: one memory latency each)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < EPT; ++k) v[k] += w[k];
            STAMP(6);
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int r = rs + RS * k;
            if (!colok) v[k] = 0.0;
            if (r < K && colok) {
                if (v[k] < lmn) lmn = v[k];
                if (v[k] > lmx) lmx = v[k];
            }
        }
        double mn, mx;
        if (a.mode == W_PSUM) {
            mn = -a.mm[JN + cl];
            mx = a.mm[cl];
        } else {
            // min / max over the lanes holding the same column (lane xor TCW, 2 TCW, .. 32),
            // then over the four waves through LDS; order-free, so any tree is exact
#pragma unroll
            for (int off = TCW; off < 64; off <<= 1) {
                const double omn = __shfl_xor(lmn, off, 64), omx = __shfl_xor(lmx, off, 64);
                if (omn < lmn) lmn = omn;
                if (omx > lmx) lmx = omx;
            }
            const int lane = tid & 63, wv = tid >> 6;
            if (lane < TCW) {
                red0[wv * TCW + lane] = lmn;
                red1[wv * TCW + lane] = lmx;
            }
            __syncthreads();
            mn = red0[cc];
            mx = red1[cc];
#pragma unroll
            for (int w = 1; w < BLOCK / 64; ++w) {
                const double x0 = red0[w * TCW + cc], x1 = red1[w * TCW + cc];
                if (x0 < mn) mn = x0;
                if (x1 > mx) mx = x1;
            }
            if (a.mode == W_MINMAX) {
                if (tid < TCW && colok) {
                    a.mm[c] = mx;
                    a.mm[JN + c] = -mn;
                }
                return;
            }
        }
        double den = mx - mn;
        if (den < 1e-8) den = 1e-8;
        STAMP(1);

#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int r = rs + RS * k;
            v[k] = det_exp(-10.0 * (v[k] - mn) / den);
            if (r < K) V[vidx(r, cc, TCW)] = v[k];
        }
        __syncthreads();
        STAMP(2);
        if (tid < nb * TCW) {
            const int b = tid / TCW, c2 = tid % TCW;
            const int r1 = min(K, (b + 1) * kSumBlock);
            const double s = lds_seq_sum(V + vidx(b * kSumBlock, c2, TCW), TCW, r1 - b * kSumBlock);
            part[tid] = s;
            if (a.mode == W_PSUM && c0 + c2 < JN) a.psum_part[(size_t)b * JN + c0 + c2] = s;
        }
        if (a.mode == W_PSUM) {
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                const int r = rs + RS * k;
                if (r < K && colok) a.prob[(size_t)r * JN + c] = v[k];
            }
            return;
        }
        __syncthreads();
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) v[k] = colok ? a.prob[(size_t)min(rs + RS * k, K - 1) * JN + cl] : 0.0;
        if (tid < TCW) {
            double ps = 0.0;
            if (colok)
                for (int b = 0; b < a.nb_total; ++b) ps += a.psum_all[(size_t)b * JN + c];
            ps_s[tid] = ps;
        }
        __syncthreads();
    }
    STAMP(3);
    {
        // every lane sums its column's block partials itself (the same sequence on every lane of
        // the column: no extra barrier), then all EPT divisions at once (branch-free, so their
        // chains overlap) before the predicated stores
        double ps;
        if (a.mode == W_USUM) {
            ps = ps_s[cc];
        } else {
            ps = lds_seq_sum(part + cc, TCW, nb);   // b ascending from 0.0, the loads batched
        }
        double pn[EPT], w[EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            pn[k] = v[k] / ps;
            w[k] = colok ? nz[k] * pn[k] : 0.0;
        }
        // every quotient made here, before any predicated store (otherwise the divisions are sunk
        // into the stores' branches one by one, and each store's data register is waited on
        // before the next branch reuses it)
#pragma unroll
        for (int k = 0; k < EPT; ++k) asm volatile("" ::"v"(pn[k]), "v"(w[k]));
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int r = rs + RS * k;
            if (r < K) V[vidx(r, cc, TCW)] = w[k];
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int r = rs + RS * k;
            if (r < K && colok) a.prob[(size_t)r * JN + c] = pn[k];
        }
    }
    __syncthreads();
    if (tid < nb * TCW) {
        const int b = tid / TCW, c2 = tid % TCW;
        const int r1 = min(K, (b + 1) * kSumBlock);
        const double s = lds_seq_sum(V + vidx(b * kSumBlock, c2, TCW), TCW, r1 - b * kSumBlock);
        part[tid] = s;
        if (a.mode == W_USUM && c0 + c2 < JN) a.u_part[(size_t)b * JN + c0 + c2] = s;
    }
    if (a.mode == W_USUM) return;
    __syncthreads();
    STAMP(4);
    if (tid < TCW && colok) a.u[c] = lds_seq_sum(part + tid, TCW, nb);
    STAMP(5);
}

template <int BLOCK, int TCW, int EPT>
__global__ __launch_bounds__(BLOCK) void k_weights_rows(WeightArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double V[];   // [K_loc][TCW]
    weights_rows<BLOCK, TCW, EPT>(a, blockIdx.x, gridDim.x, V);
}

// the weights tiles of a group of engines in one launch (engine p's nt tiles at p nt)
template <int BLOCK, int TCW, int EPT>
__global__ __launch_bounds__(BLOCK) void k_weights_rows_group(const WeightArgs* as, int nt)
{
    extern __shared__ __attribute__((aligned(16))) double V[];
    const int p = blockIdx.x / nt;
    // the engine's arguments through the constant address space (scalar loads, as a kernel argument)
    using CArgs = const __attribute__((address_space(4))) WeightArgs;
    weights_rows<BLOCK, TCW, EPT>(*(const WeightArgs*)((CArgs*)as + p), blockIdx.x - p * nt, nt, V);
}

// K_loc <= 64 (one canonical block), FUSED: one wave per flat column c = d N + t, lane r = rollout
// r, and no LDS or barrier at all: S = state + control (or the cumulative row), min / max by
// butterfly shuffles over the live lanes, P = exp(...) / (0.0 + sum_r exp), u = 0.0 + sum_r
// eps P, both sums r ascending from 0.0 through readlanes (the one-block canonical order of
// weights_rows, bit for bit).  Four columns per workgroup, grouped by XCD like the row tiles.
__device__ __forceinline__ double readlane_f64(double x, int l)
{
    const long long b = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// the column of a wave of the XCD-grouped four-column tiles
__device__ __forceinline__ int wave_column()
{
    const int nt = gridDim.x, bid = blockIdx.x;
    const int x = bid & 7, q8 = nt >> 3, r8 = nt & 7;
    const int tile = x * q8 + min(x, r8) + (bid >> 3);
    return __builtin_amdgcn_readfirstlane(tile * 4 + (int)(threadIdx.x >> 6));
}

// column c's probabilities and update term from lane r's cost v and noise nz (r < K live)
__device__ __forceinline__ void wave_weights(const WeightArgs& a, int c, int lane, int K, double v, double nz)
{
    const int JN = a.J * a.N;
    const bool live = lane < K;
    const size_t r = (size_t)min(lane, K - 1);
    double mn = live ? v : __builtin_inf(), mx = live ? v : -__builtin_inf();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double omn = __shfl_xor(mn, off, 64), omx = __shfl_xor(mx, off, 64);
        if (omn < mn) mn = omn;
        if (omx > mx) mx = omx;
    }
    double den = mx - mn;
    if (den < 1e-8) den = 1e-8;
    const double e = det_exp(-10.0 * (v - mn) / den);
    double s = 0.0;
    for (int q0 = 0; q0 < K; q0 += 8) {
        double b[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) b[q] = readlane_f64(e, min(q0 + q, K - 1));
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q0 + q < K) s += b[q];
    }
    const double ps = 0.0 + s;   // the block partials summed in block order from 0.0
    const double pn = e / ps;
    const double w = nz * pn;
    if (live) a.prob[r * JN + c] = pn;
    double s2 = 0.0;
    for (int q0 = 0; q0 < K; q0 += 8) {
        double b[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) b[q] = readlane_f64(w, min(q0 + q, K - 1));
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q0 + q < K) s2 += b[q];
    }
    if (lane == 0) a.u[c] = 0.0 + s2;
}

__global__ __launch_bounds__(256) void k_weights_wave(WeightArgs a)
{
    if (a.stop && *a.stop) return;
    const int N = a.N, JN = a.J * N, K = a.K_loc;
    const int c = wave_column();
    if (c >= JN) return;   // the whole wave
    const int lane = threadIdx.x & 63, t = c % N;
    const size_t r = (size_t)min(lane, K - 1);
    const double nz = a.noise[r * JN + c];
    double v;
    if (a.cum) {
        v = a.cum[r * JN + c];
    } else {
        const double st = a.state[r * N + t], ct = a.control[r * JN + c];
        v = st + ct;
    }
    wave_weights(a, c, lane, K, v, nz);
}

// k_weights_wave with k_reuse_pick folded in (one device, every candidate priced by the rollout
// launch, K < 64, no cumulative costs): lane l <= K holds candidate l's priced values at the
// wave's column (row K the extra rollout) beside its own generated row's (l < K_gen), all loaded
// in one round trip; every wave ranks the K previous totals itself (lane l's (total, index)
// rank, reuse_choice's order) and each workgroup makes the extra rollout's total from its cost
// rows staged in LDS (candidate_total's t-chains, one lane per row); reused row rr = l - K_gen
// takes the candidate reuse_choice chooses for rank rr by a lane shuffle, writes its params,
// noise and control at the column (and state, column t of joint 0) and prices it with the rest:
// the rows k_reuse_pick copies, with no launch between the rollouts and the weights.  LDS:
// (J + 1) N doubles when the extra rollout is a candidate.
constexpr int kPickStageLoads = 8;   // the extra rollout's (J + 1) N <= 2048 cost values, one pass

__global__ __launch_bounds__(256) void k_weights_wave_pick(WeightArgs a, ReuseArgs ra, double* params, double* noise,
                                                           double* control)
{
    extern __shared__ __attribute__((aligned(16))) double stage[];   // [J + 1][N]
    if (a.stop && *a.stop) return;
    STAMP(10);
    const int N = a.N, J = a.J, JN = J * N, K = a.K_loc, Kp = ra.K, Kg = ra.K_gen, P = (J + 1) * N;
    const int c = wave_column();
    const bool cok = c < JN;   // wave-uniform; a wave past the columns still joins the barrier
    const int cc = min(c, JN - 1), t = cc % N;
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const bool wx = ra.with_extra;
    // every load of the workgroup at once, in the order they are waited on: the previous totals
    // (the ranking), the extra rollout's cost rows (the stage; straight-line, so that no loop
    // header waits on the loads after them), then the generated row and the candidates (needed
    // only after the ranking and the t-chains), unconditional at clamped addresses
    const double cl = ra.costs[min(lane, Kp - 1)];
    const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
    double sv[kPickStageLoads];
    if (wx) {
#pragma unroll
        for (int u = 0; u < kPickStageLoads; ++u)
            if (wbase + u * 256 < P) {
                const int i = min(tid + u * 256, P - 1);
                sv[u] = i < N ? ra.x_state[i] : ra.x_control[i - N];
            }
    }
    const size_t og = (size_t)max(min(lane, Kg - 1), 0);
    double nz = a.noise[og * JN + cc], st = a.state[og * N + t], ct = a.control[og * JN + cc];
    const size_t oq = (size_t)min(lane, Kp);
    const double qp = ra.spec_params[oq * JN + cc], qn = ra.spec_noise[oq * JN + cc], qc = ra.spec_ctl[oq * JN + cc];
    const double* qrow = oq < (size_t)Kp ? ra.src_state + oq * N : ra.x_state;
    const double qs = qrow[t];
    STAMP(11);
    if (wx) {
#pragma unroll
        for (int u = 0; u < kPickStageLoads; ++u)
            if (tid + u * 256 < P) stage[tid + u * 256] = sv[u];
        __syncthreads();
    }
    STAMP(12);
    // the choice is the same for every column: wave 0 makes the extra rollout's total while wave 1
    // ranks the K previous totals, and every wave reads both after one barrier
    __shared__ int inv_s[64];   // the candidate of K-rank j
    __shared__ double xt_s;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (wv == 0) {
        if (wx) {
            // Rollout::getCost's t-chain of the extra rollout's row l (lane l <= J), then the
            // rows' sum in row order (candidate_total)
            double x = 0.0;
            if (lane <= J) {
                const double* v = stage + (size_t)lane * N;
                x = v[0];
                int u0 = 1;
                for (; u0 + 32 <= N; u0 += 32) {
                    double b[32];
#pragma unroll
                    for (int u = 0; u < 32; ++u) b[u] = v[u0 + u];
#pragma unroll
                    for (int u = 0; u < 32; ++u) x += b[u];
                }
                for (; u0 < N; ++u0) x += v[u0];
            }
            double xt = readlane_f64(x, 0);
            for (int d = 0; d < J; ++d) xt += readlane_f64(x, 1 + d);
            if (xt != xt) xt = __builtin_inf();
            if (lane == 0) xt_s = xt;
        }
    } else if (wv == 1) {
        // lane l's K-rank: (total, index) ascending among the K previous rows (independent
        // compares, eight at a time); lanes past K keep their own index, so that the push below
        // is a permutation of the wave
        int rank = 0;
        for (int m0 = 0; m0 < Kp; m0 += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int m = min(m0 + u, Kp - 1);
                const double cm = readlane_f64(cl, m);
                rank += (int)(((cm < cl) | ((cm == cl) & (m < lane))) & (m0 + u < Kp));
            }
        }
        if (lane >= Kp) rank = lane;
        // lane rank(l) receives l: the inverse permutation
        inv_s[lane] = __builtin_amdgcn_ds_permute(rank << 2, lane);
    }
    __syncthreads();
    // reused row rr takes the candidate of K-rank rr, or the extra rollout, or K-rank rr - 1
    // (reuse_choice's two compares)
    const int rr = lane - Kg;
    const int rrc = min(max(rr, 0), 63);
    const int selA = inv_s[rrc], selB = rr > 0 ? inv_s[rrc - 1] : selA;
    int src = min(selA, Kp);
    STAMP(13);
    if (wx) {
        const double xt = xt_s;
        const double cA = __shfl(cl, src, 64), cB = __shfl(cl, min(selB, Kp), 64);
        if (!(cA < xt)) src = (rr > 0 && cB >= xt) ? min(selB, Kp) : Kp;
    }
    STAMP(14);
    const double sp = __shfl(qp, src, 64), sn = __shfl(qn, src, 64), sc = __shfl(qc, src, 64),
                 ss = __shfl(qs, src, 64);
    if (!cok) return;
    if (lane >= Kg) {
        nz = sn;
        st = ss;
        ct = sc;
        if (lane < K) {
            const size_t o = (size_t)lane * JN + c;
            params[o] = sp;
            noise[o] = sn;
            control[o] = sc;
            if (c < N) ra.state[(size_t)lane * N + c] = ss;
        }
    }
    STAMP(15);
    wave_weights(a, c, lane, K, st + ct, nz);
    STAMP(16);
}

STOMP_STAMP_ACCESSORS(weights)

bool launch_weights_pick_ok(const WeightArgs& a, const ReuseArgs& ra)
{
    return a.mode == W_FUSED && !a.cum && a.K_loc == ra.K && ra.K < kSumBlock && ra.K_gen >= 0 &&
           ra.K_gen + ra.Kr == ra.K && ra.spec_params && ra.spec_noise && ra.spec_ctl &&
           (a.J + 1) * a.N <= kPickStageLoads * 256;
}

void launch_weights_pick(const WeightArgs& a, const ReuseArgs& ra, double* params, double* noise, double* control,
                         hipStream_t s)
{
    const size_t lds = ra.with_extra ? (size_t)(a.J + 1) * a.N * sizeof(double) : 0;
    hipLaunchKernelGGL(k_weights_wave_pick, dim3((a.J * a.N + 3) / 4), dim3(256), lds, s, a, ra, params, noise,
                       control);
}

// columns per workgroup of the column-tile kernel (k_weights, the fallback past the row tiles): as
// many as keep K_loc * TC <= 2048
int weights_tile(int K_loc)
{
    int tc = 16;
    while (tc > 1 && (size_t)K_loc * tc > 2048) tc >>= 1;
    return tc;
}

// Row tiles of four flat columns.  K_loc in (256, 1024]: 512-lane workgroups (four or eight rows
// per lane: the exp / division phases are per-lane chains, so more lanes finish them sooner; 12.5
// -> 11.5 us at cfg2 against 256 lanes); up to 256 rows 256 lanes (cfg1's 20 rows: 8.5 us against
// 10.8 with 512); larger K_loc: 256 lanes with up to 32 rows per lane, and
// for K_loc in (2048, 4096] two flat columns per workgroup so a lane's 32 rows still fit its
// registers (the whole K = 4096 of cfg3 on one device; the one-column k_weights tiles read a
// separate line per row there).  0 columns: the shape fits no row tile.
static int rows_tcw(int K_loc)
{
    const int nb = (K_loc + kSumBlock - 1) / kSumBlock;
    if (K_loc <= 32 * 64 && nb * 4 <= 256) return 4;
    if (K_loc <= 32 * 128 && nb * 2 <= 256) return 2;
    return 0;
}

template <int BLOCK, int TCW, int EPT>
static void launch_rows_t(const WeightArgs& a, hipStream_t s)
{
    const int nw = (a.J * a.N + TCW - 1) / TCW;
    const size_t lds = weights_rows_v_bytes(a.K_loc, TCW);
    if (lds > 48 * 1024) lds_opt_in((const void*)k_weights_rows<BLOCK, TCW, EPT>, lds);
    hipLaunchKernelGGL((k_weights_rows<BLOCK, TCW, EPT>), dim3(nw), dim3(BLOCK), lds, s, a);
}

void launch_weights(const WeightArgs& a, hipStream_t s)
{
    const int K = a.K_loc;
    if (a.mode == W_FUSED && K <= kSumBlock) {   // one canonical block: a wave per column
        hipLaunchKernelGGL(k_weights_wave, dim3((a.J * a.N + 3) / 4), dim3(256), 0, s, a);
        return;
    }
    switch (rows_tcw(K)) {
    case 4:
        if (K <= 4 * 64) return launch_rows_t<256, 4, 4>(a, s);   // few rows: the wider tile only waits longer
        if (K <= 4 * 128) return launch_rows_t<512, 4, 4>(a, s);
        if (K <= 8 * 128) return launch_rows_t<512, 4, 8>(a, s);
        if (K <= 16 * 64) return launch_rows_t<256, 4, 16>(a, s);
        return launch_rows_t<256, 4, 32>(a, s);
    case 2:
        // (512 lanes with 16 rows each: 159 VGPRs, one workgroup per CU, 96.5 against 81 us at
        // cfg3, profiles/ab/r6_weights_512.txt)
        return launch_rows_t<256, 2, 32>(a, s);
    default:
        break;
    }
    dim3 grid((a.N + a.tc - 1) / a.tc, a.J);
    const size_t lds = (size_t)a.K_loc * a.tc * sizeof(double);
    if ((size_t)a.K_loc * a.tc <= 2048)
        hipLaunchKernelGGL((k_weights<8>), grid, dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL((k_weights<16>), grid, dim3(256), lds, s, a);
}

// computeRolloutCumulativeCosts with use_cumulative_costs (policy_improvement.cpp:308-316)
__global__ void k_cumulative(WeightArgs a, double* cum)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.K_loc * a.J || (a.stop && *a.stop)) return;
    const int r = idx / a.J, d = idx % a.J;
    const int N = a.N;
    double* c = cum + ((size_t)r * a.J + d) * N;
    const double* st = a.state + (size_t)r * N;
    const double* ct = a.control + ((size_t)r * a.J + d) * N;
    for (int t = 0; t < N; ++t) c[t] = st[t] + ct[t];
    if (a.use_cumulative)
        for (int t = N - 2; t >= 0; --t) c[t] += c[t + 1];
}

void launch_cumulative(const WeightArgs& a, double* cum, hipStream_t s)
{
    const int n = a.K_loc * a.J;
    hipLaunchKernelGGL(k_cumulative, dim3((n + 255) / 256), dim3(256), 0, s, a, cum);
}

// delta = M u (policy_improvement.cpp:380), theta += 1.0 * delta (covariant_trajectory_policy.cpp:318-323).
// With u_all (multi-GPU) u is first summed over the all-gathered block partials in block order.
// One output per lane, so registers allow a deep ring: kUpdateBatch rows per batch, three
// batches in flight (the chain waits on M's rows, which the rollout launch evicts from L2)
#ifndef UPDATE_BATCH
#define UPDATE_BATCH 4
#endif
constexpr int kUpdateBatch = UPDATE_BATCH;
#ifndef UPDATE_XPRE
#define UPDATE_XPRE false
#endif

__device__ __forceinline__ void update_body(int d, int J, int N, const double* MT, const double* u,
                                            const double* u_all, int nb_total, double* theta, const int* stop,
                                            double* delta)
{
    __shared__ double us[256 + 2 * kUpdateBatch];
    const int i = threadIdx.x;
    // everything independent is issued up front: the stop flag (checked at the store), this
    // lane's u entry, then (inside band_tile) the first M rows; the LDS fill and its barrier
    // run while those rows are in flight
    const int stopped = stop ? *stop : 0;
    const size_t JN = (size_t)J * N;
    double uv = 0.0;
    if (i < N) {
        if (u_all) {
            for (int b = 0; b < nb_total; ++b) uv += u_all[(size_t)b * JN + (size_t)d * N + i];
        } else {
            uv = u[(size_t)d * N + i];
        }
    }
    auto fill = [&]() {
        if (i < N) us[i] = uv;
        if (i < 2 * kUpdateBatch) us[N + i] = 0.0;
        __syncthreads();
    };
    // k ascending, the noise phase's pinned buffer-load ring (M^T has kMatPadRows zero rows,
    // us has 2 kUpdateBatch zero rows past N: the next batch's rows are read ahead); whole waves run it, lanes past N store nothing
    int col[1] = {min(i, N - 1)};
    double acc[1][1] = {{0.0}};
    band_tile<1, 0, 1, kUpdateBatch, decltype(fill), UPDATE_XPRE>(MT, N, col, 0, N, us, 1, acc, fill);
    const double s = acc[0][0];
    if (i >= N || stopped) return;
    if (delta) delta[(size_t)d * N + i] = s;   // improvePolicy's update alone (PolicyImprovement API)
    else theta[(size_t)d * N + i] += 1.0 * s;
}

// One WG per (16 outputs, joint), 7 x 7 = 49 WGs at cfg2 (update_tile, update_device.h): the tile's
// columns of every M^T row are staged in LDS with all the loads in flight at once (M's rows come
// from HBM after the rollout launch; the ring of update_body, which k_update_group keeps, waits on
// them ~8 times), then 16 lanes run the k-ascending chain out of LDS.  LDS: 17 N doubles.
// Measured: rocprof 4.75 -> 4.57 us; 64-column tiles 5.78 us, 8 columns and LDS reads one batch
// ahead no better (profiles/ab/r3_update_tiles.txt).
__global__ __launch_bounds__(256) void k_update(int J, int N, const double* MT, const double* u, const double* u_all,
                                                int nb_total, double* theta, const int* stop, double* delta)
{
    extern __shared__ double ms[];   // [N][kUpdCols], then u[N]
    const int stopped = stop ? *stop : 0;
    update_tile(J, N, MT, u, u_all, nb_total, theta, stopped != 0, delta, blockIdx.x * kUpdCols, blockIdx.y, ms,
                threadIdx.x);
}

// the updates of a group of engines in one launch (engine p's joint d at p J + d)
__global__ __launch_bounds__(256) void k_update_group(int J, int N, const UpdateArgs* as)
{
    const int p = blockIdx.x / J;
    using CArgs = const __attribute__((address_space(4))) UpdateArgs;   // scalar loads, as a kernel argument
    const UpdateArgs& a = *(const UpdateArgs*)((CArgs*)as + p);
    update_body(blockIdx.x - p * J, J, N, a.MT, a.u, nullptr, 0, a.theta, a.stop, nullptr);
}

void launch_update_group(int J, int N, const UpdateArgs* as, int engines, hipStream_t s)
{
    if (engines > 0) hipLaunchKernelGGL(k_update_group, dim3(J * engines), dim3(256), 0, s, J, N, as);
}

// the rows path of launch_weights for a group (the engine checks weights_group_tiles() > 0)
// columns per tile of the grouped weights launch: eight while K_loc <= 128 (a group's launch has
// engines x tiles workgroups, many rounds of them: wider tiles halve the rounds at the same per-lane
// work, since a tile's time is its dependent phases, not its columns; cfg5 65 -> 44 us,
// profiles/ab/r6_group_weights_fk.txt), else four
static int group_tcw(int K_loc)
{
    return K_loc <= 128 && (K_loc + kSumBlock - 1) / kSumBlock * 8 <= 256 ? 8 : 4;
}

int weights_group_tiles(int J, int N, int K_loc)
{
    if (rows_tcw(K_loc) != 4) return 0;
    const int tcw = group_tcw(K_loc);
    return (J * N + tcw - 1) / tcw;
}

template <int BLOCK, int TCW, int EPT>
static void launch_rows_group_t(const WeightArgs* as, int engines, int nt, int K_loc, hipStream_t s)
{
    const size_t lds = weights_rows_v_bytes(K_loc, TCW);
    if (lds > 48 * 1024) lds_opt_in((const void*)k_weights_rows_group<BLOCK, TCW, EPT>, lds);
    hipLaunchKernelGGL((k_weights_rows_group<BLOCK, TCW, EPT>), dim3(nt * engines), dim3(BLOCK), lds, s, as, nt);
}

void launch_weights_group(const WeightArgs* as, int engines, int J, int N, int K_loc, hipStream_t s)
{
    const int nt = weights_group_tiles(J, N, K_loc);
    if (nt <= 0 || engines <= 0) return;
    if (group_tcw(K_loc) == 8) return launch_rows_group_t<256, 8, 4>(as, engines, nt, K_loc, s);   // 32 rows a pass
    if (K_loc <= 4 * 64) return launch_rows_group_t<256, 4, 4>(as, engines, nt, K_loc, s);
    if (K_loc <= 4 * 128) return launch_rows_group_t<512, 4, 4>(as, engines, nt, K_loc, s);
    if (K_loc <= 8 * 128) return launch_rows_group_t<512, 4, 8>(as, engines, nt, K_loc, s);
    if (K_loc <= 16 * 64) return launch_rows_group_t<256, 4, 16>(as, engines, nt, K_loc, s);
    return launch_rows_group_t<256, 4, 32>(as, engines, nt, K_loc, s);
}

void launch_update(int J, int N, const double* MT, const double* u, const double* u_all, int nb_total, double* theta,
                   const int* stop, hipStream_t s, double* delta)
{
    const size_t lds = update_tile_lds_bytes(N);
    if (lds > 48 * 1024) lds_opt_in((const void*)k_update, lds);
    hipLaunchKernelGGL(k_update, dim3((N + kUpdCols - 1) / kUpdCols, J), dim3(256), lds, s, J, N, MT, u, u_all,
                       nb_total, theta, stop, delta);
}

}  // namespace stomp
