// noise_device.h -- the noise band products and the rollout kernel's fused noise phase.
//
//   eps = sigma_d * (0 + L z)          MultivariateGaussian::sample (multivariate_gaussian.h:88-94)
//                                      via generateRollouts (policy_improvement.cpp:228-236)
//   params = theta + eps               policy_improvement.cpp:234
//   nproj = M eps                      computeProjectedNoise (policy_improvement.cpp:473-482)
//   control = sum_i w_i (D_i x)^2      computeControlCosts (covariant_trajectory_policy.cpp:228-255),
//                                      x = padded (params + nproj), 7-tap stencils instead of dense D_i
//
// Sums run over k in ascending order with one rounding per operation (the oracle's
// contract); the triangular product adds only exact zeros past k = i.
#pragma once

#include "kernels.h"
#include "stamps.h"
#include "stomp_math.h"

namespace stomp {

// acc[rr] = fma(AT[k][i], v[k * vstride + rr], acc[rr]) for k < kend ascending (the noise
// products' contract: one rounding per multiply-add, as on the matrix cores).  Unconditional loads
// in four 8-load batches that rotate roles without register copies, so three batches are in
// flight while one is summed (a copy of the next batch into the current one would make the
// compiler wait for the batch it has just issued).  AT has kMatPadRows zero rows past N and v
// kBandBatch zero rows past N, so neither the loads nor the sums need clamping: terms past
// kend are exact no-ops (zeros of L^T above the diagonal or of the padding; the accumulator
// starts at +0.0 and is never -0.0, so adding +-0.0 leaves it unchanged).
template <int RT>
__device__ __forceinline__ void band_product(const double* __restrict__ AT, int N, int i, int kend,
                                             const double* v, int vstride, double* acc)
{
    constexpr int P = kBandBatch;
    double A0[P], A1[P], A2[P], A3[P];
    auto load = [&](double* buf, int k0) {
#pragma unroll
        for (int q = 0; q < P; ++q) buf[q] = AT[(size_t)(k0 + q) * N + i];
    };
    auto sum = [&](const double* buf, int k0) {
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const double* x = v + (k0 + q) * vstride;
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) acc[rr] = __builtin_fma(buf[q], x[rr], acc[rr]);
        }
    };
    load(A0, 0);
    load(A1, P);
    load(A2, 2 * P);
    for (int k0 = 0; k0 < kend; k0 += 4 * P) {
        load(A3, k0 + 3 * P);
        sum(A0, k0);
        if (k0 + P >= kend) break;
        load(A0, k0 + 4 * P);
        sum(A1, k0 + P);
        if (k0 + 2 * P >= kend) break;
        load(A1, k0 + 5 * P);
        sum(A2, k0 + 2 * P);
        if (k0 + 3 * P >= kend) break;
        load(A2, k0 + 6 * P);
        sum(A3, k0 + 3 * P);
    }
}

// Register-blocked band product of the rollout kernel's noise phase: lane l of a wave owns
// waypoints i_t = l + 64 t (t < TI) and RT joints d0 .. d0 + RT - 1:
//   acc[t][rr] += sum_{k in [kbeg, kend)} AT[k][i_t] * v[k * vstride + rr]   (t >= T0), k ascending.
// One broadcast LDS read of v[k] feeds TI * RT products and one AT row load TI * RT / TI, so
// the VALU, not the LDS or the vector memory path, bounds it.  AT rows come through buffer
// loads (scalar row offset, one VGPR column offset per t) in a rotating four-batch ring,
// three batches ahead; whole batches only (no branch between a batch's load and its use,
// which would let the compiler sink the load to the use): the batch past kend adds exact
// zeros (AT zero rows past N, kMatPadRows >= 4 * 4 * kBandK; v zero rows up to N + kBandBatch).
#ifndef BAND_K
#define BAND_K 4
#endif
constexpr int kBandK = BAND_K;   // rows per batch
static_assert(kMatPadRows >= 4 * 4 * kBandK && kBandBatch >= kBandK, "band_tile padding");
constexpr int kCtlRun = 4;  // padded indices per lane in the rollout kernel's control stencils
// B rows per batch (default kBandK); loads reach row kend + 4B - 1 and v row kend + B - 1.
// `mid` runs after the first three batches are issued (k_update fills v there, so its own loads
// and barrier overlap the ring's first loads).
struct NoMid {
    __device__ void operator()() const {}
};
// XPRE: v's rows for the next batch are read while this batch sums (v then needs 2B zero
// rows past kend)
template <int TI, int T0, int RT, int B = kBandK, class Mid = NoMid, bool XPRE = false>
__device__ __forceinline__ void band_tile(const double* __restrict__ AT, int N, const int* col, int kbeg, int kend,
                                          const double* v, int vstride, double (*acc)[RT], Mid mid = Mid())
{
    static_assert(kMatPadRows >= 4 * B, "band_tile look-ahead past the zero rows");
    constexpr int NT = TI - T0;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)AT, 0, (int)((size_t)(N + kMatPadRows) * N * sizeof(double)), 0x00020000);
    int ioff[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) ioff[t] = col[T0 + t] * (int)sizeof(double);
    double A0[B][NT], A1[B][NT], A2[B][NT], A3[B][NT];
    auto load = [&](double (*buf)[NT], int k0) {
#pragma unroll
        for (int q = 0; q < B; ++q)
#pragma unroll
            for (int t = 0; t < NT; ++t)
                buf[q][t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                           rsrc, ioff[t], (k0 + q) * N * (int)sizeof(double), 0));
        __builtin_amdgcn_sched_barrier(0);   // keep the batch where it is issued
    };
    double xn[B][RT];
    auto sum = [&](const double (*buf)[NT], int k0) {
        double x[B][RT];
        if constexpr (XPRE) {
#pragma unroll
            for (int q = 0; q < B; ++q)
#pragma unroll
                for (int rr = 0; rr < RT; ++rr) {
                    x[q][rr] = xn[q][rr];
                    xn[q][rr] = v[(k0 + B + q) * vstride + rr];
                }
        } else {
#pragma unroll
            for (int q = 0; q < B; ++q)
#pragma unroll
                for (int rr = 0; rr < RT; ++rr) x[q][rr] = v[(k0 + q) * vstride + rr];
        }
#pragma unroll
        for (int q = 0; q < B; ++q)
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int rr = 0; rr < RT; ++rr) acc[T0 + t][rr] += buf[q][t] * x[q][rr];
    };
    const int nb = (kend - kbeg + B - 1) / B;
    int k0 = kbeg, b = 0;
    load(A0, k0);
    load(A1, k0 + B);
    load(A2, k0 + 2 * B);
    mid();
    if constexpr (XPRE) {
#pragma unroll
        for (int q = 0; q < B; ++q)
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) xn[q][rr] = v[(kbeg + q) * vstride + rr];
    }
    for (; b + 4 <= nb; b += 4, k0 += 4 * B) {
        load(A3, k0 + 3 * B); sum(A0, k0);
        load(A0, k0 + 4 * B); sum(A1, k0 + B);
        load(A1, k0 + 5 * B); sum(A2, k0 + 2 * B);
        load(A2, k0 + 6 * B); sum(A3, k0 + 3 * B);
    }
    const int rem = nb - b;   // A0, A1, A2 hold the batches at k0, k0 + B, k0 + 2B
    if (rem >= 1) sum(A0, k0);
    if (rem >= 2) sum(A1, k0 + B);
    if (rem >= 3) sum(A2, k0 + 2 * B);
}

// sum_rule wr * (D_rule x)^2 at padded index ii of one joint's padded trajectory x[0, Nall):
// the 7-tap window first (all LDS reads in flight), then the sums over the taps inside
// [0, Nall) in ascending order
__device__ __forceinline__ double control_term(const NoiseArgs& a, const double* x, int Nall, int ii)
{
    double xw[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) xw[q] = x[min(max(ii - 3 + q, 0), Nall - 1)];
    double call = 0.0;
#pragma unroll
    for (int rule = 0; rule < 3; ++rule) {
        const double wr = a.wr[rule];
        if (wr == 0.0) continue;   // adds +0.0 in the reference: exact to skip
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < 7; ++q)
            if (ii - 3 + q >= 0 && ii - 3 + q < Nall) s += a.dcoef[rule][q] * xw[q];
        call += wr * (s * s);
    }
    return call;
}

// control cost of free waypoint i from the padded per-index terms c[0, Nall): the first and
// last free waypoints also collect the six padding terms on their side
__device__ __forceinline__ double control_cost(const double* c, int N, int Nall, int i)
{
    double o = c[i + 6];
    if (N == 1) {
        for (int q = 0; q < 6; ++q) { o += c[q]; o += c[Nall - 1 - q]; }
    } else if (i == 0) {
        for (int q = 0; q < 6; ++q) o += c[q];
    } else if (i == N - 1) {
        for (int q = 0; q < 6; ++q) o += c[Nall - 1 - q];
    }
    return o;
}

// The whole generateRollouts + computeProjectedNoise + computeControlCosts work of local row
// r, done by one BLOCK-wide workgroup before it executes the row, in two calls:
// rollout_normals (z into zA) and rollout_project (writes the noise / params / control rows
// to HBM and the parameters to traj[J][N] in LDS).  zA and zB are LDS buffers of
// max((N + kBandBatch) * JP, J * Nall) doubles; JP = J rounded up to kNoiseJT.  N <= 128
// (BLOCK = 256: four waves of 32 waypoints; the engine runs the fused phase only then).
template <int BLOCK>
__device__ __forceinline__ void rollout_normals(const NoiseArgs& a, int r, double* zA, double* zB, int tid)
{
    const int J = a.J, N = a.N, JP = noise_jp(J);
    const int NB = N + kBandBatch;
    const int g = a.first_global + r;
    double* zs = zA;    // [NB][JP] standard normals
    double* eps = zB;   // [NB][JP] noise (padding zeroed here)
    for (int idx = tid; idx < NB * JP; idx += BLOCK) {
        const int k = idx / JP, d = idx - k * JP;
        if (k >= N || d >= J) { zs[idx] = 0.0; eps[idx] = 0.0; }
    }
    {
        const int P = (N + 1) / 2;
        for (int idx = tid; idx < J * P; idx += BLOCK) {
            const int d = idx / P, p = idx - d * P;
            double z0, z1;
            normal_pair(a.seed, a.iteration, d, g, p, &z0, &z1);
            zs[(2 * p) * JP + d] = z0;
            if (2 * p + 1 < N) zs[(2 * p + 1) * JP + d] = z1;
        }
    }
}

// One 16-row tile of D = A * B on the fp64 matrix cores, k ascending from +0.0, for NG groups
// of 4 joint columns: A[i][k] = AT[k][i0 + i] (rows past N read column N - 1 and are
// discarded), B[k][j] = v[k * JP + 4 g + j] (LDS; zero rows past N, zero columns past J).
// v_mfma_f64_4x4x4_4b_f64 computes four 4 x 4 blocks b = lane bits 2-3: A_b[i][k] at lane
// 16 k + 4 b + i, B_b[k][j] at 16 k + 4 b + j, D_b[i][j] at 16 i + 4 b + j
// (tools/probes/mfma_f64_4x4_map.hip).  With block b = rows 4 b .. 4 b + 3 of the tile and B
// the same in every block, one instruction advances a 16 x 4 tile by 4 k, and it is a
// k-ascending fma chain (tools/probes/mfma_f64_4x4_probe.hip): D is the oracle's matvec_fma
// bit for bit.  The NG column groups share the A operand and are independent chains.
// Lane l ends with D[4 ((l >> 2) & 3) + (l >> 4)][4 g + (l & 3)] in acc[g].
template <int NG>
__device__ __forceinline__ void mfma_tile(__amdgpu_buffer_rsrc_t rsrc, int N, int i0, int kend, const double* v,
                                          int JP, int lane, double* acc)
{
    constexpr int S = 8 / NG;   // k steps per batch; four batches rotate, three ahead of the MFMAs
    const int lk = lane >> 4;
    // lane part of the address (column, row within the step) in the VGPR offset, the step's
    // rows in the scalar offset (a lane-dependent scalar offset would become a waterfall loop)
    const int ioff = (min(i0 + (lane & 15), N - 1) + lk * N) * (int)sizeof(double);
    const double* vb = v + lk * JP + (lane & 3);
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[g] = 0.0;
    const int nsteps = (kend + 3) >> 2;
    const int nb = (nsteps + S - 1) / S;
    struct Batch {
        double a[S], b[S][NG];
    };
    Batch R0, R1, R2, R3;
    auto load = [&](Batch& R, int bi) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k4 = 4 * min(bi * S + s, nsteps - 1);   // clamped: batches past the end re-read
            R.a[s] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, ioff, k4 * N * (int)sizeof(double), 0));
#pragma unroll
            for (int g = 0; g < NG; ++g) R.b[s][g] = vb[k4 * JP + 4 * g];
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto run = [&](const Batch& R, int bi) {
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (bi * S + s < nsteps)
#pragma unroll
                for (int g = 0; g < NG; ++g) acc[g] = __builtin_amdgcn_mfma_f64_4x4x4f64(R.a[s], R.b[s][g], acc[g], 0, 0, 0);
    };
    // whole ring rounds, then the remaining batches (no branch between a load and its use)
    load(R0, 0);
    load(R1, 1);
    load(R2, 2);
    int bi = 0;
    for (; bi + 4 <= nb; bi += 4) {
        load(R3, bi + 3); run(R0, bi);
        load(R0, bi + 4); run(R1, bi + 1);
        load(R1, bi + 5); run(R2, bi + 2);
        load(R2, bi + 6); run(R3, bi + 3);
    }
    const int rem = nb - bi;
    if (rem >= 1) run(R0, bi);
    if (rem >= 2) run(R1, bi + 1);
    if (rem >= 3) run(R2, bi + 2);
}

template <int BLOCK>
__device__ __forceinline__ void rollout_control(const NoiseArgs& a, size_t row, double* xs, double* cs, int tid,
                                                double* ctl = nullptr);

// DEFER: leave x in zA for wave_control (the phased rollout prices the row on the waves the FK
// program leaves idle) instead of rollout_control here
template <int BLOCK, int NG, bool DEFER = false>
__device__ __forceinline__ void rollout_project_ng(const NoiseArgs& a, int r, double* traj, double* zA, double* zB,
                                                   int tid)
{
    const int J = a.J, N = a.N, Nall = a.Nall, JP = noise_jp(J);
    const size_t row = (size_t)r * J * N;
    const double* zs = zA;
    double* eps = zB;
    __syncthreads();   // the normals are complete
    STAMP(7);

    constexpr int NW = BLOCK / 64;
    // the wave index through readfirstlane: the compiler then knows every tile quantity is
    // wave-uniform (scalar buffer offsets; a "divergent" one becomes a waterfall loop)
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int irow = 4 * ((lane >> 2) & 3) + (lane >> 4), jcol = lane & 3;   // lane's D element
    const int nti = (N + 15) >> 4;
    const int mat_bytes = (N + kMatPadRows) * N * (int)sizeof(double);
    const __amdgpu_buffer_rsrc_t rL = __builtin_amdgcn_make_buffer_rsrc((void*)a.LT, 0, mat_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rM = __builtin_amdgcn_make_buffer_rsrc((void*)a.MT, 0, mat_bytes, 0x00020000);
    // waypoint tiles in snake order over the waves (L z costs grow with the tile index);
    // a permutation of [0, nti): odd rounds run backwards over the tiles they have
    auto tile_of = [&](int n) {
        const int round = n / NW, pos = n % NW, cnt = min(NW, nti - round * NW);
        return round * NW + ((round & 1) ? cnt - 1 - pos : pos);
    };
    // eps = sigma_d * (0 + L z): L is lower triangular, tile ti needs rows k < 16 ti + 16
    for (int n = wv; n < nti; n += NW) {
        const int ti = tile_of(n);
        double acc[NG];
        mfma_tile<NG>(rL, N, 16 * ti, min(N, 16 * ti + 16), zs, JP, lane, acc);
        const int i = 16 * ti + irow;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int d = 4 * g + jcol;
            if (i < N && d < J) {
                const double e = a.sigma.v[d] * (0.0 + acc[g]);
                traj[d * N + i] = a.theta[(size_t)d * N + i] + e;
                eps[i * JP + d] = e;
            }
        }
    }
    __syncthreads();

    STAMP(8);
    // the rows to HBM, coalesced (lane over waypoints)
    for (int idx = tid; idx < J * N; idx += BLOCK) {
        const int d = idx / N, i = idx - d * N;
        a.noise[row + idx] = eps[i * JP + d];
        a.params[row + idx] = traj[idx];
    }
    double* xs = zA;   // z is dead
    // x = params + M eps
    for (int ti = wv; ti < nti; ti += NW) {
        double acc[NG];
        mfma_tile<NG>(rM, N, 16 * ti, N, eps, JP, lane, acc);
        const int i = 16 * ti + irow;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int d = 4 * g + jcol;
            if (i < N && d < J) xs[d * Nall + i + 6] = traj[d * N + i] + acc[g];
        }
    }
    if (!DEFER) rollout_control<BLOCK>(a, row, xs, zB, tid);   // eps is dead
}

// rollout_control for joint d by one wave, no block barrier (a wave's LDS accesses execute in
// program order): the padding, the 7-tap terms of joint d into cs, its control row to HBM.
// The same expressions as rollout_control.
__device__ __forceinline__ void wave_control(const NoiseArgs& a, size_t row, double* xs, double* cs, int d, int lane)
{
    const int N = a.N, Nall = a.Nall;
    double* x = xs + d * Nall;
    double* c = cs + d * Nall;
    if (lane < 12) x[lane < 6 ? lane : N + lane] = lane < 6 ? a.start[d] : a.goal[d];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int R = kCtlRun;
    const int nrun = (Nall + R - 1) / R;
    for (int item = lane; item < nrun; item += 64) {
        const int ii0 = item * R;
        double xw[R + 6];
#pragma unroll
        for (int q = 0; q < R + 6; ++q) xw[q] = x[min(max(ii0 - 3 + q, 0), Nall - 1)];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const int ii = ii0 + u;
            double call = 0.0;
#pragma unroll
            for (int rule = 0; rule < 3; ++rule) {
                const double wr = a.wr[rule];
                if (wr == 0.0) continue;   // adds +0.0 in the reference: exact to skip
                double sacc = 0.0;
#pragma unroll
                for (int q = 0; q < 7; ++q)
                    if (ii - 3 + q >= 0 && ii - 3 + q < Nall) sacc += a.dcoef[rule][q] * xw[u + q];
                call += wr * (sacc * sacc);
            }
            if (ii < Nall) c[ii] = call;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int t = lane; t < N; t += 64) a.control[row + (size_t)d * N + t] = control_cost(c, N, Nall, t);
}

// computeControlCosts of one row from xs = the free part of params + M eps at [d][6 + i]
// (written by the caller, not yet synchronised): the padding, the 7-tap terms into cs and the
// control row to HBM
template <int BLOCK>
__device__ __forceinline__ void rollout_control(const NoiseArgs& a, size_t row, double* xs, double* cs, int tid,
                                                double* ctl)
{
    double* out = ctl ? ctl : a.control;   // ctl: the extra rollout's row
    const int J = a.J, N = a.N, Nall = a.Nall;
    for (int idx = tid; idx < J * 12; idx += BLOCK) {
        const int d = idx / 12, k = idx - d * 12;
        xs[d * Nall + (k < 6 ? k : N + k)] = k < 6 ? a.start[d] : a.goal[d];
    }
    __syncthreads();

    STAMP(9);
    {
        // lane = (joint, run of kCtlRun consecutive padded indices): one 7-tap window read
        // serves the run; taps outside [0, Nall) are skipped as in control_term
        constexpr int R = kCtlRun;
        const int nrun = (Nall + R - 1) / R;
        for (int item = tid; item < J * nrun; item += BLOCK) {
            const int d = item / nrun, ii0 = (item - d * nrun) * R;
            const double* x = xs + d * Nall;
            double xw[R + 6];
#pragma unroll
            for (int q = 0; q < R + 6; ++q) xw[q] = x[min(max(ii0 - 3 + q, 0), Nall - 1)];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int ii = ii0 + u;
                double call = 0.0;
#pragma unroll
                for (int rule = 0; rule < 3; ++rule) {
                    const double wr = a.wr[rule];
                    if (wr == 0.0) continue;   // adds +0.0 in the reference: exact to skip
                    double sacc = 0.0;
#pragma unroll
                    for (int q = 0; q < 7; ++q)
                        if (ii - 3 + q >= 0 && ii - 3 + q < Nall) sacc += a.dcoef[rule][q] * xw[u + q];
                    call += wr * (sacc * sacc);
                }
                if (ii < Nall) cs[d * Nall + ii] = call;
            }
        }
    }
    STAMP(61);
    __syncthreads();
    STAMP(62);
    {
        constexpr int R = kCtlRun;
        const int nrun = (N + R - 1) / R;
        for (int item = tid; item < J * nrun; item += BLOCK) {
            const int d = item / nrun, t0 = (item - d * nrun) * R;
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (t0 + u < N) out[row + (size_t)d * N + t0 + u] = control_cost(cs + d * Nall, N, Nall, t0 + u);
        }
    }
    STAMP(63);
}

// One reuse candidate re-based on theta and priced (policy_improvement.cpp:208-224, then
// computeProjectedNoise :473-482 and computeControlCosts): params p = psrc (theta itself when
// psrc is null: the extra rollout), noise p - theta, x = p + M (p - theta) with M eps on the fp64
// matrix cores, then rollout_control; the rows to out_params / out_noise / out_ctl.  The copy,
// roundings and order of k_noise_rows<REUSE>.  The whole block calls it; lds:
// (N + kBandBatch) JP + 2 J Nall + J N doubles.
template <int BLOCK, int NG>
__device__ __forceinline__ void price_candidate(const NoiseArgs& a, const double* psrc, double* out_params,
                                                double* out_noise, double* out_ctl, double* lds, int tid)
{
    const int J = a.J, N = a.N, Nall = a.Nall, JP = noise_jp(J), NB = N + kBandBatch, JN = J * N;
    double* eps = lds;            // [NB][JP], zero rows past N and zero columns past J
    double* xs = eps + NB * JP;   // [J][Nall]
    double* cs = xs + J * Nall;   // [J][Nall]
    double* prm = cs + J * Nall;  // [J][N]
    const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
    constexpr int kLoads = 2048 / BLOCK;
    for (int i0 = 0; i0 < JN; i0 += kLoads * BLOCK) {
        double vt[kLoads], vp[kLoads];
#pragma unroll
        for (int u = 0; u < kLoads; ++u) {
            if (i0 + wbase + u * BLOCK < JN) {   // wave-uniform: only the live loads
                const int idx = min(i0 + tid + u * BLOCK, JN - 1);
                vt[u] = a.theta[idx];
                vp[u] = psrc ? psrc[idx] : vt[u];
            }
        }
#pragma unroll
        for (int u = 0; u < kLoads; ++u) {
            const int idx = i0 + tid + u * BLOCK;
            if (idx < JN) {
                const int d = idx / N, k = idx - d * N;
                const double e = vp[u] - vt[u];
                out_params[idx] = vp[u];
                out_noise[idx] = e;
                eps[k * JP + d] = e;
                prm[idx] = vp[u];
            }
        }
    }
    for (int idx = tid; idx < NB * JP; idx += BLOCK) {
        const int k = idx / JP, d = idx - k * JP;
        if (k >= N || d >= J) eps[idx] = 0.0;
    }
    __syncthreads();
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int irow = 4 * ((lane >> 2) & 3) + (lane >> 4), jcol = lane & 3;
    const int nti = (N + 15) >> 4;
    const int mat_bytes = (N + kMatPadRows) * N * (int)sizeof(double);
    const __amdgpu_buffer_rsrc_t rM = __builtin_amdgcn_make_buffer_rsrc((void*)a.MT, 0, mat_bytes, 0x00020000);
    for (int ti = wv; ti < nti; ti += BLOCK / 64) {
        double acc[NG];
        mfma_tile<NG>(rM, N, 16 * ti, N, eps, JP, lane, acc);
        const int i = 16 * ti + irow;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int d = 4 * g + jcol;
            if (i < N && d < J) xs[d * Nall + i + 6] = prm[d * N + i] + acc[g];
        }
    }
    rollout_control<BLOCK>(a, 0, xs, cs, tid, out_ctl);
}

// k_pregen's row, first half: normals (rollout_normals, already issued) and
// eps = sigma_d (0 + L z), the same tiles and roundings as rollout_project_ng, written to
// a.pre_eps and (layout [i][JP], for pregen_meps_ng) to the LDS buffer zB.  (M eps as a
// separate half in the update launch was measured slower: 10.3 us update vs 5.1.)
template <int BLOCK, int NG>
__device__ __forceinline__ void pregen_eps_ng(const NoiseArgs& a, int r, double* zA, double* zB, int tid)
{
    const int J = a.J, N = a.N, JP = noise_jp(J);
    const size_t row = (size_t)r * J * N;
    const double* zs = zA;
    double* eps = zB;
    __syncthreads();   // the normals are complete
    constexpr int NW = BLOCK / 64;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int irow = 4 * ((lane >> 2) & 3) + (lane >> 4), jcol = lane & 3;
    const int nti = (N + 15) >> 4;
    const int mat_bytes = (N + kMatPadRows) * N * (int)sizeof(double);
    const __amdgpu_buffer_rsrc_t rL = __builtin_amdgcn_make_buffer_rsrc((void*)a.LT, 0, mat_bytes, 0x00020000);
    auto tile_of = [&](int n) {
        const int round = n / NW, pos = n % NW, cnt = min(NW, nti - round * NW);
        return round * NW + ((round & 1) ? cnt - 1 - pos : pos);
    };
    for (int n = wv; n < nti; n += NW) {
        const int ti = tile_of(n);
        double acc[NG];
        mfma_tile<NG>(rL, N, 16 * ti, min(N, 16 * ti + 16), zs, JP, lane, acc);
        const int i = 16 * ti + irow;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int d = 4 * g + jcol;
            if (i < N && d < J) {
                const double e = a.sigma.v[d] * (0.0 + acc[g]);
                eps[i * JP + d] = e;
                a.pre_eps[row + (size_t)d * N + i] = e;
            }
        }
    }
}

// second half: M eps from eps in LDS ([i][JP] with zero rows N .. N + kBandBatch and zero
// columns J .. JP, as rollout_normals leaves them) to a.pre_meps
template <int BLOCK, int NG>
__device__ __forceinline__ void pregen_meps_ng(const NoiseArgs& a, int r, const double* eps, int tid)
{
    const int J = a.J, N = a.N, JP = noise_jp(J);
    const size_t row = (size_t)r * J * N;
    __syncthreads();   // eps is complete
    constexpr int NW = BLOCK / 64;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int irow = 4 * ((lane >> 2) & 3) + (lane >> 4), jcol = lane & 3;
    const int nti = (N + 15) >> 4;
    const int mat_bytes = (N + kMatPadRows) * N * (int)sizeof(double);
    const __amdgpu_buffer_rsrc_t rM = __builtin_amdgcn_make_buffer_rsrc((void*)a.MT, 0, mat_bytes, 0x00020000);
    for (int ti = wv; ti < nti; ti += NW) {
        double acc[NG];
        mfma_tile<NG>(rM, N, 16 * ti, N, eps, JP, lane, acc);
        const int i = 16 * ti + irow;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int d = 4 * g + jcol;
            if (i < N && d < J) a.pre_meps[row + (size_t)d * N + i] = acc[g];
        }
    }
}

// one lane's share of a 4 BLOCK chunk of k_pregen's row (eps, M eps, theta)
struct PreChunk {
    double e[4], mp[4], th[4];
};

// MP: also M eps (not needed when the row is priced elsewhere)
template <int BLOCK, bool MP = true>
__device__ __forceinline__ void pre_chunk_load(const NoiseArgs& a, int r, int idx0, int tid, PreChunk& c)
{
    const int JN = a.J * a.N;
    const size_t row = (size_t)r * JN;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int idx = min(idx0 + tid + u * BLOCK, JN - 1);
        c.e[u] = a.pre_eps[row + idx];
        if (MP) c.mp[u] = a.pre_meps[row + idx];
        c.th[u] = a.theta[idx];
    }
}

// the rollout kernel's row from k_pregen's eps and M eps: params = theta + eps into traj (LDS)
// and HBM, the noise row, x = params + M eps, then the control costs (rollout_control).  first:
// chunk 0, loaded by the caller (its loads in flight with the table image's)
// XS = false: the row is priced by another workgroup (ctl_by_pre), which also writes its noise /
// params rows: no x, no M eps, no row stores.  lead: the launch's first rollout (keeps theta_gen)
template <int BLOCK, bool DEFER = false, bool XS = true>
__device__ __forceinline__ void rollout_from_pre(const NoiseArgs& a, int r, bool lead, double* traj, double* zA,
                                                 double* zB, int tid, const PreChunk& first)
{
    const int J = a.J, N = a.N, Nall = a.Nall, JN = J * N;
    const size_t row = (size_t)r * JN;
    double* xs = zA;
    for (int idx0 = 0; idx0 < JN; idx0 += 4 * BLOCK) {
        PreChunk c;
        if (idx0 == 0) c = first;
        else pre_chunk_load<BLOCK, XS>(a, r, idx0, tid, c);
        const double* e = c.e;
        const double* mp = c.mp;
        const double* th = c.th;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = idx0 + tid + u * BLOCK;
            if (idx < JN) {
                const int d = idx / N, i = idx - d * N;
                const double p = th[u] + e[u];
                traj[idx] = p;
                if (!a.rows_in_pre) {
                    if (XS) {
                        a.noise[row + idx] = e[u];
                        a.params[row + idx] = p;
                    }
                } else if (lead) {
                    a.theta_gen[idx] = th[u];
                }
                if (XS) xs[d * Nall + i + 6] = p + mp[u];
            }
        }
    }
    if (XS && !DEFER) rollout_control<BLOCK>(a, row, xs, zB, tid);
}

// computeControlCosts of row r from k_pregen's eps and M eps (covariant_trajectory_policy.cpp:
// 228-255 via policy_improvement.cpp:292-299): x = (theta + eps) + M eps, the expressions of
// rollout_from_pre, then rollout_control into a.control; the noise / params rows too unless they
// stay in the pregen buffer.  Run by the rollout launch's pregen block r, so the rollout workgroup
// of row r leaves the pricing out of its critical path.
template <int BLOCK>
__device__ __forceinline__ void pre_row_control(const NoiseArgs& a, int r, double* xs, double* cs, int tid)
{
    const int J = a.J, N = a.N, Nall = a.Nall, JN = J * N;
    for (int idx0 = 0; idx0 < JN; idx0 += 4 * BLOCK) {
        PreChunk c;
        pre_chunk_load<BLOCK>(a, r, idx0, tid, c);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = idx0 + tid + u * BLOCK;
            if (idx < JN) {
                const int d = idx / N, i = idx - d * N;
                const double p = c.th[u] + c.e[u];
                xs[d * Nall + i + 6] = p + c.mp[u];
                if (!a.rows_in_pre) {
                    a.noise[(size_t)r * JN + idx] = c.e[u];
                    a.params[(size_t)r * JN + idx] = p;
                }
            }
        }
    }
    rollout_control<BLOCK>(a, (size_t)r * JN, xs, cs, tid, nullptr);
}

// Rollout::getCost (policy_improvement.cpp:149-156) of one reuse candidate in k_reuse's order:
// its state row and J control rows staged in LDS (stage: (J + 1) N doubles) with every load in
// flight, one t-chain per row (x = v[0], then x += v[t] ascending), then part[0] + part[1] + ...
// + part[J]; NaN as +inf (the ranks stay a permutation).  The whole block calls it; thread 0
// gets the total.
template <int BLOCK>
__device__ __forceinline__ double candidate_total(const double* state, const double* control, int J, int N,
                                                  double* stage, int tid)
{
    __shared__ double part[kMaxJoints + 1];
    const int L = J + 1, P = L * N;
    for (int i0 = tid; i0 - tid < P; i0 += 4 * BLOCK) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = min(i0 + u * BLOCK, P - 1);
            v[u] = idx < N ? state[idx] : control[idx - N];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * BLOCK < P) stage[i0 + u * BLOCK] = v[u];
    }
    __syncthreads();
    if (tid < L) {
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
    double s2 = 0.0;
    if (tid == 0) {
        s2 = part[0];
        for (int d = 0; d < J; ++d) s2 += part[1 + d];
        if (s2 != s2) s2 = __builtin_inf();
    }
    return s2;
}

// the engine runs the fused phase for J <= 16 (at most four groups of 4 joint columns)
template <int BLOCK, bool DEFER = false>
__device__ __forceinline__ void rollout_project(const NoiseArgs& a, int r, double* traj, double* zA, double* zB,
                                                int tid)
{
    if (a.J <= 8) rollout_project_ng<BLOCK, 2, DEFER>(a, r, traj, zA, zB, tid);
    else rollout_project_ng<BLOCK, 4, DEFER>(a, r, traj, zA, zB, tid);
}

}  // namespace stomp
