// k_noise.hip -- noise sampling, projection and control cost, fused per (rollout tile, joint).
//
// Generated rows are normally produced inside the rollout kernel (noise_device.h); this
// kernel serves the reused rows (projection + control of re-based noise), the extra
// noiseless rollout's control cost, and N > 128 where the fused phase does not apply.
//
//   eps = sigma_d * (0 + L z)          MultivariateGaussian::sample (multivariate_gaussian.h:88-94)
//                                      via generateRollouts (policy_improvement.cpp:228-236)
//   params = theta + eps               policy_improvement.cpp:234
//   nproj = M eps                      computeProjectedNoise (policy_improvement.cpp:473-482)
//   control = sum_i w_i (D_i x)^2      computeControlCosts (covariant_trajectory_policy.cpp:228-255),
//                                      x = padded (params + nproj), 7-tap stencils instead of dense D_i
//
// One workgroup owns RT rollouts of one joint; lane i owns time step i and keeps RT
// accumulators.  L^T / M^T are read straight from L2 (lane i reads column i, so a wave's
// load is 512 contiguous bytes) eight k at a time so eight loads are in flight per lane;
// z and eps sit in LDS as [k][RT] so one k costs RT/2 broadcast ds_read_b128.  Sums run
// over k in ascending order, one rounding per operation (the oracle's contract); the
// triangular product stops at k = i exactly like the oracle's loop.
#include "noise_device.h"
#include "stamps.h"

namespace stomp {

template <int BLOCK, int RT>
__global__ __launch_bounds__(BLOCK) void k_noise(NoiseArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (a.stop && *a.stop) return;
    const int N = a.N, Nall = a.Nall, J = a.J;
    const int NB = N + kBandBatch;   // rows incl. the zero padding the band products read
    double* zs = lds;              // NB*RT  [k][rr]
    double* eps = zs + RT * NB;    // NB*RT  [k][rr]
    double* xs = eps + RT * NB;    // RT*Nall
    double* cs = xs + RT * Nall;   // RT*Nall
    const int d = blockIdx.y;
    const int r0 = a.row_begin + blockIdx.x * RT;
    const int tid = threadIdx.x;
    const int i = tid;
    const double sig = a.sigma.v[d];
    STAMP(0);

    for (int idx = tid; idx < kBandBatch * RT; idx += BLOCK) {
        zs[N * RT + idx] = 0.0;
        eps[N * RT + idx] = 0.0;
    }
    bool gen[RT];
    bool any_gen = false;
#pragma unroll
    for (int rr = 0; rr < RT; ++rr) {
        const int r = r0 + rr;
        const int g = a.first_global + r;
        gen[rr] = (r < a.K_loc) && !a.zero_noise && g < a.K_gen_global;
        any_gen |= gen[rr];
    }
    // standard normals of all generated rows, (row, pair) items spread over the whole block
    {
        const int P = (N + 1) / 2;
        for (int idx = tid; idx < RT * P; idx += BLOCK) {
            const int rr = idx / P, p = idx - rr * P;
            const int r = r0 + rr, g = a.first_global + r;
            if (!((r < a.K_loc) && !a.zero_noise && g < a.K_gen_global)) continue;
            double z0, z1;
            normal_pair(a.seed, a.iteration, d, g, p, &z0, &z1);
            zs[(2 * p) * RT + rr] = z0;
            if (2 * p + 1 < N) zs[(2 * p + 1) * RT + rr] = z1;
        }
    }
#pragma unroll
    for (int rr = 0; rr < RT; ++rr) {
        const int r = r0 + rr;
        if (gen[rr]) continue;
        if (r >= a.K_loc) {
            for (int t = tid; t < N; t += BLOCK) { zs[t * RT + rr] = 0.0; eps[t * RT + rr] = 0.0; }
        } else if (a.zero_noise) {
            // addExtraRollouts: noise = parameters - theta with parameters == theta, +0.0 exactly
            for (int t = tid; t < N; t += BLOCK) {
                eps[t * RT + rr] = 0.0;
                a.noise[((size_t)r * J + d) * N + t] = 0.0;
            }
        } else {
            // reused rollout: noise re-based on the current theta by the reuse kernel
            for (int t = tid; t < N; t += BLOCK) eps[t * RT + rr] = a.noise[((size_t)r * J + d) * N + t];
        }
    }
    __syncthreads();
    STAMP(1);

    // Loops run to a wave-uniform bound with clamped, unconditional loads so a lane's eight
    // loads are in flight together.  The extra terms are exact no-ops: L^T is exactly zero
    // above the diagonal (k > i) and past N the multiplier is forced to 0.0, and an
    // accumulator that starts at +0.0 never becomes -0.0, so adding +-0.0 leaves it unchanged.
    const int wave_end = min(N, __builtin_amdgcn_readfirstlane(tid & ~63) + 64);
    if (any_gen && i < N) {
        double acc[RT];
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) acc[rr] = 0.0;
        band_product<RT>(a.LT, N, i, wave_end, zs, RT, acc);
        const double th = a.theta[(size_t)d * N + i];
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            if (!gen[rr]) continue;
            const int r = r0 + rr;
            const double e = sig * (0.0 + acc[rr]);
            a.noise[((size_t)r * J + d) * N + i] = e;
            a.params[((size_t)r * J + d) * N + i] = th + e;
            eps[i * RT + rr] = e;
        }
    }
    __syncthreads();
    STAMP(2);

    if (i < N) {
        double acc[RT];
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) acc[rr] = 0.0;
        band_product<RT>(a.MT, N, i, N, eps, RT, acc);
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            const int r = r0 + rr;
            double p = 0.0;
            if (r < a.K_loc) {
                if (a.zero_noise == 2) {   // the extra rollout of theta: params = theta, copied here
                    p = a.theta[(size_t)d * N + i];
                    a.params[((size_t)r * J + d) * N + i] = p;
                } else {
                    p = a.params[((size_t)r * J + d) * N + i];
                }
            }
            xs[rr * Nall + i + 6] = p + acc[rr];
        }
    }
    STAMP(3);
    for (int idx = tid; idx < RT * 12; idx += BLOCK) {
        const int rr = idx / 12, row = idx % 12;
        xs[rr * Nall + (row < 6 ? row : N + row)] = row < 6 ? a.start[d] : a.goal[d];
    }
    __syncthreads();

    for (int ii = tid; ii < Nall; ii += BLOCK) {
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) cs[rr * Nall + ii] = control_term(a, xs + rr * Nall, Nall, ii);
    }
    __syncthreads();
    STAMP(4);

    if (i < N) {
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            const int r = r0 + rr;
            if (r >= a.K_loc) continue;
            const double o = control_cost(cs + rr * Nall, N, Nall, i);
            a.control[((size_t)r * J + d) * N + i] = o;
        }
    }
    STAMP(5);
}

// k_reuse's choice for reused row rr (policy_improvement.cpp:176-225) in two dependent memory
// round trips: (1) the K totals and the extra rollout's J + 1 cost rows (its total's stage), with
// the caller's independent loads (`independent`) in flight beside them; (2) each wave ranks the K
// previous rows by their totals alone (one wave per 64: no barrier before the caller's loads of
// the rows of K-rank rr and rr - 1, `dependent(A, B)`), while wave 0 runs the extra rollout's
// t-chains.  Inserting the extra rollout (index -1: ahead of equal totals) into the K-order moves
// rank rr to K-rank rr (its total < the extra's), to the extra, or to K-rank rr - 1 (its total >=
// the extra's): k_reuse's (cost, index) order, decided from two compares.  Returns the candidate
// (K: the extra rollout).  LDS: costs [K rounded up to 8], stage [(J + 1) N].
constexpr int kReuseRowsMax = 1024;   // candidates the reused rows' kernels rank themselves

template <int BLOCK, class Independent, class Dependent>
__device__ __forceinline__ int reuse_choice(const ReuseArgs& ra, int J, int N, int rr, double* costs, double* stage,
                                            int tid, Independent&& independent, Dependent&& dependent)
{
    constexpr int kCostLoads = (kReuseRowsMax + BLOCK - 1) / BLOCK;
    const int K = ra.K, L = J + 1, P = L * N;
    const bool wx = ra.with_extra;
    __shared__ double part[kMaxJoints + 1];
    __shared__ int sel[2];
    double cv[kCostLoads];
    // a wave issues only the loads of its own live elements (wave-uniform skips: a row's JN
    // elements are ~1.4 per lane at cfg1, and each clamped duplicate load still costs the CU's
    // address and data path)
    const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
#pragma unroll
    for (int u = 0; u < kCostLoads; ++u)
        if (wbase + u * BLOCK < K) cv[u] = ra.costs[min(tid + u * BLOCK, K - 1)];
    independent();
    if (wx) {
        for (int i0 = tid; i0 - tid < P; i0 += 4 * BLOCK) {   // candidate_total's stage
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int idx = min(i0 + u * BLOCK, P - 1);
                if (wbase + u * BLOCK < P - (i0 - tid)) v[u] = idx < N ? ra.x_state[idx] : ra.x_control[idx - N];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * BLOCK < P) stage[i0 + u * BLOCK] = v[u];
        }
    }
    // the totals, then +inf up to a multiple of 8 (ranks past K count nothing: inf is below no
    // total, and equals only an inf total of a lower index)
#pragma unroll
    for (int u = 0; u < kCostLoads; ++u) {
        const int c = tid + u * BLOCK;
        if (c < K) costs[c] = cv[u];
        else if (c < ((K + 7) & ~7)) costs[c] = __builtin_inf();
    }
    __syncthreads();
    STAMP(6);
    // K-rank of candidate c: (total, index) ascending among the K previous rows
    auto k_rank = [&](int c) {
        const double cc = costs[c];
        int rank = 0;
        for (int c0 = 0; c0 < K; c0 += 8) {
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = costs[c0 + u];
#pragma unroll
            for (int u = 0; u < 8; ++u)   // branch-free
                rank += (int)((x[u] < cc) | ((x[u] == cc) & (c0 + u < c)));
        }
        return rank;
    };
    int selA, selB;
    if (K <= 64) {   // every wave ranks all K itself: no barrier before the row loads
        const int lane = tid & 63;
        const int rank = lane < K ? k_rank(lane) : -2;
        const unsigned long long ma = __ballot(rank == rr), mb = __ballot(rank == rr - 1);
        selA = __builtin_amdgcn_readfirstlane(__ffsll((long long)ma) - 1);
        selB = rr > 0 ? __builtin_amdgcn_readfirstlane(__ffsll((long long)mb) - 1) : selA;
    } else {
        for (int c = tid; c < K; c += BLOCK) {
            const int rank = k_rank(c);
            if (rank == rr) sel[0] = c;       // ranks are a permutation: one writer each
            if (rank == rr - 1) sel[1] = c;
        }
        __syncthreads();
        selA = sel[0];
        selB = rr > 0 ? sel[1] : selA;
    }
    STAMP(10);
    dependent(selA, selB);
    STAMP(11);
    if (wx && tid < L) {
        // Rollout::getCost's t-chain of the extra rollout's row tid: x = v[0], then x += v[t]
        // ascending (candidate_total's order)
        const double* v = stage + (size_t)tid * N;
        double x = v[0];
        int t = 1;
        for (; t + 16 <= N; t += 16) {
            double b[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) b[u] = v[t + u];
#pragma unroll
            for (int u = 0; u < 16; ++u) x += b[u];
        }
        for (; t < N; ++t) x += v[t];
        part[tid] = x;
    }
    STAMP(12);
    __syncthreads();
    STAMP(7);
    int src = selA;
    if (wx) {
        double xt = part[0];
        for (int d = 0; d < J; ++d) xt += part[1 + d];
        if (xt != xt) xt = __builtin_inf();
        if (!(costs[selA] < xt)) src = (rr > 0 && costs[selB] >= xt) ? selB : K;
    }
    return src;
}

// The reused rows of an iteration (policy_improvement.cpp:208-224: noise re-based on theta),
// then computeProjectedNoise (:473-482) and computeControlCosts: one workgroup per row and all its
// joints (BLOCK / 64 waves >= the row's 16-waypoint tiles: one round), M eps on the fp64 matrix
// cores (mfma_tile: the k-ascending fma chains of the rollout kernel's noise phase, band_product's
// sums bit for bit), x = params + M eps, then rollout_control (control_term / control_cost's
// expressions).  REUSE: the row is not copied yet; the workgroup of reused row rr finds the
// candidate of rank rr in k_reuse's (cost, index) order (the extra rollout at -1), writes its
// params, the noise params - theta and its state row (k_reuse's copy), then prices it from
// registers and LDS.  The K previous rows' totals come from the rollout launch's totals blocks;
// the extra rollout's is made here (candidate_total's stage and sums), overlapped with the loads
// of the two rows rank rr can be besides the extra rollout's (see the prologue).
template <int BLOCK, int NG, bool REUSE>
__global__ __launch_bounds__(BLOCK) void k_noise_rows(NoiseArgs a, ReuseArgs ra)
{
    extern __shared__ __attribute__((aligned(16))) double lds_nr[];
    if (a.stop && *a.stop) return;
    const int J = a.J, N = a.N, Nall = a.Nall, JP = noise_jp(J), NB = N + kBandBatch;
    const int r = a.row_begin + blockIdx.x;
    const size_t row = (size_t)r * J * N;
    double* eps = lds_nr;              // [NB][JP], zero rows past N and zero columns past J
    double* xs = eps + NB * JP;        // [J][Nall]
    double* cs = xs + J * Nall;        // [J][Nall]
    double* prm = cs + J * Nall;       // [J][N] the params row
    const int tid = threadIdx.x;
    STAMP(0);
    const double* psrc = a.params + row;
    const double* nsrc = a.noise + row;
    // the noise and params rows: every load of the workgroup in flight at once (coalesced)
    constexpr int kRowLoads = 4096 / BLOCK;   // the row in few passes
    const int JN = J * N;
    int first = tid;                          // the generic passes start here
    if constexpr (REUSE) {
        // the choice with theta and the extra rollout's rows loaded beside the totals, the two
        // K-ranked candidates' rows beside the t-chains (reuse_choice)
        const int K = ra.K, rr = r - ra.K_gen;
        const bool wx = ra.with_extra;
        double* costs = prm + JN;   // [K + 7] the previous rows' totals (the rollout launch's), inf
        double th[kRowLoads], px[kRowLoads], pa[kRowLoads], pb[kRowLoads];
        double sx = 0.0, sa, sb;
        const int ti = min(tid, N - 1);
        const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
        auto live = [&](int u) { return wbase + u * BLOCK < JN; };
        int selA, selB;
        const int src = reuse_choice<BLOCK>(
            ra, J, N, rr, costs, xs, tid,   // stage: xs, cs (dead until the projection)
            [&]() {
#pragma unroll
                for (int u = 0; u < kRowLoads; ++u)
                    if (live(u)) th[u] = a.theta[min(tid + u * BLOCK, JN - 1)];
                if (wx) {
#pragma unroll
                    for (int u = 0; u < kRowLoads; ++u)
                        if (live(u)) px[u] = ra.x_params[min(tid + u * BLOCK, JN - 1)];
                    sx = ra.x_state[ti];
                }
            },
            [&](int A, int B) {
                selA = A;
                selB = B;
                const double* rA = ra.src_params + (size_t)A * JN;
                const double* rB = ra.src_params + (size_t)B * JN;
#pragma unroll
                for (int u = 0; u < kRowLoads; ++u) {
                    const int idx = min(tid + u * BLOCK, JN - 1);
                    if (live(u)) {
                        pa[u] = rA[idx];
                        pb[u] = rB[idx];
                    }
                }
                sa = ra.src_state[(size_t)A * N + ti];
                sb = ra.src_state[(size_t)B * N + ti];
            });
        const int pick = src == selA ? 0 : (src == selB ? 1 : 2);
        if (tid < N) ra.state[(size_t)r * N + tid] = pick == 0 ? sa : (pick == 1 ? sb : sx);
#pragma unroll
        for (int u = 0; u < kRowLoads; ++u) {
            const int idx = tid + u * BLOCK;
            if (idx < JN) {
                const int d = idx / N, k = idx - d * N;
                const double p = pick == 0 ? pa[u] : (pick == 1 ? pb[u] : px[u]);
                const double e = p - th[u];   // k_reuse's copy: params, noise = params - theta
                a.params[row + idx] = p;
                a.noise[row + idx] = e;
                eps[k * JP + d] = e;
                prm[idx] = p;
            }
        }
        psrc = src < K ? ra.src_params + (size_t)src * JN : ra.x_params;
        const double* ssrc = src < K ? ra.src_state + (size_t)src * N : ra.x_state;
        for (int i = tid + BLOCK; i < N; i += BLOCK) ra.state[(size_t)r * N + i] = ssrc[i];
        first = tid + kRowLoads * BLOCK;
    }
    for (int i0 = first; i0 - tid < JN; i0 += kRowLoads * BLOCK) {
        double ve[kRowLoads], vp[kRowLoads];
#pragma unroll
        for (int u = 0; u < kRowLoads; ++u) {
            const int idx = min(i0 + u * BLOCK, JN - 1);
            vp[u] = psrc[idx];
            ve[u] = REUSE ? a.theta[idx] : nsrc[idx];
        }
#pragma unroll
        for (int u = 0; u < kRowLoads; ++u) {
            const int idx = i0 + u * BLOCK;
            if (idx < JN) {
                const int d = idx / N, k = idx - d * N;
                double e = ve[u];
                if constexpr (REUSE) {
                    e = vp[u] - ve[u];
                    a.params[row + idx] = vp[u];
                    a.noise[row + idx] = e;
                }
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
    STAMP(1);
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
    STAMP(2);
    rollout_control<BLOCK>(a, row, xs, cs, tid);
    STAMP(5);
}


// The reuse step when the rollout launch priced every candidate ahead (CostArgs::spec_*,
// price_candidate: candidate c's row re-based on theta, M eps and control costs; row K the extra
// rollout): the workgroup of reused row rr makes the choice (reuse_choice) with the extra
// rollout's priced rows loaded beside the totals and the two K-ranked candidates' priced rows
// beside the t-chains, then writes the chosen candidate's params, noise, control and state rows
// (k_noise_rows<REUSE>'s rows, computed ahead by the same expressions).
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_reuse_pick(NoiseArgs a, ReuseArgs ra)
{
    extern __shared__ __attribute__((aligned(16))) double lds_rp[];
    if (a.stop && *a.stop) return;
    const int J = a.J, N = a.N, JN = J * N, K = ra.K;
    const int r = a.row_begin + blockIdx.x, rr = r - ra.K_gen;
    const size_t row = (size_t)r * JN;
    const int tid = threadIdx.x;
    STAMP(0);
    double* costs = lds_rp;                      // [K rounded up to 8]
    double* stage = costs + ((K + 7) & ~7);      // [J + 1][N]
    constexpr int kL = 2048 / BLOCK;             // the rows' first pass in registers
    double xp[kL], xn[kL], xc[kL], ap[kL], an[kL], ac[kL], bp[kL], bn[kL], bc[kL];
    double sx = 0.0, sa, sb;
    const int ti = min(tid, N - 1);
    const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
    auto live = [&](int u) { return wbase + u * BLOCK < JN; };
    const size_t xo = (size_t)K * JN;
    int selA, selB;
    const int src = reuse_choice<BLOCK>(
        ra, J, N, rr, costs, stage, tid,
        [&]() {
            if (ra.with_extra) {
#pragma unroll
                for (int u = 0; u < kL; ++u) {
                    const size_t idx = xo + min(tid + u * BLOCK, JN - 1);
                    if (live(u)) {
                        xp[u] = ra.spec_params[idx];
                        xn[u] = ra.spec_noise[idx];
                        xc[u] = ra.spec_ctl[idx];
                    }
                }
                sx = ra.x_state[ti];
            }
        },
        [&](int A, int B) {
            selA = A;
            selB = B;
            const size_t oa = (size_t)A * JN, ob = (size_t)B * JN;
#pragma unroll
            for (int u = 0; u < kL; ++u) {
                const int idx = min(tid + u * BLOCK, JN - 1);
                if (live(u)) {
                    ap[u] = ra.spec_params[oa + idx];
                    an[u] = ra.spec_noise[oa + idx];
                    ac[u] = ra.spec_ctl[oa + idx];
                    bp[u] = ra.spec_params[ob + idx];
                    bn[u] = ra.spec_noise[ob + idx];
                    bc[u] = ra.spec_ctl[ob + idx];
                }
            }
            sa = ra.src_state[(size_t)A * N + ti];
            sb = ra.src_state[(size_t)B * N + ti];
        });
    const int pick = src == selA ? 0 : (src == selB ? 1 : 2);
    if (tid < N) ra.state[(size_t)r * N + tid] = pick == 0 ? sa : (pick == 1 ? sb : sx);
#pragma unroll
    for (int u = 0; u < kL; ++u) {
        const int idx = tid + u * BLOCK;
        if (idx < JN) {
            a.params[row + idx] = pick == 0 ? ap[u] : (pick == 1 ? bp[u] : xp[u]);
            a.noise[row + idx] = pick == 0 ? an[u] : (pick == 1 ? bn[u] : xn[u]);
            a.control[row + idx] = pick == 0 ? ac[u] : (pick == 1 ? bc[u] : xc[u]);
        }
    }
    // rows longer than the register pass, and state rows longer than the block: copied
    const size_t os = (size_t)src * JN;
    for (int idx = tid + kL * BLOCK; idx < JN; idx += BLOCK) {
        a.params[row + idx] = ra.spec_params[os + idx];
        a.noise[row + idx] = ra.spec_noise[os + idx];
        a.control[row + idx] = ra.spec_ctl[os + idx];
    }
    const double* ssrc = src < K ? ra.src_state + (size_t)src * N : ra.x_state;
    for (int i = tid + BLOCK; i < N; i += BLOCK) ra.state[(size_t)r * N + i] = ssrc[i];
    STAMP(5);
}

namespace {

size_t noise_rows_lds(const NoiseArgs& a, int n)
{
    return ((size_t)(a.N + kBandBatch) * noise_jp(a.J) + 2 * (size_t)a.J * a.Nall + (size_t)a.J * a.N + (size_t)n) *
           sizeof(double);
}

template <int BLOCK, int NG, bool REUSE>
void launch_noise_rows_t(const NoiseArgs& a, const ReuseArgs& ra, int rows, size_t lds, hipStream_t s)
{
    if (lds > 64 * 1024) lds_opt_in((const void*)k_noise_rows<BLOCK, NG, REUSE>, lds);
    hipLaunchKernelGGL((k_noise_rows<BLOCK, NG, REUSE>), dim3(rows), dim3(BLOCK), lds, s, a, ra);
}

template <bool REUSE>
void launch_noise_rows(const NoiseArgs& a, const ReuseArgs& ra, int rows, size_t lds, hipStream_t s)
{
    // one wave per 16-waypoint tile of the projection (N <= 128: 8 waves)
    if (a.N <= 128) {
        if (a.J <= 2 * kNoiseJT) launch_noise_rows_t<512, 2, REUSE>(a, ra, rows, lds, s);
        else launch_noise_rows_t<512, 4, REUSE>(a, ra, rows, lds, s);
    } else {
        if (a.J <= 2 * kNoiseJT) launch_noise_rows_t<1024, 2, REUSE>(a, ra, rows, lds, s);
        else launch_noise_rows_t<1024, 4, REUSE>(a, ra, rows, lds, s);
    }
}
}  // namespace

bool launch_reuse_rows_ok(const NoiseArgs& a, int K, int Kr)
{
    return !a.zero_noise && a.first_global == 0 && a.row_begin >= a.K_gen_global && a.K_loc - a.row_begin == Kr &&
           a.J <= 4 * kNoiseJT && K + 1 <= kReuseRowsMax && noise_rows_lds(a, K + 8) <= kRolloutLdsMax;
}

void launch_reuse_rows(const NoiseArgs& a, const ReuseArgs& ra, hipStream_t s)
{
    const int rows = a.K_loc - a.row_begin;
    if (rows <= 0) return;
    launch_noise_rows<true>(a, ra, rows, noise_rows_lds(a, ra.K + 8), s);   // the totals + inf padding
}

size_t price_candidate_lds_bytes(int J, int N)
{
    return ((size_t)(N + kBandBatch) * noise_jp(J) + 2 * (size_t)J * (N + 12) + (size_t)J * N) * sizeof(double);
}

namespace {
size_t reuse_pick_lds(const NoiseArgs& a, int K)
{
    return ((size_t)((K + 7) & ~7) + (size_t)(a.J + 1) * a.N) * sizeof(double);
}
}  // namespace

bool launch_reuse_pick_ok(const NoiseArgs& a, int K, int Kr)
{
    return launch_reuse_rows_ok(a, K, Kr) && price_candidate_lds_bytes(a.J, a.N) <= kRolloutLdsMax &&
           reuse_pick_lds(a, K) <= 64 * 1024;
}

void launch_reuse_pick(const NoiseArgs& a, const ReuseArgs& ra, hipStream_t s)
{
    const int rows = a.K_loc - a.row_begin;
    if (rows <= 0) return;
    hipLaunchKernelGGL(k_reuse_pick<512>, dim3(rows), dim3(512), reuse_pick_lds(a, ra.K), s, a, ra);
}

STOMP_STAMP_ACCESSORS(noise)

void launch_noise(const NoiseArgs& a, hipStream_t s)
{
    const int rows = a.K_loc - a.row_begin;
    if (rows <= 0) return;
    if (!a.zero_noise && a.first_global + a.row_begin >= a.K_gen_global && a.J <= 4 * kNoiseJT &&
        noise_rows_lds(a, 0) <= kRolloutLdsMax) {
        // every row is a reused one (no normals, no L z): the per-row matrix-core kernel
        launch_noise_rows<false>(a, ReuseArgs{}, rows, noise_rows_lds(a, 0), s);
        return;
    }
    const int block = a.N <= 128 ? 128 : 256;
#ifndef NOISE_RT
#define NOISE_RT 4
#endif
    const int rt = rows >= NOISE_RT ? NOISE_RT : 1;
    const size_t lds = (size_t)rt * (2 * (a.N + kBandBatch) + 2 * a.Nall) * sizeof(double);
    dim3 grid((rows + rt - 1) / rt, a.J);
    if (rt == NOISE_RT) {
        if (block == 128) hipLaunchKernelGGL((k_noise<128, NOISE_RT>), grid, dim3(128), lds, s, a);
        else hipLaunchKernelGGL((k_noise<256, NOISE_RT>), grid, dim3(256), lds, s, a);
    } else {
        if (block == 128) hipLaunchKernelGGL((k_noise<128, 1>), grid, dim3(128), lds, s, a);
        else hipLaunchKernelGGL((k_noise<256, 1>), grid, dim3(256), lds, s, a);
    }
}

}  // namespace stomp
