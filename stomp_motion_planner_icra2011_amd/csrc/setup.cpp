// setup.cpp -- host setup of the STOMP engine (see setup.h for the reference map).
#include "setup.h"

#include <cmath>
#include <cstring>

namespace stomp {

const double kDiffRules[kNumDiffRules][kDiffRuleLength] = {
    {0, 0, -2 / 6.0, -3 / 6.0, 6 / 6.0, -1 / 6.0, 0},
    {0, -1 / 12.0, 16 / 12.0, -30 / 12.0, 16 / 12.0, -1 / 12.0, 0},
    {0, 1 / 12.0, -17 / 12.0, 46 / 12.0, -46 / 12.0, 17 / 12.0, -1 / 12.0}};

namespace {

// Banded Gram matrix G = D^T D of a 7-tap stencil matrix with row entries
// D(k, k+j) = coef[j+3] (truncated at the borders).  The dense product summed
// over k in ascending order only adds exact zeros outside the band, so summing
// the in-band k ascending is the same number.
void banded_gram(const double* coef, int n, std::vector<double>& G)
{
    G.assign((size_t)n * n, 0.0);
    for (int a = 0; a < n; ++a) {
        for (int b = a - 6; b <= a + 6; ++b) {
            if (b < 0 || b >= n) continue;
            int k0 = std::max(a, b) - 3, k1 = std::min(a, b) + 3;
            double s = 0.0;
            bool any = false;
            for (int k = std::max(k0, 0); k <= std::min(k1, n - 1); ++k) {
                double x = coef[a - k + 3] * coef[b - k + 3];
                s = any ? s + x : 0.0 + x;
                any = true;
            }
            G[(size_t)a * n + b] = s;
        }
    }
}

bool cholesky(const std::vector<double>& A, int n, std::vector<double>& C)
{
    C.assign((size_t)n * n, 0.0);
    for (int j = 0; j < n; ++j) {
        double s = A[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) s -= C[(size_t)j * n + k] * C[(size_t)j * n + k];
        if (!(s > 0.0)) return false;
        double cjj = std::sqrt(s);
        C[(size_t)j * n + j] = cjj;
        for (int i = j + 1; i < n; ++i) {
            double t = A[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) t -= C[(size_t)i * n + k] * C[(size_t)j * n + k];
            C[(size_t)i * n + j] = t / cjj;
        }
    }
    return true;
}

// A^-1 = C^-T C^-1, one unit column at a time (forward then back substitution)
bool spd_inverse(const std::vector<double>& A, int n, std::vector<double>& X)
{
    std::vector<double> C, y(n);
    if (!cholesky(A, n, C)) return false;
    X.assign((size_t)n * n, 0.0);
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
    return true;
}

}  // namespace

std::string noise_setup(const std::vector<double>& R, int n, std::vector<double>& Rinv, std::vector<double>& L,
                        std::vector<double>& M)
{
    if (n <= 0 || R.size() != (size_t)n * n) return "control cost matrix has the wrong size";
    if (!spd_inverse(R, n, Rinv) || !cholesky(Rinv, n, L)) return "control cost matrix R is not positive definite";
    M.assign((size_t)n * n, 0.0);
    for (int p = 0; p < n; ++p) {
        double cmax = Rinv[p];
        for (int p2 = 1; p2 < n; ++p2)
            if (Rinv[(size_t)p2 * n + p] > cmax) cmax = Rinv[(size_t)p2 * n + p];
        double sc = 1.0 / ((double)n * cmax);
        for (int i = 0; i < n; ++i) M[(size_t)i * n + p] = Rinv[(size_t)i * n + p] * sc;
    }
    return std::string();
}

std::string compute_setup(const SetupInput& in, SetupOutput& out)
{
    const int J = in.J, N = in.N, Nall = N + 2 * kPad;
    out.Nall = Nall;
    // group trajectory duration (Nall-1)*disc truncated to int by getDuration()
    // (stomp_trajectory.cpp:86, stomp_trajectory.h:141,255-258)
    int duration = (int)((double)(Nall - 1) * in.discretization);
    out.dt = (double)duration / (double)(N + 1);
    if (!(out.dt > 0.0)) return "trajectory duration truncates to zero (getDuration() returns int)";

    double mult = 1.0;
    for (int d = 0; d < kNumDiffRules; ++d) {
        mult /= out.dt;
        for (int j = 0; j < kDiffRuleLength; ++j) out.dcoef[d][j] = mult * kDiffRules[d][j];
    }
    std::vector<double> G;
    out.Rall.assign((size_t)Nall * Nall, 0.0);
    for (int i = 0; i < Nall; ++i) out.Rall[(size_t)i * Nall + i] = 1.0 * in.ridge_factor;
    for (int d = 0; d < kNumDiffRules; ++d) {
        banded_gram(out.dcoef[d], Nall, G);
        for (size_t k = 0; k < G.size(); ++k) out.Rall[k] += in.smoothness_costs[d] * G[k];
    }
    std::vector<double> Rfree((size_t)N * N);
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) Rfree[(size_t)i * N + j] = out.Rall[(size_t)(i + kPad) * Nall + (j + kPad)];
    {
        std::string msg = noise_setup(Rfree, N, out.Rinv, out.L, out.M);
        if (!msg.empty()) return msg;
    }

    // StompCost: Q = sum_i (w_i * disc^(i+1)) D_i^T D_i + ridge I with raw stencils
    out.Qinv.assign((size_t)J * N * N, 0.0);
    double max_scale = 0.0;
    std::vector<double> Qfull, Qfree((size_t)N * N), Qi;
    for (int jt = 0; jt < J; ++jt) {
        Qfull.assign((size_t)Nall * Nall, 0.0);
        double m2 = 1.0;
        for (int d = 0; d < kNumDiffRules; ++d) {
            m2 *= in.discretization;
            banded_gram(kDiffRules[d], Nall, G);
            double w = in.joint_cost[jt] * in.smoothness_costs[d];
            double f = w * m2;
            for (size_t k = 0; k < G.size(); ++k) Qfull[k] += f * G[k];
        }
        for (int i = 0; i < Nall; ++i) Qfull[(size_t)i * Nall + i] += 1.0 * in.ridge_factor;
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) Qfree[(size_t)i * N + j] = Qfull[(size_t)(i + kPad) * Nall + (j + kPad)];
        if (!spd_inverse(Qfree, N, Qi)) return "joint cost matrix Q is not positive definite";
        double mx = Qi[0];
        for (size_t k = 1; k < Qi.size(); ++k)
            if (Qi[k] > mx) mx = Qi[k];
        if (max_scale < mx) max_scale = mx;
        std::memcpy(out.Qinv.data() + (size_t)jt * N * N, Qi.data(), sizeof(double) * N * N);
    }
    double inv_scale = 1.0 / max_scale;
    for (double& v : out.Qinv) v *= inv_scale;

    out.theta.assign((size_t)J * N, 0.0);
    std::vector<double> lin(N);
    for (int d = 0; d < J; ++d) {
        for (int c = 0; c < N; ++c) {
            double a = 0.0;
            for (int i = 0; i < kPad; ++i) a += in.start[d] * out.Rall[(size_t)i * Nall + (c + kPad)];
            double b = 0.0;
            for (int i = 0; i < kPad; ++i) b += in.goal[d] * out.Rall[(size_t)(N + kPad + i) * Nall + (c + kPad)];
            lin[c] = (a + b) * 2.0;
        }
        for (int i = 0; i < N; ++i) {
            double s = 0.0;
            for (int k = 0; k < N; ++k) s += (-0.5 * out.Rinv[(size_t)i * N + k]) * lin[k];
            out.theta[(size_t)d * N + i] = s;
        }
    }
    return std::string();
}

}  // namespace stomp
