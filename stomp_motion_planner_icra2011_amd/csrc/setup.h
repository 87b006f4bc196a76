// setup.h -- once-per-problem host setup of the STOMP engine (not on the hot path).
//
// Computes the quantities the reference builds before its iteration loop:
//   policy differentiation stencils   createDifferentiationMatrices  covariant_trajectory_policy.cpp:204-226
//   R (all variables), R^-1 (free)    initializeCosts                covariant_trajectory_policy.cpp:168-191
//   L = chol(R^-1)                    MultivariateGaussian ctor      multivariate_gaussian.h:76-86
//   M (projection)                    preComputeProjectionMatrices   policy_improvement.cpp:421-441
//   Q^-1 per joint, scaled            StompCost + scale              stomp_cost.cpp:47-105, stomp_optimizer.cpp:100-125
//   theta_0                           setToMinControlCost            covariant_trajectory_policy.cpp:102-148
// Every sum is sequential in index order with one rounding per operation, so the
// result does not depend on the compiler (build with -ffp-contract=off).
#pragma once

#include <string>
#include <vector>

namespace stomp {

constexpr int kDiffRuleLength = 7;
constexpr int kNumDiffRules = 3;
constexpr int kPad = kDiffRuleLength - 1;

// stomp_utils.h:49-56
extern const double kDiffRules[kNumDiffRules][kDiffRuleLength];

struct SetupInput {
    int J = 0, N = 0;
    double discretization = 0.05;
    double smoothness_costs[3] = {0, 1, 0};
    double ridge_factor = 0.0;
    std::vector<double> joint_cost;  // J
    std::vector<double> start, goal; // J
};

struct SetupOutput {
    int Nall = 0;
    double dt = 0.0;                                  // policy movement_dt_
    double dcoef[kNumDiffRules][kDiffRuleLength];     // policy D_i row entries (scaled stencils)
    std::vector<double> Rall;                         // Nall x Nall
    std::vector<double> Rinv, L, M;                   // N x N (row-major)
    std::vector<double> Qinv;                         // J x N x N (scaled)
    std::vector<double> theta;                        // J x N
};

// Returns an empty string on success, otherwise the error message.
std::string compute_setup(const SetupInput& in, SetupOutput& out);

// PolicyImprovement::initialize's per-dimension noise set-up from a control-cost matrix R
// (n x n, row-major; policy_improvement.cpp:77-86, 421-441): Rinv = R^-1, L = chol(Rinv) (the
// MultivariateGaussian factor, multivariate_gaussian.h:76-86) and the projection M (Rinv with
// column p scaled by 1 / (n max_i Rinv(i, p))).  compute_setup uses it for the free block of R.
std::string noise_setup(const std::vector<double>& R, int n, std::vector<double>& Rinv, std::vector<double>& L,
                        std::vector<double>& M);

}  // namespace stomp
