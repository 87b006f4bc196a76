// stomp_facade.cpp -- reference-shaped C++ classes over the engine's C ABI.
// See include/stomp_motion_planner/stomp_facade.h for the mapping to the reference.
#include "stomp_motion_planner/stomp_facade.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <utility>

#include "setup.h"
#include "stomp_math.h"

namespace stomp_motion_planner {

namespace {
std::string engine_error(stomp_engine* e, int rc)
{
    char buf[32];
    std::snprintf(buf, sizeof buf, "error %d: ", rc);
    return std::string(buf) + (e ? stomp_engine_last_error(e) : stomp_last_error());
}
}  // namespace

// ------------------------------------------------------------------ Task

bool Task::executeBatch(std::vector<std::vector<VectorXd>>& parameters, std::vector<VectorXd>& costs,
                        const int iteration_number)
{
    costs.assign(parameters.size(), VectorXd());
    for (size_t r = 0; r < parameters.size(); ++r)
        if (!execute(parameters[r], costs[r], iteration_number)) return false;
    return true;
}

// ------------------------------------------------------------------ StompOptimizer

StompOptimizer::StompOptimizer(StompTrajectory* trajectory, const StompRobotModel* robot_model,
                               const StompParameters* parameters, StompCollisionSpace* collision_space,
                               const Constraints& constraints, int device, void* stream)
    : trajectory_(trajectory), parameters_(parameters)
{
    if (!trajectory || !robot_model || !parameters || !collision_space) {
        error_ = "StompOptimizer: null argument";
        return;
    }
    J_ = trajectory->num_joints;
    N_ = trajectory->num_points;
    const StompParameters& p = *parameters;
    if ((int)trajectory->start.size() != J_ || (int)trajectory->goal.size() != J_ ||
        (int)robot_model->joints.size() != J_) {
        error_ = "StompOptimizer: start/goal/joint tables must have num_joints entries";
        return;
    }
    // policy_improvement_loop.cpp:99-100 reads one noise_stddev / noise_decay per joint
    // (and reads past the end when they are short); here a short list is an error
    if ((int)p.noise_stddev.size() != J_ || (int)p.noise_decay.size() != J_) {
        error_ = "StompOptimizer: noise_stddev and noise_decay need one entry per joint";
        return;
    }
    // the descriptor's tables: copies owned here (createSibling reads them any time later)
    segments_ = robot_model->segments;
    joints_ = robot_model->joints;
    spheres_ = robot_model->collision_points;
    inertias_ = robot_model->inertias;
    noise_stddev_ = p.noise_stddev;
    noise_decay_ = p.noise_decay;
    start_ = trajectory->start;
    goal_ = trajectory->goal;
    stomp_engine_desc d{};
    d.abi_version = STOMP_ENGINE_ABI_VERSION;
    d.num_joints = J_;
    d.num_time_steps = N_;
    d.num_rollouts = p.num_rollouts;
    d.num_reused_rollouts = p.num_reused_rollouts;
    d.num_segments = (int32_t)robot_model->segments.size();
    d.segments = segments_.data();
    d.num_spheres = (int32_t)spheres_.size();
    d.spheres = spheres_.data();
    d.joints = joints_.data();
    d.grid = collision_space->grid;
    d.discretization = p.trajectory_discretization;
    d.smoothness_costs[0] = p.smoothness_cost_velocity;
    d.smoothness_costs[1] = p.smoothness_cost_acceleration;
    d.smoothness_costs[2] = p.smoothness_cost_jerk;
    d.ridge_factor = p.ridge_factor;
    d.smoothness_cost_weight = p.smoothness_cost_weight;
    d.obstacle_cost_weight = p.obstacle_cost_weight;
    d.constraint_cost_weight = p.constraint_cost_weight;
    d.torque_cost_weight = p.torque_cost_weight;
    d.noise_stddev = noise_stddev_.data();
    d.noise_decay = noise_decay_.data();
    d.use_cumulative_costs = p.use_cumulative_costs ? 1 : 0;
    d.start = start_.data();
    d.goal = goal_.data();
    d.seed = p.seed;
    d.max_iterations = p.max_iterations;
    d.max_iterations_after_collision_free = p.max_iterations_after_collision_free;
    d.device = device;
    d.stream = stream;
    d.rank = 0;
    d.world_size = 1;
    d.inertias = inertias_.size() == segments_.size() ? inertias_.data() : nullptr;
    d.torque_root = robot_model->torque_root;
    d.torque_tip = robot_model->torque_tip;
    for (int k = 0; k < 3; ++k) d.gravity[k] = robot_model->gravity[k];
    constraints_ = constraints;
    d.num_orientation_constraints = (int32_t)constraints_.orientation_constraints.size();
    d.orientation_constraints = constraints_.orientation_constraints.data();
    desc_ = d;
    int rc = stomp_engine_create(&d, &engine_);
    if (rc) {
        error_ = engine_error(nullptr, rc);
        engine_ = nullptr;
        return;
    }
    policy_ = std::make_shared<CovariantTrajectoryPolicy>(this);
}

StompOptimizer::~StompOptimizer()
{
    if (engine_) stomp_engine_destroy(engine_);
}

bool StompOptimizer::check(int rc)
{
    if (rc == 0) return true;
    error_ = engine_error(engine_, rc);
    return false;
}

stomp_engine* StompOptimizer::createSibling(int num_rollouts, int num_reused_rollouts, bool use_cumulative_costs,
                                            std::string& err) const
{
    if (!engine_) {
        err = "no engine";
        return nullptr;
    }
    stomp_engine_desc d = desc_;
    d.num_rollouts = num_rollouts;
    d.num_reused_rollouts = num_reused_rollouts;
    d.use_cumulative_costs = use_cumulative_costs ? 1 : 0;
    stomp_engine* e = nullptr;
    const int rc = stomp_engine_create(&d, &e);
    if (rc) {
        err = engine_error(nullptr, rc);
        return nullptr;
    }
    return e;
}

bool StompOptimizer::optimize()
{
    if (!engine_) return false;
    stats_ = STOMPStatistics();
    stats_.costs.assign(parameters_->max_iterations > 0 ? parameters_->max_iterations : 1, 0.0);
    stomp_stats st{};
    if (!check(stomp_engine_optimize(engine_, &st, stats_.costs.data()))) return false;
    stats_.iterations = st.iterations;
    stats_.success = st.success != 0;
    stats_.success_iteration = st.success_iteration;
    stats_.collision_success_iteration = st.collision_success_iteration;
    stats_.last_improvement_iteration = st.last_improvement_iteration;
    stats_.best_cost = st.best_cost;
    stats_.success_duration = st.success_duration;
    stats_.collision_success_duration = st.collision_success_duration;
    stats_.costs.resize(st.iterations);
    // the torques of the final trajectory (stomp_optimizer.cpp:384-398), when the robot model
    // carries the inertias the reference reads from its URDF
    stats_.torques.assign(N_, 0.0);
    if (stomp_engine_get_best_torques(engine_, stats_.torques.data()) != 0) stats_.torques.clear();
    // group_trajectory_ = best_group_trajectory_; updateFullTrajectory (stomp_optimizer.cpp:368-369)
    std::vector<double> best((size_t)J_ * N_);
    if (!check(stomp_engine_get_best_trajectory(engine_, best.data()))) return false;
    trajectory_->free.assign(J_, VectorXd(N_));
    for (int j = 0; j < J_; ++j)
        for (int t = 0; t < N_; ++t) trajectory_->free[j][t] = best[(size_t)j * N_ + t];
    return true;
}

bool StompOptimizer::initialize(int num_time_steps)
{
    if (!engine_) return false;
    if (num_time_steps != N_) {
        error_ = "initialize: num_time_steps is fixed when the engine is created";
        return false;
    }
    return true;
}

bool StompOptimizer::execute(std::vector<VectorXd>& parameters, VectorXd& costs, const int iteration_number)
{
    std::vector<VectorXd> c;
    std::vector<bool> cf;
    if (!executeBatch({parameters}, c, cf, iteration_number)) return false;
    costs = c[0];
    last_cf_ = cf[0];
    // last_trajectory_cost_ = costs.sum() (stomp_optimizer.cpp:1155), sequential
    double sum = 0.0;
    for (double v : costs) sum += v;
    last_cost_ = sum;
    return true;
}

bool StompOptimizer::executeBatch(std::vector<std::vector<VectorXd>>& parameters, std::vector<VectorXd>& costs,
                                  const int iteration_number)
{
    std::vector<bool> cf;
    return executeBatch(static_cast<const std::vector<std::vector<VectorXd>>&>(parameters), costs, cf,
                        iteration_number);
}

bool StompOptimizer::executeBatch(const std::vector<std::vector<VectorXd>>& parameters, std::vector<VectorXd>& costs,
                                  std::vector<bool>& collision_free, const int iteration_number)
{
    if (!engine_) return false;
    const int E = (int)parameters.size();
    std::vector<double> prm((size_t)E * J_ * N_);
    for (int r = 0; r < E; ++r) {
        if ((int)parameters[r].size() != J_) {
            error_ = "execute: parameters need one vector per joint";
            return false;
        }
        for (int j = 0; j < J_; ++j) {
            if ((int)parameters[r][j].size() != N_) {
                error_ = "execute: parameter vectors need num_time_steps entries";
                return false;
            }
            for (int t = 0; t < N_; ++t) prm[((size_t)r * J_ + j) * N_ + t] = parameters[r][j][t];
        }
    }
    std::vector<double> c((size_t)E * N_);
    std::vector<uint8_t> cf(E > 0 ? E : 1), cs(E > 0 ? E : 1);
    // StompOptimizer::iteration_ is iteration_number - 1 inside runSingleIteration
    if (!check(stomp_engine_eval(engine_, prm.data(), E, c.data(), cf.data(), nullptr, iteration_number - 1,
                                 cs.data())))
        return false;
    if (E > 0) last_cs_ = cs[E - 1] != 0;
    costs.assign(E, VectorXd(N_));
    collision_free.assign(E, false);
    for (int r = 0; r < E; ++r) {
        for (int t = 0; t < N_; ++t) costs[r][t] = c[(size_t)r * N_ + t];
        collision_free[r] = cf[r] != 0;
    }
    return true;
}

bool StompOptimizer::getPolicy(std::shared_ptr<Policy>& policy)
{
    policy = policy_;
    return engine_ != nullptr;
}

bool StompOptimizer::setPolicy(const std::shared_ptr<Policy> /*policy*/)
{
    return true;   // the reference ignores the argument as well (stomp_optimizer.cpp:1173-1176)
}

bool StompOptimizer::getControlCostWeight(double& control_cost_weight)
{
    control_cost_weight = parameters_->smoothness_cost_weight;   // stomp_optimizer.cpp:1178-1182
    return true;
}

// ------------------------------------------------------------------ CovariantTrajectoryPolicy

bool CovariantTrajectoryPolicy::setNumTimeSteps(const int num_time_steps)
{
    return num_time_steps == owner_->N_;
}

bool CovariantTrajectoryPolicy::getNumTimeSteps(int& num_time_steps)
{
    num_time_steps = owner_->N_;
    return true;
}

bool CovariantTrajectoryPolicy::getNumDimensions(int& num_dimensions)
{
    num_dimensions = owner_->J_;
    return true;
}

bool CovariantTrajectoryPolicy::getNumParameters(std::vector<int>& num_params)
{
    num_params.assign(owner_->J_, owner_->N_);
    return true;
}

bool CovariantTrajectoryPolicy::getBasisFunctions(std::vector<MatrixXd>& basis_functions)
{
    // identity basis (covariant_trajectory_policy.cpp:193-202)
    MatrixXd I(owner_->N_, owner_->N_);
    for (int i = 0; i < owner_->N_; ++i) I(i, i) = 1.0;
    basis_functions.assign(owner_->J_, I);
    return true;
}

bool CovariantTrajectoryPolicy::getControlCosts(std::vector<MatrixXd>& control_costs)
{
    MatrixXd R(owner_->N_, owner_->N_);
    if (!owner_->check(stomp_engine_get_matrix(owner_->engine_, "R", 0, R.data_.data()))) return false;
    control_costs.assign(owner_->J_, R);
    return true;
}

bool CovariantTrajectoryPolicy::updateParameters(const std::vector<MatrixXd>& updates)
{
    // covariant_trajectory_policy.cpp:306-342: row 0 of each update, divisor 1.0
    const int J = owner_->J_, N = owner_->N_;
    if ((int)updates.size() != J) return false;
    std::vector<double> th((size_t)J * N);
    if (!owner_->check(stomp_engine_get_theta(owner_->engine_, th.data()))) return false;
    for (int d = 0; d < J; ++d) {
        if (updates[d].cols() != N || updates[d].rows() < 1) return false;
        for (int t = 0; t < N; ++t) th[(size_t)d * N + t] += updates[d](0, t) / 1.0;
    }
    return owner_->check(stomp_engine_set_theta(owner_->engine_, th.data()));
}

bool CovariantTrajectoryPolicy::getParameters(std::vector<VectorXd>& parameters)
{
    const int J = owner_->J_, N = owner_->N_;
    std::vector<double> th((size_t)J * N);
    if (!owner_->check(stomp_engine_get_theta(owner_->engine_, th.data()))) return false;
    parameters.assign(J, VectorXd(N));
    for (int d = 0; d < J; ++d)
        for (int t = 0; t < N; ++t) parameters[d][t] = th[(size_t)d * N + t];
    return true;
}

bool CovariantTrajectoryPolicy::setParameters(const std::vector<VectorXd>& parameters)
{
    const int J = owner_->J_, N = owner_->N_;
    if ((int)parameters.size() != J) return false;
    std::vector<double> th((size_t)J * N);
    for (int d = 0; d < J; ++d) {
        if ((int)parameters[d].size() != N) return false;
        for (int t = 0; t < N; ++t) th[(size_t)d * N + t] = parameters[d][t];
    }
    return owner_->check(stomp_engine_set_theta(owner_->engine_, th.data()));
}

bool CovariantTrajectoryPolicy::loadDifferentiation()
{
    if (!D_.empty()) return true;
    const int A = owner_->N_ + 12;
    std::vector<MatrixXd> D(3, MatrixXd(A, A));
    const char* names[3] = {"D0", "D1", "D2"};
    for (int i = 0; i < 3; ++i)
        if (!owner_->check(stomp_engine_get_matrix(owner_->engine_, names[i], 0, D[i].data_.data()))) return false;
    D_ = D;
    return true;
}

// costs_all += (weight * derivative_costs_[i]) * (D_i x)^2 for the three rules, x = parameters_all_[d]
// with the free segment replaced (covariant_trajectory_policy.cpp:236-243, 285-291); the dense
// row products run over the stencil's band (the other entries of D_i are exact zeros), summed left
// to right as in the engine and the oracle; Eigen's GEMV may order the sum differently (DESIGN.md 3,
// parity unpinned there)
void CovariantTrajectoryPolicy::accumulateCosts(int d, const VectorXd& free, const double weight,
                                                VectorXd& costs_all) const
{
    const int N = owner_->N_, A = N + 12;
    const StompTrajectory& tr = *owner_->trajectory_;
    VectorXd x(A);
    for (int i = 0; i < A; ++i) x[i] = i < 6 ? tr.start[d] : (i >= 6 + N ? tr.goal[d] : free[i - 6]);
    const StompParameters& p = *owner_->parameters_;
    const double dc[3] = {p.smoothness_cost_velocity, p.smoothness_cost_acceleration, p.smoothness_cost_jerk};
    for (int r = 0; r < 3; ++r) {
        const double w = weight * dc[r];
        for (int i = 0; i < A; ++i) {
            double acc = 0.0;
            const int c0 = i - 3 < 0 ? 0 : i - 3, c1 = i + 3 >= A ? A - 1 : i + 3;
            for (int c = c0; c <= c1; ++c) acc += D_[r](i, c) * x[c];
            costs_all[i] += w * (acc * acc);
        }
    }
}

static void fold_padding(const VectorXd& costs_all, int N, VectorXd& out)
{
    // control_costs[d] = free segment, padding costs folded into the end points (:245-250)
    out.assign(costs_all.begin() + 6, costs_all.begin() + 6 + N);
    for (int i = 0; i < 6; ++i) {
        out[0] += costs_all[i];
        out[N - 1] += costs_all[N + 12 - (i + 1)];
    }
}

bool CovariantTrajectoryPolicy::computeControlCosts(const std::vector<MatrixXd>& /*control_cost_matrices*/,
                                                    const std::vector<VectorXd>& parameters,
                                                    const std::vector<VectorXd>& noise, const double weight,
                                                    std::vector<VectorXd>& control_costs)
{
    const int J = owner_->J_, N = owner_->N_;
    if ((int)parameters.size() != J || (int)noise.size() != J || !loadDifferentiation()) return false;
    control_costs.assign(J, VectorXd());
    for (int d = 0; d < J; ++d) {
        if ((int)parameters[d].size() != N || (int)noise[d].size() != N) return false;
        VectorXd x(N), costs_all(N + 12, 0.0);
        for (int t = 0; t < N; ++t) x[t] = parameters[d][t] + noise[d][t];
        accumulateCosts(d, x, weight, costs_all);
        fold_padding(costs_all, N, control_costs[d]);
    }
    return true;
}

bool CovariantTrajectoryPolicy::computeControlCosts(const std::vector<MatrixXd>& /*control_cost_matrices*/,
                                                    const std::vector<std::vector<VectorXd>>& parameters,
                                                    const double weight, std::vector<VectorXd>& control_costs)
{
    const int J = owner_->J_, N = owner_->N_;
    if ((int)parameters.size() != J || !loadDifferentiation()) return false;
    control_costs.assign(J, VectorXd());
    for (int d = 0; d < J; ++d) {
        VectorXd costs_all(N + 12, 0.0);
        for (const VectorXd& x : parameters[d]) {   // [num_time_steps] N
            if ((int)x.size() != N) return false;
            accumulateCosts(d, x, weight, costs_all);
        }
        fold_padding(costs_all, N, control_costs[d]);
    }
    return true;
}

// ------------------------------------------------------------------ PolicyImprovement

// The host rollout set (policy_improvement.cpp:64-489 for any Policy).  Arithmetic contract as
// the engine's and the oracle's: L z and M eps as k-ascending fma chains,
// rollout sums in 64-rollout blocks, the deterministic exp of stomp_math.h, everything else one
// rounding per operation in the reference's order.
struct PolicyImprovement::HostRollouts {
    struct Rollout {
        std::vector<VectorXd> parameters, noise, noise_projected, control_costs, probabilities;
        VectorXd state_costs;
    };
    int J = 0, N = 0, K = 0, Kr = 0, Kx = 0, K_gen = 0;
    bool reused_next = false, extra_added = false;
    std::vector<MatrixXd> R;                       // control_costs_ (policy->getControlCosts)
    std::vector<std::vector<double>> Rinv, L, M;   // per dimension, N x N row-major
    std::vector<Rollout> rollouts, extra;
    std::vector<VectorXd> parameters;              // parameters_ (copyParametersFromPolicy)
    double control_cost_weight = 0.0;

    Rollout blank() const
    {
        Rollout r;
        r.parameters.assign(J, VectorXd(N, 0.0));
        r.noise = r.noise_projected = r.control_costs = r.probabilities = r.parameters;
        r.state_costs.assign(N, 0.0);
        return r;
    }
    // y = A x, k ascending, one rounding per multiply-add; lower: the triangle k <= i only (the
    // zeros above it add nothing)
    void fma_product(const std::vector<double>& A, const VectorXd& x, VectorXd& y, bool lower) const
    {
        y.assign(N, 0.0);
        for (int i = 0; i < N; ++i) {
            double s = 0.0;
            const int kend = lower ? i + 1 : N;
            for (int k = 0; k < kend; ++k) s = std::fma(A[(size_t)i * N + k], x[k], s);
            y[i] = s;
        }
    }
    // Rollout::getCost (policy_improvement.cpp:149-156), sums in index order
    static double cost(const Rollout& r)
    {
        double c = r.state_costs[0];
        for (size_t t = 1; t < r.state_costs.size(); ++t) c += r.state_costs[t];
        for (const VectorXd& x : r.control_costs) {
            double sd = x[0];
            for (size_t t = 1; t < x.size(); ++t) sd += x[t];
            c += sd;
        }
        return c;
    }
    // sum_r v(r) in fixed 64-rollout blocks (the engine's canonical order; sequential for K <= 64)
    template <class F>
    double blocked_sum(int n, F v) const
    {
        double total = 0.0;
        for (int b0 = 0; b0 < n; b0 += 64) {
            double part = 0.0;
            const int b1 = b0 + 64 < n ? b0 + 64 : n;
            for (int r = b0; r < b1; ++r) part += v(r);
            total += part;
        }
        return total;
    }
};

PolicyImprovement::PolicyImprovement() = default;
PolicyImprovement::~PolicyImprovement()
{
    if (own_) stomp_engine_destroy(own_);
}

bool PolicyImprovement::check(int rc)
{
    if (rc == 0) return true;
    error_ = engine_error(engine_, rc);
    return false;
}

bool PolicyImprovement::initialize(const int num_rollouts, const int num_time_steps, const int num_reused_rollouts,
                                   const int num_extra_rollouts, std::shared_ptr<Policy> policy,
                                   bool use_cumulative_costs)
{
    initialized_ = false;
    host_.reset();
    owner_ = nullptr;
    engine_ = nullptr;
    if (own_) {
        stomp_engine_destroy(own_);
        own_ = nullptr;
    }
    if (!policy) {
        error_ = "PolicyImprovement::initialize: null policy";
        return false;
    }
    policy_ = policy;
    N_ = num_time_steps;
    use_cumulative_ = use_cumulative_costs;
    noise_iteration_ = 1;
    auto* ctp = dynamic_cast<CovariantTrajectoryPolicy*>(policy.get());
    if (ctp && ctp->owner() && ctp->owner()->ok()) {
        owner_ = ctp->owner();
        engine_ = owner_->engine_;
        J_ = owner_->J_;
        K_ = owner_->parameters_->num_rollouts;
        seed_ = owner_->parameters_->seed;
        if (num_time_steps != owner_->N_) {
            error_ = "PolicyImprovement::initialize: num_time_steps differs from the engine's";
            return false;
        }
    }
    if (!setNumRollouts(num_rollouts, num_reused_rollouts, num_extra_rollouts)) return false;
    return (initialized_ = true);
}

// PolicyImprovement::initialize (policy_improvement.cpp:64-94) with the rollout set on the host
bool PolicyImprovement::hostInitialize(int num_rollouts, int num_reused_rollouts, int num_extra_rollouts)
{
    auto h = std::make_shared<HostRollouts>();
    int J = 0;
    std::vector<int> np;
    if (!policy_->setNumTimeSteps(N_) || !policy_->getControlCosts(h->R) || !policy_->getNumDimensions(J) ||
        !policy_->getNumParameters(np) || !policy_->getParameters(h->parameters)) {
        error_ = "PolicyImprovement::initialize: policy query failed";
        return false;
    }
    if (J <= 0 || (int)np.size() != J || (int)h->R.size() != J || (int)h->parameters.size() != J) {
        error_ = "PolicyImprovement::initialize: policy dimensions disagree";
        return false;
    }
    for (int d = 0; d < J; ++d)
        if (np[d] != N_ || h->R[d].rows() != N_ || h->R[d].cols() != N_ || (int)h->parameters[d].size() != N_) {
            error_ = "PolicyImprovement::initialize: num_parameters must equal num_time_steps (identity basis)";
            return false;
        }
    h->J = J;
    h->N = N_;
    h->Rinv.resize(J);
    h->L.resize(J);
    h->M.resize(J);
    for (int d = 0; d < J; ++d) {
        // inv_control_costs_, MultivariateGaussian(0, R^-1), preComputeProjectionMatrices
        std::string msg = stomp::noise_setup(h->R[d].data_, N_, h->Rinv[d], h->L[d], h->M[d]);
        if (!msg.empty()) {
            error_ = "PolicyImprovement::initialize: " + msg;
            return false;
        }
    }
    J_ = J;
    host_ = h;
    return setNumRollouts(num_rollouts, num_reused_rollouts, num_extra_rollouts);
}

bool PolicyImprovement::setNumRollouts(const int num_rollouts, const int num_reused_rollouts,
                                       const int num_extra_rollouts)
{
    if (num_reused_rollouts >= num_rollouts) {   // policy_improvement.cpp:102-106
        error_ = "Number of reused rollouts must be strictly less than number of rollouts.";
        return false;
    }
    if (num_rollouts <= 0 || num_reused_rollouts < 0 || num_extra_rollouts < 0) {
        error_ = "setNumRollouts: negative or zero rollout count";
        return false;
    }
    if (owner_ && num_extra_rollouts == 1) {
        // on the device: the optimizer's engine for its own counts and setting (its reuse state
        // starts over on the next getRollouts), else an engine of our own for the new ones
        host_.reset();
        if (own_) {
            stomp_engine_destroy(own_);
            own_ = nullptr;
        }
        K_ = num_rollouts;
        if (num_rollouts == owner_->parameters_->num_rollouts &&
            num_reused_rollouts == owner_->parameters_->num_reused_rollouts &&
            use_cumulative_ == owner_->parameters_->use_cumulative_costs) {
            engine_ = owner_->engine_;
            return check(stomp_pi_reset(engine_));
        }
        std::string err;
        own_ = owner_->createSibling(num_rollouts, num_reused_rollouts, use_cumulative_, err);
        engine_ = own_;
        if (!own_) {
            error_ = "setNumRollouts: " + err;
            return false;
        }
        return true;
    }
    if (!host_) return hostInitialize(num_rollouts, num_reused_rollouts, num_extra_rollouts);
    HostRollouts& h = *host_;
    h.K = num_rollouts;
    h.Kr = num_reused_rollouts;
    h.Kx = num_extra_rollouts;
    h.K_gen = 0;
    h.rollouts.assign(h.K, h.blank());
    h.extra.assign(h.Kx, h.blank());
    h.reused_next = false;
    h.extra_added = false;
    K_ = h.K;
    return true;
}

bool PolicyImprovement::getRollouts(std::vector<std::vector<VectorXd>>& rollouts,
                                    const std::vector<double>& noise_stddev)
{
    if (!initialized_) { error_ = "getRollouts: not initialized"; return false; }
    if ((int)noise_stddev.size() != J_) { error_ = "getRollouts: one noise_stddev per dimension"; return false; }
    if (!host_) {
        if (engine_ == own_) {
            // generateRollouts perturbs the policy's current parameters: the optimizer's theta
            std::vector<double> th((size_t)J_ * N_);
            if (!check(stomp_engine_get_theta(owner_->engine_, th.data())) ||
                !check(stomp_engine_set_theta(own_, th.data())))
                return false;
        }
        std::vector<double> buf((size_t)K_ * J_ * N_);
        int32_t n = 0;
        if (!check(stomp_pi_get_rollouts(engine_, noise_iteration_, noise_stddev.data(), buf.data(), &n))) return false;
        ++noise_iteration_;
        K_gen_ = n;
        rollouts.assign(n, std::vector<VectorXd>(J_, VectorXd(N_)));
        for (int r = 0; r < n; ++r)
            for (int d = 0; d < J_; ++d)
                for (int t = 0; t < N_; ++t) rollouts[r][d][t] = buf[((size_t)r * J_ + d) * N_ + t];
        return true;
    }
    // generateRollouts (policy_improvement.cpp:158-239)
    HostRollouts& h = *host_;
    if (!policy_->getParameters(h.parameters)) { error_ = "getRollouts: policy getParameters failed"; return false; }
    h.K_gen = h.K - h.Kr;
    if (!h.reused_next) {
        h.K_gen = h.K;
        if (h.Kr > 0) h.reused_next = true;
    } else {
        // the best K_r of the previous rollouts and the extra rollouts, by (cost, index): the
        // extra ones carry the negative indices -r-1, as the reference's sorter
        std::vector<std::pair<double, int>> sorter;
        for (int r = 0; r < h.K; ++r) sorter.push_back({HostRollouts::cost(h.rollouts[r]), r});
        if (h.extra_added) {
            for (int r = 0; r < h.Kx; ++r) sorter.push_back({HostRollouts::cost(h.extra[r]), -r - 1});
            h.extra_added = false;
        }
        std::sort(sorter.begin(), sorter.end());
        std::vector<HostRollouts::Rollout> reused;
        for (int r = 0; r < h.Kr; ++r) {
            const int idx = sorter[r].second;
            reused.push_back(idx >= 0 ? h.rollouts[idx] : h.extra[-idx - 1]);
        }
        for (int r = 0; r < h.Kr; ++r) {
            HostRollouts::Rollout& dst = h.rollouts[h.K_gen + r];
            dst = reused[r];
            for (int d = 0; d < h.J; ++d)
                for (int t = 0; t < h.N; ++t) dst.noise[d][t] = dst.parameters[d][t] - h.parameters[d][t];
        }
    }
    // new rollouts: eps = sigma_d * (0 + L z), z the counter-based normals of (seed, iteration,
    // dimension, rollout); parameters = theta + eps
    VectorXd z(h.N), lz;
    for (int d = 0; d < h.J; ++d)
        for (int r = 0; r < h.K_gen; ++r) {
            for (int p = 0; 2 * p < h.N; ++p) {
                double z0, z1;
                stomp::normal_pair(seed_, noise_iteration_, d, r, p, &z0, &z1);
                z[2 * p] = z0;
                if (2 * p + 1 < h.N) z[2 * p + 1] = z1;
            }
            h.fma_product(h.L[d], z, lz, true);
            HostRollouts::Rollout& ro = h.rollouts[r];
            for (int t = 0; t < h.N; ++t) {
                ro.noise[d][t] = noise_stddev[d] * (0.0 + lz[t]);
                ro.parameters[d][t] = h.parameters[d][t] + ro.noise[d][t];
            }
        }
    ++noise_iteration_;
    K_gen_ = h.K_gen;
    rollouts.clear();
    for (int r = 0; r < h.K_gen; ++r) rollouts.push_back(h.rollouts[r].parameters);
    // computeProjectedNoise for every rollout (:283-290, 473-482)
    for (HostRollouts::Rollout& ro : h.rollouts)
        for (int d = 0; d < h.J; ++d) h.fma_product(h.M[d], ro.noise[d], ro.noise_projected[d], false);
    return true;
}

bool PolicyImprovement::setRolloutCosts(const MatrixXd& costs, const double control_cost_weight,
                                        std::vector<double>& rollout_costs_total)
{
    if (!initialized_) { error_ = "setRolloutCosts: not initialized"; return false; }
    if (costs.cols() != N_ || costs.rows() < K_gen_) {
        error_ = "setRolloutCosts: costs must be num_rollouts x num_time_steps";
        return false;
    }
    if (!host_) {
        std::vector<double> c((size_t)K_ * N_, 0.0);
        for (int r = 0; r < K_gen_; ++r)
            for (int t = 0; t < N_; ++t) c[(size_t)r * N_ + t] = costs(r, t);
        rollout_costs_total.assign(K_, 0.0);
        return check(stomp_pi_set_rollout_costs(engine_, c.data(), control_cost_weight, rollout_costs_total.data()));
    }
    // :262-281: the control costs of every rollout (computeRolloutControlCosts, :484-489), then
    // the state costs of the new ones
    HostRollouts& h = *host_;
    h.control_cost_weight = control_cost_weight;
    for (HostRollouts::Rollout& ro : h.rollouts)
        if (!policy_->computeControlCosts(h.R, ro.parameters, ro.noise_projected, 0.5 * h.control_cost_weight,
                                          ro.control_costs)) {
            error_ = "setRolloutCosts: policy computeControlCosts failed";
            return false;
        }
    for (int r = 0; r < h.K_gen; ++r)
        for (int t = 0; t < h.N; ++t) h.rollouts[r].state_costs[t] = costs(r, t);
    rollout_costs_total.resize(h.K);
    for (int r = 0; r < h.K; ++r) rollout_costs_total[r] = HostRollouts::cost(h.rollouts[r]);
    return true;
}

bool PolicyImprovement::improvePolicy(std::vector<MatrixXd>& parameter_updates)
{
    if (!initialized_) { error_ = "improvePolicy: not initialized"; return false; }
    if (!host_) {
        std::vector<double> u((size_t)J_ * N_);
        if (!check(stomp_pi_improve_policy(engine_, u.data()))) return false;
        parameter_updates.assign(J_, MatrixXd(N_, N_));
        for (int d = 0; d < J_; ++d)
            for (int t = 0; t < N_; ++t) parameter_updates[d](0, t) = u[(size_t)d * N_ + t];
        return true;
    }
    // :385-401: cumulative costs (:301-320), probabilities (:322-368), updates (:370-383)
    HostRollouts& h = *host_;
    const int K = h.K, N = h.N;
    parameter_updates.assign(h.J, MatrixXd(N, N));
    std::vector<double> cum((size_t)K * N);
    VectorXd upd(N), delta;
    for (int d = 0; d < h.J; ++d) {
        for (int r = 0; r < K; ++r) {
            double* c = cum.data() + (size_t)r * N;
            for (int t = 0; t < N; ++t) c[t] = h.rollouts[r].state_costs[t] + h.rollouts[r].control_costs[d][t];
            if (use_cumulative_)
                for (int t = N - 2; t >= 0; --t) c[t] += c[t + 1];
        }
        for (int t = 0; t < N; ++t) {
            double mn = cum[t], mx = mn;
            for (int r = 1; r < K; ++r) {
                const double c = cum[(size_t)r * N + t];
                if (c < mn) mn = c;
                if (c > mx) mx = c;
            }
            double denom = mx - mn;
            if (denom < 1e-8) denom = 1e-8;
            for (int r = 0; r < K; ++r)
                h.rollouts[r].probabilities[d][t] = stomp::det_exp(-10.0 * (cum[(size_t)r * N + t] - mn) / denom);
            const double psum = h.blocked_sum(K, [&](int r) { return h.rollouts[r].probabilities[d][t]; });
            for (int r = 0; r < K; ++r) h.rollouts[r].probabilities[d][t] /= psum;
            upd[t] = h.blocked_sum(
                K, [&](int r) { return h.rollouts[r].noise[d][t] * h.rollouts[r].probabilities[d][t]; });
        }
        // projection_matrix_[d] * the row (dense, k ascending, one rounding per operation)
        delta.assign(N, 0.0);
        for (int i = 0; i < N; ++i) {
            double s = 0.0;
            for (int k = 0; k < N; ++k) s += h.M[d][(size_t)i * N + k] * upd[k];
            delta[i] = s;
        }
        for (int t = 0; t < N; ++t) parameter_updates[d](0, t) = delta[t];
    }
    return true;
}

bool PolicyImprovement::addExtraRollouts(std::vector<std::vector<VectorXd>>& rollouts,
                                         std::vector<VectorXd>& rollout_costs)
{
    if (!initialized_) { error_ = "addExtraRollouts: not initialized"; return false; }
    if (!host_) {
        if (rollouts.size() != 1 || rollout_costs.size() != 1 || (int)rollouts[0].size() != J_ ||
            (int)rollout_costs[0].size() != N_) {
            error_ = "addExtraRollouts: one extra rollout ([J] N parameters, N costs)";
            return false;
        }
        std::vector<double> prm((size_t)J_ * N_);
        for (int d = 0; d < J_; ++d) {
            if ((int)rollouts[0][d].size() != N_) { error_ = "addExtraRollouts: bad parameter size"; return false; }
            for (int t = 0; t < N_; ++t) prm[(size_t)d * N_ + t] = rollouts[0][d][t];
        }
        return check(stomp_pi_add_extra_rollouts(engine_, 1, prm.data(), rollout_costs[0].data()));
    }
    // :443-489: noise = parameters - theta, its projection and control costs
    HostRollouts& h = *host_;
    if ((int)rollouts.size() != h.Kx || (int)rollout_costs.size() != h.Kx) {
        error_ = "addExtraRollouts: num_extra_rollouts rollouts and costs";
        return false;
    }
    if (!policy_->getParameters(h.parameters)) { error_ = "addExtraRollouts: policy getParameters failed"; return false; }
    for (int r = 0; r < h.Kx; ++r) {
        if ((int)rollouts[r].size() != h.J || (int)rollout_costs[r].size() != h.N) {
            error_ = "addExtraRollouts: bad rollout size";
            return false;
        }
        HostRollouts::Rollout& ro = h.extra[r];
        ro.parameters = rollouts[r];
        ro.state_costs = rollout_costs[r];
        for (int d = 0; d < h.J; ++d) {
            if ((int)ro.parameters[d].size() != h.N) { error_ = "addExtraRollouts: bad parameter size"; return false; }
            for (int t = 0; t < h.N; ++t) ro.noise[d][t] = ro.parameters[d][t] - h.parameters[d][t];
            h.fma_product(h.M[d], ro.noise[d], ro.noise_projected[d], false);
        }
        if (!policy_->computeControlCosts(h.R, ro.parameters, ro.noise_projected, 0.5 * h.control_cost_weight,
                                          ro.control_costs)) {
            error_ = "addExtraRollouts: policy computeControlCosts failed";
            return false;
        }
    }
    h.extra_added = true;
    return true;
}

// ------------------------------------------------------------------ PolicyImprovementLoop

bool PolicyImprovementLoop::initialize(std::shared_ptr<Task> task)
{
    optimizer_ = owner_ = nullptr;
    if (!task) {
        error_ = "PolicyImprovementLoop::initialize: null task";
        return false;
    }
    std::shared_ptr<Policy> policy;
    if (!task->getPolicy(policy) || !policy) {
        error_ = "PolicyImprovementLoop::initialize: the task has no policy";
        return false;
    }
    auto* ctp = dynamic_cast<CovariantTrajectoryPolicy*>(policy.get());
    if (!ctp || !ctp->owner() || !ctp->owner()->ok()) {
        error_ = "PolicyImprovementLoop::initialize: a task whose policy is not a StompOptimizer's needs the "
                 "StompParameters (initialize(task, parameters))";
        return false;
    }
    return initialize(task, *ctp->owner()->parameters_);
}

bool PolicyImprovementLoop::initialize(std::shared_ptr<Task> task, const StompParameters& p)
{
    optimizer_ = owner_ = nullptr;
    if (!task) {
        error_ = "PolicyImprovementLoop::initialize: null task";
        return false;
    }
    std::shared_ptr<Policy> policy;
    if (!task->getPolicy(policy) || !policy) {
        error_ = "PolicyImprovementLoop::initialize: the task has no policy";
        return false;
    }
    auto* ctp = dynamic_cast<CovariantTrajectoryPolicy*>(policy.get());
    if (ctp && ctp->owner() && ctp->owner()->ok()) owner_ = ctp->owner();
    optimizer_ = dynamic_cast<StompOptimizer*>(task.get());
    task_ = task;
    policy_ = policy;
    // readParameters (policy_improvement_loop.cpp:112-123)
    num_rollouts_ = p.num_rollouts;
    if (owner_) {
        num_time_steps_ = owner_->N_;
    } else if (!policy_->getNumTimeSteps(num_time_steps_)) {
        error_ = "PolicyImprovementLoop::initialize: policy getNumTimeSteps failed";
        return false;
    }
    noise_stddev_ = p.noise_stddev;
    noise_decay_ = p.noise_decay;
    if (!task_->initialize(num_time_steps_) || !task_->getControlCostWeight(control_cost_weight_)) {
        error_ = "PolicyImprovementLoop::initialize: task initialize / getControlCostWeight failed";
        return false;
    }
    int dims = 0;
    policy_->getNumDimensions(dims);
    if (dims != (int)noise_stddev_.size() || dims != (int)noise_decay_.size()) {
        error_ = "PolicyImprovementLoop::initialize: noise_stddev / noise_decay need one entry per dimension";
        return false;
    }
    policy_improvement_.setNoiseSeed(p.seed);
    if (!policy_improvement_.initialize(num_rollouts_, num_time_steps_, p.num_reused_rollouts, 1, policy_,
                                        p.use_cumulative_costs)) {
        error_ = policy_improvement_.lastError();
        return false;
    }
    return true;
}

bool PolicyImprovementLoop::runSingleIteration(int iteration_number)
{
    if (!task_) {
        error_ = "runSingleIteration: not initialized";
        return false;
    }
    if (!fused_ || !optimizer_ || optimizer_ != owner_ || !policy_improvement_.onEngine())
        return runGeneric(iteration_number);
    // the whole iteration as the engine's fused launch sequence
    stomp_iter_out out{};
    int rc = stomp_engine_iterate(optimizer_->engine_, iteration_number, &out);
    if (rc) {
        error_ = engine_error(optimizer_->engine_, rc);
        return false;
    }
    optimizer_->last_cost_ = out.cost;
    optimizer_->last_cf_ = out.collision_free != 0;
    optimizer_->last_cs_ = out.constraints_satisfied != 0;
    return true;
}

// policy_improvement_loop.cpp:143-202 step by step
bool PolicyImprovementLoop::runGeneric(int iteration_number)
{
    const int J = (int)noise_stddev_.size();
    std::vector<double> noise(J);
    for (int i = 0; i < J; ++i) noise[i] = noise_stddev_[i] * std::pow(noise_decay_[i], iteration_number - 1);
    policy_improvement_.setNoiseIteration(iteration_number);
    if (!policy_improvement_.getRollouts(rollouts_, noise)) {
        error_ = policy_improvement_.lastError();
        return false;
    }
    std::vector<VectorXd> costs;
    if (!task_->executeBatch(rollouts_, costs, iteration_number) || costs.size() != rollouts_.size()) {
        error_ = "runSingleIteration: Task::execute failed";
        return false;
    }
    MatrixXd rollout_costs(num_rollouts_, num_time_steps_);
    for (size_t r = 0; r < costs.size(); ++r) {
        if ((int)costs[r].size() != num_time_steps_) {
            error_ = "runSingleIteration: Task::execute returned the wrong number of costs";
            return false;
        }
        for (int t = 0; t < num_time_steps_; ++t) rollout_costs((int)r, t) = costs[r][t];
    }
    std::vector<double> all_costs;
    if (!policy_improvement_.setRolloutCosts(rollout_costs, control_cost_weight_, all_costs) ||
        !policy_improvement_.improvePolicy(parameter_updates_)) {
        error_ = policy_improvement_.lastError();
        return false;
    }
    if (!policy_->updateParameters(parameter_updates_) || !policy_->getParameters(parameters_)) {
        error_ = "runSingleIteration: policy update failed";
        return false;
    }
    // the noiseless rollout, then into the reuse pool (:180-192)
    VectorXd tmp_cost;
    if (!task_->execute(parameters_, tmp_cost, iteration_number)) {
        error_ = "runSingleIteration: noiseless Task::execute failed";
        return false;
    }
    std::vector<std::vector<VectorXd>> extra(1, parameters_);
    std::vector<VectorXd> extra_cost(1, tmp_cost);
    if (!policy_improvement_.addExtraRollouts(extra, extra_cost)) {
        error_ = policy_improvement_.lastError();
        return false;
    }
    return true;
}

}  // namespace stomp_motion_planner
