// stomp_facade.cpp -- reference-shaped C++ classes over the engine's C ABI.
// See include/stomp_motion_planner/stomp_facade.h for the mapping to the reference.
#include "stomp_motion_planner/stomp_facade.h"

#include <cmath>
#include <cstdio>

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
    stomp_engine_desc d{};
    d.abi_version = STOMP_ENGINE_ABI_VERSION;
    d.num_joints = J_;
    d.num_time_steps = N_;
    d.num_rollouts = p.num_rollouts;
    d.num_reused_rollouts = p.num_reused_rollouts;
    d.num_segments = (int32_t)robot_model->segments.size();
    d.segments = robot_model->segments.data();
    d.num_spheres = (int32_t)robot_model->collision_points.size();
    d.spheres = robot_model->collision_points.data();
    d.joints = robot_model->joints.data();
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
    d.noise_stddev = p.noise_stddev.data();
    d.noise_decay = p.noise_decay.data();
    d.use_cumulative_costs = p.use_cumulative_costs ? 1 : 0;
    d.start = trajectory->start.data();
    d.goal = trajectory->goal.data();
    d.seed = p.seed;
    d.max_iterations = p.max_iterations;
    d.max_iterations_after_collision_free = p.max_iterations_after_collision_free;
    d.device = device;
    d.stream = stream;
    d.rank = 0;
    d.world_size = 1;
    d.inertias = robot_model->inertias.size() == robot_model->segments.size() ? robot_model->inertias.data() : nullptr;
    d.torque_root = robot_model->torque_root;
    d.torque_tip = robot_model->torque_tip;
    for (int k = 0; k < 3; ++k) d.gravity[k] = robot_model->gravity[k];
    d.num_orientation_constraints = (int32_t)constraints.orientation_constraints.size();
    d.orientation_constraints = constraints.orientation_constraints.data();
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
// row products run over the stencil's band (the other entries of D_i are exact zeros)
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
    auto* ctp = dynamic_cast<CovariantTrajectoryPolicy*>(policy.get());
    if (!ctp || !ctp->owner() || !ctp->owner()->ok()) {
        error_ = "PolicyImprovement::initialize: the policy must be a StompOptimizer's CovariantTrajectoryPolicy";
        return false;
    }
    owner_ = ctp->owner();
    engine_ = owner_->engine_;
    policy_ = policy;
    J_ = owner_->J_;
    N_ = owner_->N_;
    K_ = owner_->parameters_->num_rollouts;
    if (num_time_steps != N_) {
        error_ = "PolicyImprovement::initialize: num_time_steps differs from the engine's";
        return false;
    }
    if (use_cumulative_costs != owner_->parameters_->use_cumulative_costs) {
        error_ = "PolicyImprovement::initialize: use_cumulative_costs differs from the engine's";
        return false;
    }
    if (!setNumRollouts(num_rollouts, num_reused_rollouts, num_extra_rollouts)) return false;
    noise_iteration_ = 1;
    return (initialized_ = true);
}

bool PolicyImprovement::setNumRollouts(const int num_rollouts, const int num_reused_rollouts,
                                       const int num_extra_rollouts)
{
    if (num_reused_rollouts >= num_rollouts) {   // policy_improvement.cpp:102-106
        error_ = "Number of reused rollouts must be strictly less than number of rollouts.";
        return false;
    }
    if (!owner_ || num_rollouts != K_ || num_reused_rollouts != owner_->parameters_->num_reused_rollouts ||
        num_extra_rollouts != 1) {
        error_ = "setNumRollouts: the engine's rollout counts are fixed at creation (and one extra rollout)";
        return false;
    }
    return true;
}

bool PolicyImprovement::getRollouts(std::vector<std::vector<VectorXd>>& rollouts,
                                    const std::vector<double>& noise_stddev)
{
    if (!initialized_) { error_ = "getRollouts: not initialized"; return false; }
    if ((int)noise_stddev.size() != J_) { error_ = "getRollouts: one noise_stddev per dimension"; return false; }
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

bool PolicyImprovement::setRolloutCosts(const MatrixXd& costs, const double control_cost_weight,
                                        std::vector<double>& rollout_costs_total)
{
    if (!initialized_) { error_ = "setRolloutCosts: not initialized"; return false; }
    if (costs.cols() != N_ || costs.rows() < K_gen_) {
        error_ = "setRolloutCosts: costs must be num_rollouts x num_time_steps";
        return false;
    }
    std::vector<double> c((size_t)K_ * N_, 0.0);
    for (int r = 0; r < K_gen_; ++r)
        for (int t = 0; t < N_; ++t) c[(size_t)r * N_ + t] = costs(r, t);
    rollout_costs_total.assign(K_, 0.0);
    return check(stomp_pi_set_rollout_costs(engine_, c.data(), control_cost_weight, rollout_costs_total.data()));
}

bool PolicyImprovement::improvePolicy(std::vector<MatrixXd>& parameter_updates)
{
    if (!initialized_) { error_ = "improvePolicy: not initialized"; return false; }
    std::vector<double> u((size_t)J_ * N_);
    if (!check(stomp_pi_improve_policy(engine_, u.data()))) return false;
    parameter_updates.assign(J_, MatrixXd(N_, N_));
    for (int d = 0; d < J_; ++d)
        for (int t = 0; t < N_; ++t) parameter_updates[d](0, t) = u[(size_t)d * N_ + t];
    return true;
}

bool PolicyImprovement::addExtraRollouts(std::vector<std::vector<VectorXd>>& rollouts,
                                         std::vector<VectorXd>& rollout_costs)
{
    if (!initialized_) { error_ = "addExtraRollouts: not initialized"; return false; }
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
        error_ = "PolicyImprovementLoop::initialize: the task's policy must be a StompOptimizer's "
                 "CovariantTrajectoryPolicy";
        return false;
    }
    owner_ = ctp->owner();
    optimizer_ = dynamic_cast<StompOptimizer*>(task.get());
    task_ = task;
    policy_ = policy;
    // readParameters (policy_improvement_loop.cpp:112-123) from the optimizer's parameters
    const StompParameters& p = *owner_->parameters_;
    num_rollouts_ = p.num_rollouts;
    num_time_steps_ = owner_->N_;
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
    if (!fused_ || !optimizer_ || optimizer_ != owner_) return runGeneric(iteration_number);
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
