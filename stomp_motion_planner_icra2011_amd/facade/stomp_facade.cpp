// stomp_facade.cpp -- reference-shaped C++ classes over the engine's C ABI.
// See include/stomp_motion_planner/stomp_facade.h for the mapping to the reference.
#include "stomp_motion_planner/stomp_facade.h"

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
    stats_.costs.resize(st.iterations);
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
    return true;
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

// ------------------------------------------------------------------ PolicyImprovementLoop

bool PolicyImprovementLoop::initialize(std::shared_ptr<Task> task)
{
    optimizer_ = dynamic_cast<StompOptimizer*>(task.get());
    if (!optimizer_ || !optimizer_->ok()) {
        error_ = "PolicyImprovementLoop::initialize: the task must be a constructed StompOptimizer";
        optimizer_ = nullptr;
        return false;
    }
    task_ = task;
    return true;
}

bool PolicyImprovementLoop::runSingleIteration(int iteration_number)
{
    if (!optimizer_) {
        error_ = "runSingleIteration: not initialized";
        return false;
    }
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

}  // namespace stomp_motion_planner
