// stomp_facade.h -- C++ host API mirroring the reference's plugin/operator classes on the
// hot path, forwarding to the MI355X engine through the C ABI (stomp_engine.h).
//
// Paths below are relative to /root/reference/stomp_motion_planner/.  Names, argument
// meaning and the bool-return error convention follow the reference:
//   Task                       include/stomp_motion_planner/task.h:49-93
//   Policy                     include/stomp_motion_planner/policy.h:47-134
//   CovariantTrajectoryPolicy  include/stomp_motion_planner/covariant_trajectory_policy.h:56-146
//   PolicyImprovement          include/stomp_motion_planner/policy_improvement.h:65-126
//   PolicyImprovementLoop      include/stomp_motion_planner/policy_improvement_loop.h:52-98
//   StompOptimizer             include/stomp_motion_planner/stomp_optimizer.h:63-213
// What changes at the boundary (no ROS, Eigen 2, KDL or boost in this build):
//   * Eigen::VectorXd -> VectorXd (std::vector<double>); Eigen::MatrixXd -> MatrixXd below
//   * boost::shared_ptr -> std::shared_ptr; ros::NodeHandle arguments are dropped (the
//     values the reference reads from the parameter server arrive in StompParameters)
//   * the KDL tree / collision points / distance field arrive as plain tables
//     (StompRobotModel, StompCollisionSpace); orientation path constraints arrive as
//     Constraints; the ROS publishers are not taken (no visualisation)
//   * when the policy is a StompOptimizer's, the rollouts, the policy parameters and the
//     PolicyImprovement state live in HBM: in the optimizer's engine for its own counts, or, for
//     other counts (setNumRollouts) or another use_cumulative_costs, in a second engine of the
//     same problem on the same device; any other Policy (or more than one extra rollout) runs
//     PolicyImprovement on the host with the same arithmetic and noise stream
// Failures return false and leave the reason in lastError() (the reference logs with
// ROS_ERROR and returns false).  One optimizer owns one engine (one HIP device stream).
#ifndef STOMP_MOTION_PLANNER_STOMP_FACADE_H
#define STOMP_MOTION_PLANNER_STOMP_FACADE_H

#include <algorithm>
#include <cstdint>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "stomp_engine.h"

namespace stomp_motion_planner {

using VectorXd = std::vector<double>;

// Dense row-major matrix standing in for Eigen::MatrixXd at the API boundary.
struct MatrixXd {
    int rows_ = 0, cols_ = 0;
    std::vector<double> data_;
    MatrixXd() = default;
    MatrixXd(int r, int c) : rows_(r), cols_(c), data_((size_t)r * c, 0.0) {}
    int rows() const { return rows_; }
    int cols() const { return cols_; }
    double& operator()(int r, int c) { return data_[(size_t)r * cols_ + c]; }
    double operator()(int r, int c) const { return data_[(size_t)r * cols_ + c]; }
    void resize(int r, int c)
    {
        rows_ = r;
        cols_ = c;
        data_.assign((size_t)r * c, 0.0);
    }
};

namespace detail {
template <class M>
MatrixXd to_mat(const M& m)
{
    MatrixXd o((int)m.rows(), (int)m.cols());
    for (int r = 0; r < o.rows(); ++r)
        for (int c = 0; c < o.cols(); ++c) o(r, c) = m(r, c);
    return o;
}
template <class M>
void from_mat(const MatrixXd& s, M& m)
{
    m.resize(s.rows(), s.cols());
    for (int r = 0; r < s.rows(); ++r)
        for (int c = 0; c < s.cols(); ++c) m(r, c) = s(r, c);
}
}  // namespace detail

// Eigen-shaped arguments.  The reference's Task / Policy / PolicyImprovement calls pass
// Eigen::VectorXd and Eigen::MatrixXd; the template overloads below take any vector type with
// size(), data() and resize(n) (Eigen::VectorXd, std::vector<double>) and any matrix type with
// rows(), cols(), resize(r, c) and operator()(r, c) (Eigen::MatrixXd), so the node's calls compile
// unchanged against this header, which does not include Eigen.  The std::vector overloads are the
// exact matches for this header's own types.
namespace detail {
template <class V>
VectorXd to_vec(const V& v)
{
    return VectorXd(v.data(), v.data() + v.size());
}
template <class V>
void from_vec(const VectorXd& s, V& v)
{
    v.resize(s.size());
    std::copy(s.begin(), s.end(), v.data());
}
template <class V>
std::vector<VectorXd> to_vecs(const std::vector<V>& v)
{
    std::vector<VectorXd> o;
    o.reserve(v.size());
    for (const V& x : v) o.push_back(to_vec(x));
    return o;
}
template <class V>
void from_vecs(const std::vector<VectorXd>& s, std::vector<V>& v)
{
    v.resize(s.size());
    for (size_t i = 0; i < s.size(); ++i) from_vec(s[i], v[i]);
}
}  // namespace detail

// config/params.yaml + StompParameters (stomp_parameters.cpp:50-76)
struct StompParameters {
    double trajectory_duration = 5.0;
    double trajectory_discretization = 0.05;
    int max_iterations = 500;
    int max_iterations_after_collision_free = 100;
    double smoothness_cost_weight = 1e-6;
    double obstacle_cost_weight = 1.0;
    double constraint_cost_weight = 0.0;
    double torque_cost_weight = 0.0;
    double smoothness_cost_velocity = 0.0;
    double smoothness_cost_acceleration = 1.0;
    double smoothness_cost_jerk = 0.0;
    double ridge_factor = 0.0;
    bool use_cumulative_costs = false;
    int num_rollouts = 10;
    int num_reused_rollouts = 5;
    std::vector<double> noise_stddev;   // per joint (policy_improvement_loop.cpp:99-100)
    std::vector<double> noise_decay;    // per joint
    uint64_t seed = 0x53544F4D50000000ull;
};

// StompRobotModel::StompPlanningGroup as the engine needs it: the kinematic tree in DFS
// order, the planning-group joints and the collision points (stomp_robot_model.h).
struct StompRobotModel {
    std::vector<stomp_segment> segments;
    std::vector<stomp_joint> joints;          // planning-group joints, J
    std::vector<stomp_sphere> collision_points;
    // inverse dynamics of the torque term (stomp_robot_model.cpp:185-189): segment inertias
    // and the chain torque_root (exclusive) -> torque_tip (inclusive); needed only when
    // torque_cost_weight > 1e-9
    std::vector<stomp_inertia> inertias;      // per segment
    int torque_root = -1, torque_tip = -1;
    double gravity[3] = {0.0, 0.0, -9.8};
};

// motion_planning_msgs::Constraints as StompOptimizer consumes it (stomp_optimizer.cpp:195-201):
// orientation path constraints only
struct Constraints {
    std::vector<stomp_orientation_constraint> orientation_constraints;
};

// StompCollisionSpace's distance field (stomp_collision_space.h:187-191).
struct StompCollisionSpace {
    stomp_grid grid{};
};

// StompTrajectory restricted to what optimize() reads and writes: the start / goal
// configurations (the padding rows) and the free block, J x N row-major.
struct StompTrajectory {
    int num_joints = 0, num_points = 0;   // num_points = N free waypoints
    VectorXd start, goal;                 // J
    std::vector<VectorXd> free;           // [J] N: written by StompOptimizer::optimize()
};

class Policy {
public:
    virtual ~Policy() = default;
    virtual bool setNumTimeSteps(const int num_time_steps) = 0;
    virtual bool getNumTimeSteps(int& num_time_steps) = 0;
    virtual bool getNumDimensions(int& num_dimensions) = 0;
    virtual bool getNumParameters(std::vector<int>& num_params) = 0;
    virtual bool getBasisFunctions(std::vector<MatrixXd>& basis_functions) = 0;
    virtual bool getControlCosts(std::vector<MatrixXd>& control_costs) = 0;
    virtual bool updateParameters(const std::vector<MatrixXd>& updates) = 0;
    virtual bool getParameters(std::vector<VectorXd>& parameters) = 0;
    virtual bool setParameters(const std::vector<VectorXd>& parameters) = 0;
    // policy.h:128-131: control costs of time-varying parameters [J][T] N (summed over T), and of
    // one parameter set plus noise ([J] N each); weight multiplies every squared derivative
    virtual bool computeControlCosts(const std::vector<MatrixXd>& control_cost_matrices,
                                     const std::vector<std::vector<VectorXd>>& parameters, const double weight,
                                     std::vector<VectorXd>& control_costs) = 0;
    virtual bool computeControlCosts(const std::vector<MatrixXd>& control_cost_matrices,
                                     const std::vector<VectorXd>& parameters, const std::vector<VectorXd>& noise,
                                     const double weight, std::vector<VectorXd>& control_costs) = 0;
};

class StompOptimizer;

// The policy of one optimizer: theta lives in HBM inside the engine.
class CovariantTrajectoryPolicy : public Policy {
public:
    explicit CovariantTrajectoryPolicy(StompOptimizer* owner) : owner_(owner) {}
    bool setNumTimeSteps(const int num_time_steps) override;
    bool getNumTimeSteps(int& num_time_steps) override;
    bool getNumDimensions(int& num_dimensions) override;
    bool getNumParameters(std::vector<int>& num_params) override;
    bool getBasisFunctions(std::vector<MatrixXd>& basis_functions) override;
    bool getControlCosts(std::vector<MatrixXd>& control_costs) override;
    bool updateParameters(const std::vector<MatrixXd>& updates) override;
    bool getParameters(std::vector<VectorXd>& parameters) override;
    bool setParameters(const std::vector<VectorXd>& parameters) override;
    // covariant_trajectory_policy.cpp:228-304 on the host (the engine prices its own rollouts
    // inside the iteration): x = the padded trajectory (start / goal rows) with the free part
    // set, costs_all += (weight * derivative_cost_i) * (D_i x)^2, the padding costs folded
    // into the first / last free entries
    bool computeControlCosts(const std::vector<MatrixXd>& control_cost_matrices,
                             const std::vector<std::vector<VectorXd>>& parameters, const double weight,
                             std::vector<VectorXd>& control_costs) override;
    bool computeControlCosts(const std::vector<MatrixXd>& control_cost_matrices, const std::vector<VectorXd>& parameters,
                             const std::vector<VectorXd>& noise, const double weight,
                             std::vector<VectorXd>& control_costs) override;
    StompOptimizer* owner() const { return owner_; }
    // Eigen-shaped forms (see detail::): parameters [J] of N, updates [J] of N x N (row 0 used)
    template <class V>
    bool getParameters(std::vector<V>& parameters)
    {
        std::vector<VectorXd> p;
        if (!getParameters(p)) return false;
        detail::from_vecs(p, parameters);
        return true;
    }
    template <class V>
    bool setParameters(const std::vector<V>& parameters)
    {
        return setParameters(detail::to_vecs(parameters));
    }
    template <class M>
    bool updateParameters(const std::vector<M>& updates)
    {
        std::vector<MatrixXd> u;
        for (const M& m : updates) u.push_back(detail::to_mat(m));
        return updateParameters(u);
    }

private:
    bool loadDifferentiation();
    void accumulateCosts(int d, const VectorXd& free, const double weight, VectorXd& costs_all) const;
    StompOptimizer* owner_;
    std::vector<MatrixXd> D_;      // differentiation matrices (N+12)^2, covariant_trajectory_policy.cpp:204-226
};

class Task {
public:
    virtual ~Task() = default;
    virtual bool initialize(int num_time_steps) = 0;
    virtual bool execute(std::vector<VectorXd>& parameters, VectorXd& costs, const int iteration_number) = 0;
    virtual bool getPolicy(std::shared_ptr<Policy>& policy) = 0;
    virtual bool setPolicy(const std::shared_ptr<Policy> policy) = 0;
    virtual bool getControlCostWeight(double& control_cost_weight) = 0;
    // Not in the reference's Task: execute() of a batch of rollouts ([E][J] N -> [E] N), which
    // PolicyImprovementLoop calls; the default executes them one by one
    virtual bool executeBatch(std::vector<std::vector<VectorXd>>& parameters, std::vector<VectorXd>& costs,
                              const int iteration_number);
};

// Adapter bases for plugins written against the reference's own signatures.  The virtuals of Task
// and Policy above take this header's VectorXd / MatrixXd; a Task or Policy written for the
// reference overrides virtuals taking Eigen::VectorXd / Eigen::MatrixXd (task.h:62-91,
// policy.h:59-132) and a ros::NodeHandle in Task::initialize.  Deriving such a class from
// TaskT<Eigen::VectorXd, ros::NodeHandle> or PolicyT<Eigen::VectorXd, Eigen::MatrixXd> instead of
// Task / Policy lets it compile unchanged: the adapters declare the reference's virtuals with those
// types (Vector: size(), data(), resize(n); Matrix: rows(), cols(), resize(r, c), operator()(r, c);
// NodeHandle: default-constructible, passed as a fresh object since no parameter server exists
// here) and implement the facade's virtuals by converting and forwarding.  The policy pointers stay
// std::shared_ptr (boost::shared_ptr in the reference, see the file header).
template <class Vector, class NodeHandle>
class TaskT : public Task {
    static_assert(!std::is_same<Vector, VectorXd>::value, "TaskT<VectorXd> is Task itself");

public:
    // task.h:62 and :70 with the caller's types
    virtual bool initialize(NodeHandle& node_handle, int num_time_steps) = 0;
    virtual bool execute(std::vector<Vector>& parameters, Vector& costs, const int iteration_number) = 0;

    bool initialize(int num_time_steps) final
    {
        NodeHandle nh{};
        return initialize(nh, num_time_steps);
    }
    bool execute(std::vector<VectorXd>& parameters, VectorXd& costs, const int iteration_number) final
    {
        std::vector<Vector> p;
        detail::from_vecs(parameters, p);
        Vector c;
        if (!execute(p, c, iteration_number)) return false;
        // task.h:70 takes parameters by non-const reference and the loop keeps what execute left
        // there as the extra rollout (policy_improvement_loop.cpp:182-190): a plugin's in-place
        // edits come back
        parameters = detail::to_vecs(p);
        costs = detail::to_vec(c);
        return true;
    }
};

template <class Vector, class Matrix>
class PolicyT : public Policy {
    static_assert(!std::is_same<Vector, VectorXd>::value && !std::is_same<Matrix, MatrixXd>::value,
                  "PolicyT<VectorXd, MatrixXd> is Policy itself");

public:
    // policy.h:91-132 with the caller's types (the int-valued virtuals are Policy's own)
    virtual bool getBasisFunctions(std::vector<Matrix>& basis_functions) = 0;
    virtual bool getControlCosts(std::vector<Matrix>& control_costs) = 0;
    virtual bool updateParameters(const std::vector<Matrix>& updates) = 0;
    virtual bool getParameters(std::vector<Vector>& parameters) = 0;
    virtual bool setParameters(const std::vector<Vector>& parameters) = 0;
    virtual bool computeControlCosts(const std::vector<Matrix>& control_cost_matrices,
                                     const std::vector<std::vector<Vector>>& parameters, const double weight,
                                     std::vector<Vector>& control_costs) = 0;
    virtual bool computeControlCosts(const std::vector<Matrix>& control_cost_matrices,
                                     const std::vector<Vector>& parameters, const std::vector<Vector>& noise,
                                     const double weight, std::vector<Vector>& control_costs) = 0;

    bool getBasisFunctions(std::vector<MatrixXd>& basis_functions) final
    {
        std::vector<Matrix> b;
        if (!getBasisFunctions(b)) return false;
        basis_functions = mats(b);
        return true;
    }
    bool getControlCosts(std::vector<MatrixXd>& control_costs) final
    {
        std::vector<Matrix> c;
        if (!getControlCosts(c)) return false;
        control_costs = mats(c);
        return true;
    }
    bool updateParameters(const std::vector<MatrixXd>& updates) final { return updateParameters(unmats(updates)); }
    bool getParameters(std::vector<VectorXd>& parameters) final
    {
        std::vector<Vector> p;
        if (!getParameters(p)) return false;
        parameters = detail::to_vecs(p);
        return true;
    }
    bool setParameters(const std::vector<VectorXd>& parameters) final
    {
        std::vector<Vector> p;
        detail::from_vecs(parameters, p);
        return setParameters(p);
    }
    bool computeControlCosts(const std::vector<MatrixXd>& control_cost_matrices,
                             const std::vector<std::vector<VectorXd>>& parameters, const double weight,
                             std::vector<VectorXd>& control_costs) final
    {
        std::vector<std::vector<Vector>> p(parameters.size());
        for (size_t d = 0; d < parameters.size(); ++d) detail::from_vecs(parameters[d], p[d]);
        std::vector<Vector> c;
        if (!computeControlCosts(unmats(control_cost_matrices), p, weight, c)) return false;
        control_costs = detail::to_vecs(c);
        return true;
    }
    bool computeControlCosts(const std::vector<MatrixXd>& control_cost_matrices, const std::vector<VectorXd>& parameters,
                             const std::vector<VectorXd>& noise, const double weight,
                             std::vector<VectorXd>& control_costs) final
    {
        std::vector<Vector> p, n, c;
        detail::from_vecs(parameters, p);
        detail::from_vecs(noise, n);
        if (!computeControlCosts(unmats(control_cost_matrices), p, n, weight, c)) return false;
        control_costs = detail::to_vecs(c);
        return true;
    }

private:
    static std::vector<MatrixXd> mats(const std::vector<Matrix>& m)
    {
        std::vector<MatrixXd> o;
        o.reserve(m.size());
        for (const Matrix& x : m) o.push_back(detail::to_mat(x));
        return o;
    }
    static std::vector<Matrix> unmats(const std::vector<MatrixXd>& m)
    {
        std::vector<Matrix> o(m.size());
        for (size_t i = 0; i < m.size(); ++i) detail::from_mat(m[i], o[i]);
        return o;
    }
};

struct STOMPStatistics {   // msg/STOMPStatistics.msg without the ROS header
    int iterations = 0;
    bool success = false;
    int success_iteration = -1;
    double success_duration = 0.0;             // seconds from the loop's start (device wall clock)
    int collision_success_iteration = -1;
    double collision_success_duration = 0.0;
    int last_improvement_iteration = -1;
    double best_cost = 0.0;
    std::vector<double> costs;     // last_trajectory_cost_ per iteration
    std::vector<double> torques;   // per free waypoint, sum |tau| of the best trajectory (empty without inertias)
};

class StompOptimizer : public Task {
public:
    // stomp_optimizer.cpp:50-70 (the ROS publishers are not taken, see the file header)
    StompOptimizer(StompTrajectory* trajectory, const StompRobotModel* robot_model, const StompParameters* parameters,
                   StompCollisionSpace* collision_space, const Constraints& constraints = Constraints(),
                   int device = 0, void* stream = nullptr);
    // the planner node's call shape (stomp_planner_node.cpp:228-230: trajectory, robot model,
    // planning group, parameters, the visualisation / marker / statistics publishers, collision
    // space, path constraints): the group and the publishers are taken and ignored (the robot
    // model passed here is already the planning group's; nothing is visualised)
    template <class Group, class Publisher>
    StompOptimizer(StompTrajectory* trajectory, const StompRobotModel* robot_model, const Group* /*planning_group*/,
                   const StompParameters* parameters, const Publisher& /*vis_marker_array_publisher*/,
                   const Publisher& /*vis_marker_publisher*/, const Publisher& /*stats_publisher*/,
                   StompCollisionSpace* collision_space, const Constraints& constraints = Constraints())
        : StompOptimizer(trajectory, robot_model, parameters, collision_space, constraints)
    {
    }
    ~StompOptimizer() override;
    StompOptimizer(const StompOptimizer&) = delete;
    StompOptimizer& operator=(const StompOptimizer&) = delete;

    // stomp_optimizer.cpp:249-401: runs the loop, writes best_group_trajectory_ back into
    // the caller's trajectory; false if the engine failed (the reference returns void)
    bool optimize();
    const STOMPStatistics& getStatistics() const { return stats_; }

    // Task (stomp_optimizer.cpp:1063-1165, 1167-1182)
    bool initialize(int num_time_steps) override;
    bool execute(std::vector<VectorXd>& parameters, VectorXd& costs, const int iteration_number) override;
    bool getPolicy(std::shared_ptr<Policy>& policy) override;
    bool setPolicy(const std::shared_ptr<Policy> policy) override;
    bool getControlCostWeight(double& control_cost_weight) override;
    // Task::execute with Eigen-shaped vectors (task.h:70)
    template <class V>
    bool execute(std::vector<V>& parameters, V& costs, const int iteration_number)
    {
        std::vector<VectorXd> p = detail::to_vecs(parameters);
        VectorXd c;
        if (!execute(p, c, iteration_number)) return false;
        detail::from_vec(c, costs);
        return true;
    }
    // the reference's setSharedPtr / resetSharedPtr (stomp_optimizer.cpp:1202-1210): the loop here
    // holds no owning pointer to its task, so these are no-ops kept for the node's call sequence
    void setSharedPtr(const std::shared_ptr<StompOptimizer>& /*self*/) {}
    void resetSharedPtr() {}

    // batched Task::execute: parameters [E][J] N -> costs [E] N (one engine launch)
    bool executeBatch(std::vector<std::vector<VectorXd>>& parameters, std::vector<VectorXd>& costs,
                      const int iteration_number) override;
    // ... and the collision flags
    bool executeBatch(const std::vector<std::vector<VectorXd>>& parameters, std::vector<VectorXd>& costs,
                      std::vector<bool>& collision_free, const int iteration_number);

    bool ok() const { return engine_ != nullptr; }
    const std::string& lastError() const { return error_; }
    stomp_engine* engine() { return engine_; }
    int numJoints() const { return J_; }
    int numTimeSteps() const { return N_; }

    // last_trajectory_cost_ / last_trajectory_collision_free_ after runSingleIteration
    double lastTrajectoryCost() const { return last_cost_; }
    bool lastTrajectoryCollisionFree() const { return last_cf_; }
    bool lastTrajectoryConstraintsSatisfied() const { return last_cs_; }

    const StompParameters& parameters() const { return *parameters_; }
    const StompTrajectory& trajectory() const { return *trajectory_; }

private:
    friend class PolicyImprovementLoop;
    friend class PolicyImprovement;
    friend class CovariantTrajectoryPolicy;
    bool check(int rc);
    // an engine of the same problem with other rollout counts / cumulative-cost setting (the
    // device rollout set of a PolicyImprovement that asks for them); nullptr and err on failure
    stomp_engine* createSibling(int num_rollouts, int num_reused_rollouts, bool use_cumulative_costs,
                                std::string& err) const;
    StompTrajectory* trajectory_;
    const StompParameters* parameters_;
    // the engine's descriptor, kept for createSibling: its tables point into the copies below,
    // taken at construction (the caller may resize or reassign its vectors afterwards).  The
    // distance field is the one exception: grid.data stays the caller's buffer, which must
    // outlive the optimizer as the collision space does in the reference (StompOptimizer keeps
    // its collision_space_ pointer, stomp_optimizer.cpp:61); a sibling uploads its own copy
    stomp_engine_desc desc_{};
    Constraints constraints_;           // desc_.orientation_constraints points here
    std::vector<stomp_segment> segments_;
    std::vector<stomp_joint> joints_;
    std::vector<stomp_sphere> spheres_;
    std::vector<stomp_inertia> inertias_;
    std::vector<double> noise_stddev_, noise_decay_, start_, goal_;
    stomp_engine* engine_ = nullptr;
    std::shared_ptr<Policy> policy_;
    int J_ = 0, N_ = 0;
    double last_cost_ = 0.0;
    bool last_cf_ = false;
    bool last_cs_ = true;
    STOMPStatistics stats_;
    std::string error_;
};

// policy_improvement.h:65-126 / policy_improvement.cpp:64-489.  Where the rollout set lives,
// with the same results:
//   * when the policy is a StompOptimizer's CovariantTrajectoryPolicy, on the device (stomp_pi_* of
//     the C ABI): in that optimizer's engine for its own counts and use_cumulative_costs, else in
//     a second engine of the same problem made for the requested counts / setting (initialize,
//     setNumRollouts), whose theta is refreshed from the optimizer's before each getRollouts;
//   * the host, for any other Policy or more than one extra rollout (the engine evaluates one
//     noiseless extra rollout): the reference's algorithm over the Policy interface (getControlCosts ->
//     R^-1, chol, projection; computeControlCosts; getParameters), with the engine's noise stream
//     (Philox normals keyed by seed, iteration, dimension, rollout) and arithmetic contract (fma
//     chains for L z and M eps, 64-rollout blocked sums, deterministic exp).
// The policy's num_parameters must equal num_time_steps in every dimension (identity basis, as
// computeParameterUpdates' noise .* probabilities requires).
class PolicyImprovement {
public:
    PolicyImprovement();
    ~PolicyImprovement();
    PolicyImprovement(const PolicyImprovement&) = delete;
    PolicyImprovement& operator=(const PolicyImprovement&) = delete;
    bool initialize(const int num_rollouts, const int num_time_steps, const int num_reused_rollouts,
                    const int num_extra_rollouts, std::shared_ptr<Policy> policy, bool use_cumulative_costs = true);
    // policy_improvement.cpp:96-147: new counts, the reuse state reset (the next getRollouts
    // generates every rollout); counts the engine was not created with move the rollout set to
    // the host
    bool setNumRollouts(const int num_rollouts, const int num_reused_rollouts, const int num_extra_rollouts);
    // the K_gen new rollouts [K_gen][J] N; noise_stddev per joint
    bool getRollouts(std::vector<std::vector<VectorXd>>& rollouts, const std::vector<double>& noise_stddev);
    // costs: num_rollouts x N state costs (rows >= K_gen ignored); totals: Rollout::getCost of all K
    bool setRolloutCosts(const MatrixXd& costs, const double control_cost_weight,
                         std::vector<double>& rollout_costs_total);
    // [J] N x N matrices, row 0 = the update (policy_improvement.cpp:370-383)
    bool improvePolicy(std::vector<MatrixXd>& parameter_updates);
    bool addExtraRollouts(std::vector<std::vector<VectorXd>>& rollouts, std::vector<VectorXd>& rollout_costs);
    // the same four calls with Eigen-shaped vectors / matrices (policy_improvement.h:86-126)
    template <class V>
    bool getRollouts(std::vector<std::vector<V>>& rollouts, const std::vector<double>& noise_stddev)
    {
        std::vector<std::vector<VectorXd>> r;
        if (!getRollouts(r, noise_stddev)) return false;
        rollouts.resize(r.size());
        for (size_t i = 0; i < r.size(); ++i) detail::from_vecs(r[i], rollouts[i]);
        return true;
    }
    template <class M>
    bool setRolloutCosts(const M& costs, const double control_cost_weight, std::vector<double>& rollout_costs_total)
    {
        return setRolloutCosts(detail::to_mat(costs), control_cost_weight, rollout_costs_total);
    }
    template <class M>
    bool improvePolicy(std::vector<M>& parameter_updates)
    {
        std::vector<MatrixXd> u;
        if (!improvePolicy(u)) return false;
        parameter_updates.resize(u.size());
        for (size_t i = 0; i < u.size(); ++i) detail::from_mat(u[i], parameter_updates[i]);
        return true;
    }
    template <class V>
    bool addExtraRollouts(std::vector<std::vector<V>>& rollouts, std::vector<V>& rollout_costs)
    {
        std::vector<std::vector<VectorXd>> r;
        for (const auto& x : rollouts) r.push_back(detail::to_vecs(x));
        std::vector<VectorXd> c = detail::to_vecs(rollout_costs);
        return addExtraRollouts(r, c);
    }
    // The noise of getRollouts is a counter-based stream keyed by an iteration number (the
    // reference's generators are stateful); each getRollouts uses the current key and advances
    // it by one, starting at 1.  PolicyImprovementLoop sets it to runSingleIteration's number.
    void setNoiseIteration(int iteration) { noise_iteration_ = iteration; }
    // the noise key of the host rollout set (the engine's comes from StompParameters::seed;
    // a StompOptimizer's policy sets it from there)
    void setNoiseSeed(uint64_t seed) { seed_ = seed; }
    // true while the rollout set lives on the device (the optimizer's engine or one of its own)
    bool onEngine() const { return engine_ != nullptr && !host_; }
    // true when that device rollout set is an engine of this PolicyImprovement's own (other counts)
    bool onOwnEngine() const { return onEngine() && engine_ == own_; }
    const std::string& lastError() const { return error_; }

private:
    struct HostRollouts;
    bool check(int rc);
    bool hostInitialize(int num_rollouts, int num_reused_rollouts, int num_extra_rollouts);
    std::shared_ptr<Policy> policy_;
    StompOptimizer* owner_ = nullptr;
    stomp_engine* engine_ = nullptr;
    stomp_engine* own_ = nullptr;       // the second engine (counts other than the optimizer's)
    std::shared_ptr<HostRollouts> host_;
    uint64_t seed_ = 0x53544F4D50000000ull;
    int J_ = 0, N_ = 0, K_ = 0, K_gen_ = 0, noise_iteration_ = 1;
    bool use_cumulative_ = false;
    bool initialized_ = false;
    std::string error_;
};

// policy_improvement_loop.cpp:88-202.  Drives any Task: getRollouts, Task::executeBatch,
// setRolloutCosts, improvePolicy, updateParameters, the noiseless execute and addExtraRollouts,
// as the reference does.  When the task is a StompOptimizer the whole iteration runs as the
// engine's fused launch sequence instead (stomp_engine_iterate, bit-identical results), unless
// setUseFusedIteration(false).  The loop parameters (rollout counts, noise schedule) are the
// ones of the StompOptimizer that owns the task's policy, or, for a task whose policy is not a
// StompOptimizer's, the StompParameters given to initialize (the reference reads the same
// params.yaml values from the node handle, policy_improvement_loop.cpp:112-123).
class PolicyImprovementLoop {
public:
    bool initialize(std::shared_ptr<Task> task);
    bool initialize(std::shared_ptr<Task> task, const StompParameters& parameters);
    bool runSingleIteration(int iteration_number);
    void setUseFusedIteration(bool on) { fused_ = on; }
    const std::string& lastError() const { return error_; }

private:
    bool runGeneric(int iteration_number);
    std::shared_ptr<Task> task_;
    std::shared_ptr<Policy> policy_;
    StompOptimizer* optimizer_ = nullptr;   // the task, when it is a StompOptimizer
    StompOptimizer* owner_ = nullptr;       // the optimizer owning the policy
    PolicyImprovement policy_improvement_;
    bool fused_ = true;
    int num_rollouts_ = 0, num_time_steps_ = 0;
    std::vector<double> noise_stddev_, noise_decay_;
    double control_cost_weight_ = 0.0;
    std::vector<std::vector<VectorXd>> rollouts_;
    std::vector<MatrixXd> parameter_updates_;
    std::vector<VectorXd> parameters_;
    std::string error_;
};

}  // namespace stomp_motion_planner

#endif
