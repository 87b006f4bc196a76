// facade_driver.cpp -- drives the C++ facade (include/stomp_motion_planner/stomp_facade.h)
// the way the reference's planner node drives StompOptimizer (stomp_planner_node.cpp:228-234)
// and the way optimize() drives PolicyImprovementLoop (stomp_optimizer.cpp:262-293).
//
// usage: facade_driver <problem.txt> <sdf.bin> <mode> [out.txt] [in.txt]
//   mode validate      : argument checks only (no device needed)
//   mode optimize      : StompOptimizer::optimize(), writes stats, costs, torques and the best trajectory
//   mode loop          : PolicyImprovementLoop::runSingleIteration 1..10 (fused engine iteration),
//                        writes cost and theta
//   mode generic_loop  : the same loop over a user Task (ForwardingTask below), which takes the
//                        step-by-step PolicyImprovement path with per-rollout Task::execute
//   mode unfused_loop  : the StompOptimizer task with setUseFusedIteration(false)
//   mode pi_steps      : PolicyImprovement driven by hand as policy_improvement_loop.cpp:143-202
//                        does, plus the rollout totals of every setRolloutCosts
//   mode control_costs : both Policy::computeControlCosts overloads on parameters / noise read
//                        from in.txt
//   mode pi_user       : PolicyImprovementLoop over a user Policy (UserPolicy: theta on the host)
//                        and a user Task (forwarding to the optimizer's execute): the host
//                        PolicyImprovement path; writes cost and theta per iteration
//   mode pi_setnum     : pi_steps after setNumRollouts(K, K_r + delta, 1) on the optimizer's policy
//                        (in.txt: the new K_r): counts the engine was not created with
//   mode pi_host_cpu   : the host PolicyImprovement with a synthetic policy and task, no device
//                        (the sanitizer build runs it)
// The problem file is whitespace-separated text written by tests/facade_util.py.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "stomp_motion_planner/stomp_facade.h"

using namespace stomp_motion_planner;

namespace {

struct Problem {
    StompParameters params;
    StompRobotModel robot;
    StompTrajectory traj;
    StompCollisionSpace space;
    std::vector<uint16_t> sdf;   // d2 per voxel
};

bool load(const char* path, const char* sdf_path, Problem& p)
{
    std::ifstream f(path);
    if (!f) return false;
    int J, N, nseg, nsph, n;
    f >> J >> N >> nseg >> nsph >> n;
    p.traj.num_joints = J;
    p.traj.num_points = N;
    p.robot.segments.resize(nseg);
    for (auto& s : p.robot.segments) {
        f >> s.parent >> s.q_index;
        for (double& v : s.rot) f >> v;
        for (double& v : s.trans) f >> v;
        for (double& v : s.axis) f >> v;
    }
    p.robot.collision_points.resize(nsph);
    for (auto& s : p.robot.collision_points) {
        f >> s.segment >> s.radius >> s.clearance;
        for (double& v : s.pos) f >> v;
    }
    p.robot.joints.resize(J);
    for (auto& j : p.robot.joints) f >> j.has_limits >> j.min >> j.max >> j.joint_cost;
    p.traj.start.resize(J);
    p.traj.goal.resize(J);
    for (double& v : p.traj.start) f >> v;
    for (double& v : p.traj.goal) f >> v;
    StompParameters& q = p.params;
    q.noise_stddev.resize(J);
    q.noise_decay.resize(J);
    for (double& v : q.noise_stddev) f >> v;
    for (double& v : q.noise_decay) f >> v;
    int cum;
    f >> q.trajectory_discretization >> q.max_iterations >> q.max_iterations_after_collision_free >>
        q.smoothness_cost_weight >> q.obstacle_cost_weight >> q.smoothness_cost_velocity >>
        q.smoothness_cost_acceleration >> q.smoothness_cost_jerk >> q.ridge_factor >> cum >> q.num_rollouts >>
        q.num_reused_rollouts >> q.seed;
    q.use_cumulative_costs = cum != 0;
    stomp_grid& g = p.space.grid;
    g.nx = g.ny = g.nz = n;
    f >> g.origin[0] >> g.origin[1] >> g.origin[2] >> g.resolution;
    f >> p.robot.torque_root >> p.robot.torque_tip >> p.robot.gravity[0] >> p.robot.gravity[1] >> p.robot.gravity[2];
    p.robot.inertias.resize(nseg);
    for (auto& in : p.robot.inertias) {
        f >> in.mass;
        for (double& v : in.com) f >> v;
        for (double& v : in.inertia) f >> v;
    }
    if (!f) return false;
    p.sdf.resize((size_t)n * n * n);
    std::ifstream b(sdf_path, std::ios::binary);
    b.read(reinterpret_cast<char*>(p.sdf.data()), p.sdf.size() * sizeof(uint16_t));
    if (!b) return false;
    g.data = p.sdf.data();
    g.data_on_device = 0;
    return true;
}

void write_vec(FILE* out, const std::vector<double>& v)
{
    for (double x : v) std::fprintf(out, "%.17g\n", x);
}

// A Task that is not a StompOptimizer: it forwards to one (e.g. a wrapper adding logging or
// cost shaping in a user's planner).  PolicyImprovementLoop cannot take the engine's fused
// iteration for it and runs the reference's step-by-step loop.
class ForwardingTask : public Task {
public:
    explicit ForwardingTask(std::shared_ptr<StompOptimizer> o) : o_(std::move(o)) {}
    bool initialize(int num_time_steps) override { return o_->initialize(num_time_steps); }
    bool execute(std::vector<VectorXd>& parameters, VectorXd& costs, const int iteration_number) override
    {
        ++executions;
        return o_->execute(parameters, costs, iteration_number);
    }
    bool getPolicy(std::shared_ptr<Policy>& policy) override { return o_->getPolicy(policy); }
    bool setPolicy(const std::shared_ptr<Policy> policy) override { return o_->setPolicy(policy); }
    bool getControlCostWeight(double& w) override { return o_->getControlCostWeight(w); }
    int executions = 0;

private:
    std::shared_ptr<StompOptimizer> o_;
};

// A user's Policy: CovariantTrajectoryPolicy written against the Policy interface with theta on
// the host (covariant_trajectory_policy.cpp:168-342): R and the stencil matrices D_i come from the
// optimizer's policy / engine once, then everything runs here.
class UserPolicy : public Policy {
public:
    UserPolicy(StompOptimizer& opt, const StompTrajectory& tr, const StompParameters& q)
        : J_(opt.numJoints()), N_(opt.numTimeSteps()), start_(tr.start), goal_(tr.goal)
    {
        std::shared_ptr<Policy> ctp;
        opt.getPolicy(ctp);
        ok_ = ctp->getControlCosts(R_) && ctp->getParameters(theta_);
        const int A = N_ + 12;
        const char* names[3] = {"D0", "D1", "D2"};
        for (int i = 0; i < 3 && ok_; ++i) {
            D_[i] = MatrixXd(A, A);
            ok_ = stomp_engine_get_matrix(opt.engine(), names[i], 0, D_[i].data_.data()) == 0;
        }
        w_[0] = q.smoothness_cost_velocity;
        w_[1] = q.smoothness_cost_acceleration;
        w_[2] = q.smoothness_cost_jerk;
    }
    bool ok() const { return ok_; }
    bool setNumTimeSteps(const int n) override { return n == N_; }
    bool getNumTimeSteps(int& n) override { n = N_; return true; }
    bool getNumDimensions(int& d) override { d = J_; return true; }
    bool getNumParameters(std::vector<int>& np) override { np.assign(J_, N_); return true; }
    bool getBasisFunctions(std::vector<MatrixXd>& b) override
    {
        MatrixXd I(N_, N_);
        for (int i = 0; i < N_; ++i) I(i, i) = 1.0;
        b.assign(J_, I);
        return true;
    }
    bool getControlCosts(std::vector<MatrixXd>& c) override { c = R_; return true; }
    bool updateParameters(const std::vector<MatrixXd>& u) override
    {
        if ((int)u.size() != J_) return false;
        for (int d = 0; d < J_; ++d)
            for (int t = 0; t < N_; ++t) theta_[d][t] += u[d](0, t) / 1.0;
        return true;
    }
    bool getParameters(std::vector<VectorXd>& p) override { p = theta_; return true; }
    bool setParameters(const std::vector<VectorXd>& p) override { theta_ = p; return true; }
    bool computeControlCosts(const std::vector<MatrixXd>&, const std::vector<std::vector<VectorXd>>&, const double,
                             std::vector<VectorXd>&) override
    {
        return false;   // not used by PolicyImprovement
    }
    bool computeControlCosts(const std::vector<MatrixXd>&, const std::vector<VectorXd>& parameters,
                             const std::vector<VectorXd>& noise, const double weight,
                             std::vector<VectorXd>& costs) override
    {
        const int A = N_ + 12;
        costs.assign(J_, VectorXd(N_));
        for (int d = 0; d < J_; ++d) {
            VectorXd x(A), all(A, 0.0);
            for (int i = 0; i < A; ++i)
                x[i] = i < 6 ? start_[d] : (i >= 6 + N_ ? goal_[d] : parameters[d][i - 6] + noise[d][i - 6]);
            for (int r = 0; r < 3; ++r) {
                const double w = weight * w_[r];
                for (int i = 0; i < A; ++i) {
                    double acc = 0.0;
                    for (int c = std::max(i - 3, 0); c <= std::min(i + 3, A - 1); ++c) acc += D_[r](i, c) * x[c];
                    all[i] += w * (acc * acc);
                }
            }
            for (int t = 0; t < N_; ++t) costs[d][t] = all[t + 6];
            for (int i = 0; i < 6; ++i) {
                costs[d][0] += all[i];
                costs[d][N_ - 1] += all[A - (i + 1)];
            }
        }
        return true;
    }

private:
    int J_, N_;
    VectorXd start_, goal_;
    std::vector<MatrixXd> R_;
    MatrixXd D_[3];
    double w_[3];
    std::vector<VectorXd> theta_;
    bool ok_ = false;
};

// A user's Task over that policy: the state costs from the optimizer (stomp_optimizer.cpp:1063-1165)
class UserTask : public Task {
public:
    UserTask(std::shared_ptr<StompOptimizer> o, std::shared_ptr<Policy> p) : o_(std::move(o)), p_(std::move(p)) {}
    bool initialize(int n) override { return o_->initialize(n); }
    bool execute(std::vector<VectorXd>& parameters, VectorXd& costs, const int it) override
    {
        return o_->execute(parameters, costs, it);
    }
    bool executeBatch(std::vector<std::vector<VectorXd>>& parameters, std::vector<VectorXd>& costs,
                      const int it) override
    {
        return o_->executeBatch(parameters, costs, it);
    }
    bool getPolicy(std::shared_ptr<Policy>& policy) override { policy = p_; return true; }
    bool setPolicy(const std::shared_ptr<Policy> policy) override { p_ = policy; return true; }
    bool getControlCostWeight(double& w) override { return o_->getControlCostWeight(w); }

private:
    std::shared_ptr<StompOptimizer> o_;
    std::shared_ptr<Policy> p_;
};

// A synthetic policy / task pair with no device: R = tridiagonal (2, -1) + I per dimension,
// control cost weight * x^2, state cost (x - 1)^2 summed over dimensions
class ToyPolicy : public Policy {
public:
    ToyPolicy(int J, int N) : J_(J), N_(N), theta_(J, VectorXd(N, 0.0)) {}
    bool setNumTimeSteps(const int n) override { return n == N_; }
    bool getNumTimeSteps(int& n) override { n = N_; return true; }
    bool getNumDimensions(int& d) override { d = J_; return true; }
    bool getNumParameters(std::vector<int>& np) override { np.assign(J_, N_); return true; }
    bool getBasisFunctions(std::vector<MatrixXd>& b) override { b.assign(J_, MatrixXd(N_, N_)); return true; }
    bool getControlCosts(std::vector<MatrixXd>& c) override
    {
        MatrixXd R(N_, N_);
        for (int i = 0; i < N_; ++i) {
            R(i, i) = 3.0;
            if (i > 0) R(i, i - 1) = -1.0;
            if (i + 1 < N_) R(i, i + 1) = -1.0;
        }
        c.assign(J_, R);
        return true;
    }
    bool updateParameters(const std::vector<MatrixXd>& u) override
    {
        for (int d = 0; d < J_; ++d)
            for (int t = 0; t < N_; ++t) theta_[d][t] += u[d](0, t);
        return true;
    }
    bool getParameters(std::vector<VectorXd>& p) override { p = theta_; return true; }
    bool setParameters(const std::vector<VectorXd>& p) override { theta_ = p; return true; }
    bool computeControlCosts(const std::vector<MatrixXd>&, const std::vector<std::vector<VectorXd>>&, const double,
                             std::vector<VectorXd>&) override
    {
        return false;
    }
    bool computeControlCosts(const std::vector<MatrixXd>&, const std::vector<VectorXd>& prm,
                             const std::vector<VectorXd>& nz, const double w, std::vector<VectorXd>& c) override
    {
        c.assign(J_, VectorXd(N_));
        for (int d = 0; d < J_; ++d)
            for (int t = 0; t < N_; ++t) {
                const double x = prm[d][t] + nz[d][t];
                c[d][t] = w * x * x;
            }
        return true;
    }

private:
    int J_, N_;
    std::vector<VectorXd> theta_;
};

class ToyTask : public Task {
public:
    explicit ToyTask(std::shared_ptr<Policy> p) : p_(std::move(p)) {}
    bool initialize(int) override { return true; }
    bool execute(std::vector<VectorXd>& prm, VectorXd& costs, const int) override
    {
        const int N = (int)prm[0].size();
        costs.assign(N, 0.0);
        for (const VectorXd& row : prm)
            for (int t = 0; t < N; ++t) costs[t] += (row[t] - 1.0) * (row[t] - 1.0);
        return true;
    }
    bool getPolicy(std::shared_ptr<Policy>& p) override { p = p_; return true; }
    bool setPolicy(const std::shared_ptr<Policy> p) override { p_ = p; return true; }
    bool getControlCostWeight(double& w) override { w = 1e-3; return true; }

private:
    std::shared_ptr<Policy> p_;
};

int run_loop(PolicyImprovementLoop& loop, StompOptimizer& opt, std::shared_ptr<Policy> policy, FILE* out)
{
    for (int it = 1; it <= 10; ++it) {
        if (!loop.runSingleIteration(it)) {
            std::cerr << loop.lastError() << "\n";
            return 9;
        }
        std::vector<VectorXd> theta;
        policy->getParameters(theta);
        std::fprintf(out, "%.17g %d\n", opt.lastTrajectoryCost(), opt.lastTrajectoryCollisionFree() ? 1 : 0);
        for (const auto& row : theta) write_vec(out, row);
    }
    return 0;
}

}  // namespace

// Stand-ins with the member names of Eigen::VectorXd / Eigen::MatrixXd that the facade's template
// overloads use (size, data, resize, operator()), and of the node's planning group / ROS
// publisher arguments: the node's own calls, type-checked and run through the Eigen-shaped API
struct EigenLikeVector {
    std::vector<double> v;
    long size() const { return (long)v.size(); }
    const double* data() const { return v.data(); }
    double* data() { return v.data(); }
    void resize(long n) { v.assign((size_t)n, 0.0); }
    double& operator()(long i) { return v[(size_t)i]; }
    double operator()(long i) const { return v[(size_t)i]; }
};
struct EigenLikeMatrix {
    long r = 0, c = 0;
    std::vector<double> d;
    long rows() const { return r; }
    long cols() const { return c; }
    void resize(long rr, long cc) { r = rr; c = cc; d.assign((size_t)(rr * cc), 0.0); }
    double& operator()(long i, long j) { return d[(size_t)(i * c + j)]; }
    double operator()(long i, long j) const { return d[(size_t)(i * c + j)]; }
};
struct NodePlanningGroup {};
struct NodePublisher {};
struct NodeHandleLike {};   // ros::NodeHandle's place in Task::initialize (task.h:62)

// UserPolicy written as a reference plugin: the overrides take the Eigen-shaped types of
// policy.h:59-132 (here the stand-ins), through the PolicyT adapter
class EigenUserPolicy : public PolicyT<EigenLikeVector, EigenLikeMatrix> {
public:
    EigenUserPolicy(StompOptimizer& opt, const StompTrajectory& tr, const StompParameters& q)
        : J_(opt.numJoints()), N_(opt.numTimeSteps()), start_(tr.start), goal_(tr.goal)
    {
        std::shared_ptr<Policy> ctp;
        opt.getPolicy(ctp);
        std::vector<MatrixXd> R;
        std::vector<VectorXd> th;
        ok_ = ctp->getControlCosts(R) && ctp->getParameters(th);
        R_.resize(R.size());
        for (size_t d = 0; d < R.size(); ++d) {
            R_[d].resize(R[d].rows(), R[d].cols());
            R_[d].d = R[d].data_;
        }
        theta_.resize(th.size());
        for (size_t d = 0; d < th.size(); ++d) theta_[d].v = th[d];
        const int A = N_ + 12;
        const char* names[3] = {"D0", "D1", "D2"};
        for (int i = 0; i < 3 && ok_; ++i) {
            D_[i].resize(A, A);
            ok_ = stomp_engine_get_matrix(opt.engine(), names[i], 0, D_[i].d.data()) == 0;
        }
        w_[0] = q.smoothness_cost_velocity;
        w_[1] = q.smoothness_cost_acceleration;
        w_[2] = q.smoothness_cost_jerk;
    }
    bool ok() const { return ok_; }
    bool setNumTimeSteps(const int n) override { return n == N_; }
    bool getNumTimeSteps(int& n) override { n = N_; return true; }
    bool getNumDimensions(int& d) override { d = J_; return true; }
    bool getNumParameters(std::vector<int>& np) override { np.assign(J_, N_); return true; }
    bool getBasisFunctions(std::vector<EigenLikeMatrix>& b) override
    {
        b.assign(J_, EigenLikeMatrix());
        for (auto& m : b) {
            m.resize(N_, N_);
            for (int i = 0; i < N_; ++i) m(i, i) = 1.0;
        }
        return true;
    }
    bool getControlCosts(std::vector<EigenLikeMatrix>& c) override { c = R_; return true; }
    bool updateParameters(const std::vector<EigenLikeMatrix>& u) override
    {
        if ((int)u.size() != J_) return false;
        for (int d = 0; d < J_; ++d)
            for (int t = 0; t < N_; ++t) theta_[d](t) += u[d](0, t) / 1.0;
        return true;
    }
    bool getParameters(std::vector<EigenLikeVector>& p) override { p = theta_; return true; }
    bool setParameters(const std::vector<EigenLikeVector>& p) override { theta_ = p; return true; }
    bool computeControlCosts(const std::vector<EigenLikeMatrix>&, const std::vector<std::vector<EigenLikeVector>>&,
                             const double, std::vector<EigenLikeVector>&) override
    {
        return false;   // not used by PolicyImprovement
    }
    bool computeControlCosts(const std::vector<EigenLikeMatrix>&, const std::vector<EigenLikeVector>& parameters,
                             const std::vector<EigenLikeVector>& noise, const double weight,
                             std::vector<EigenLikeVector>& costs) override
    {
        const int A = N_ + 12;
        costs.assign(J_, EigenLikeVector());
        for (int d = 0; d < J_; ++d) {
            costs[d].resize(N_);
            std::vector<double> x(A), all(A, 0.0);
            for (int i = 0; i < A; ++i)
                x[i] = i < 6 ? start_[d] : (i >= 6 + N_ ? goal_[d] : parameters[d](i - 6) + noise[d](i - 6));
            for (int r = 0; r < 3; ++r) {
                const double w = weight * w_[r];
                for (int i = 0; i < A; ++i) {
                    double acc = 0.0;
                    for (int c = std::max(i - 3, 0); c <= std::min(i + 3, A - 1); ++c) acc += D_[r](i, c) * x[c];
                    all[i] += w * (acc * acc);
                }
            }
            for (int t = 0; t < N_; ++t) costs[d](t) = all[t + 6];
            for (int i = 0; i < 6; ++i) {
                costs[d](0) += all[i];
                costs[d](N_ - 1) += all[A - (i + 1)];
            }
        }
        return true;
    }

private:
    int J_, N_;
    VectorXd start_, goal_;
    std::vector<EigenLikeMatrix> R_;
    EigenLikeMatrix D_[3];
    double w_[3];
    std::vector<EigenLikeVector> theta_;
    bool ok_ = false;
};

// UserTask written as a reference plugin (task.h:62-91: the node handle, Eigen-shaped execute),
// through the TaskT adapter
class EigenUserTask : public TaskT<EigenLikeVector, NodeHandleLike> {
public:
    EigenUserTask(std::shared_ptr<StompOptimizer> o, std::shared_ptr<Policy> p) : o_(std::move(o)), p_(std::move(p)) {}
    bool initialize(NodeHandleLike& /*node_handle*/, int num_time_steps) override
    {
        return o_->initialize(num_time_steps);
    }
    bool execute(std::vector<EigenLikeVector>& parameters, EigenLikeVector& costs, const int iteration_number) override
    {
        ++executions;
        return o_->execute(parameters, costs, iteration_number);   // the optimizer's Eigen-shaped overload
    }
    bool getPolicy(std::shared_ptr<Policy>& policy) override { policy = p_; return true; }
    bool setPolicy(const std::shared_ptr<Policy> policy) override { p_ = policy; return true; }
    bool getControlCostWeight(double& w) override { return o_->getControlCostWeight(w); }
    int executions = 0;

private:
    std::shared_ptr<StompOptimizer> o_;
    std::shared_ptr<Policy> p_;
};

// a reference-signature plugin that edits its parameters in place (task.h:70 takes them by
// non-const reference): clamps every value to [-1, 1] and prices the clamped rows
class ClampingTask : public TaskT<EigenLikeVector, NodeHandleLike> {
public:
    bool initialize(NodeHandleLike&, int) override { return true; }
    bool execute(std::vector<EigenLikeVector>& parameters, EigenLikeVector& costs, const int) override
    {
        costs.resize(parameters.empty() ? 0 : parameters[0].size());
        for (auto& row : parameters)
            for (long i = 0; i < row.size(); ++i) {
                row(i) = std::min(1.0, std::max(-1.0, row(i)));
                costs(i) += row(i);
            }
        return true;
    }
    bool getPolicy(std::shared_ptr<Policy>&) override { return false; }
    bool setPolicy(const std::shared_ptr<Policy>) override { return false; }
    bool getControlCostWeight(double& w) override { w = 0.0; return true; }
};

int main(int argc, char** argv)
{
    if (argc >= 2 && std::string(argv[1]) == "taskt_writeback") {
        // TaskT::execute hands the plugin's in-place edits back through the facade's Task (no device)
        ClampingTask t;
        Task& base = t;
        std::vector<VectorXd> prm = {{-2.0, 0.5, 3.0}, {0.25, -7.0, 1.0}};
        VectorXd c;
        if (!base.execute(prm, c, 1)) return 60;
        const double want[2][3] = {{-1.0, 0.5, 1.0}, {0.25, -1.0, 1.0}};
        for (int d = 0; d < 2; ++d)
            for (int i = 0; i < 3; ++i)
                if (prm[d][i] != want[d][i]) {
                    std::cerr << "row " << d << " entry " << i << ": " << prm[d][i] << " expected " << want[d][i] << "\n";
                    return 61;
                }
        if (c.size() != 3 || c[0] != -0.75 || c[1] != -0.5 || c[2] != 2.0) return 62;
        std::cout << "taskt_writeback OK\n";
        return 0;
    }
    if (argc < 4) {
        std::cerr << "usage: facade_driver problem.txt sdf.bin validate|optimize|loop [out]\n";
        return 2;
    }
    Problem p;
    if (!load(argv[1], argv[2], p)) {
        std::cerr << "cannot read problem\n";
        return 2;
    }
    const std::string mode = argv[3];
    if (mode == "pi_host_cpu") {
        // the host PolicyImprovement end to end without a device; the loop must reduce the cost
        const int J = 3, N = 20;
        auto policy = std::make_shared<ToyPolicy>(J, N);
        auto task = std::make_shared<ToyTask>(policy);
        StompParameters q;
        q.num_rollouts = 70;   // two 64-rollout summation blocks
        q.num_reused_rollouts = 7;
        q.noise_stddev.assign(J, 0.5);
        q.noise_decay.assign(J, 0.99);
        PolicyImprovementLoop loop;
        if (!loop.initialize(task, q)) {
            std::cerr << loop.lastError() << "\n";
            return 20;
        }
        auto cost = [&]() {
            std::vector<VectorXd> th;
            policy->getParameters(th);
            VectorXd c;
            task->execute(th, c, 0);
            double s = 0.0;
            for (double v : c) s += v;
            return s;
        };
        const double c0 = cost();
        for (int it = 1; it <= 30; ++it)
            if (!loop.runSingleIteration(it)) {
                std::cerr << loop.lastError() << "\n";
                return 21;
            }
        const double c1 = cost();
        if (!(c1 < 0.5 * c0)) {
            std::cerr << "host PolicyImprovement did not reduce the cost: " << c0 << " -> " << c1 << "\n";
            return 22;
        }
        std::cout << "pi_host_cpu OK " << c0 << " -> " << c1 << "\n";
        return 0;
    }
    if (mode == "validate") {
        // one noise_stddev entry short: the reference would read past the end
        // (policy_improvement_loop.cpp:99-100); the facade refuses
        Problem bad = p;
        bad.params.noise_stddev.pop_back();
        StompOptimizer o1(&bad.traj, &bad.robot, &bad.params, &bad.space);
        if (o1.ok() || o1.lastError().find("noise_stddev") == std::string::npos) return 3;
        // reused >= rollouts: PolicyImprovement::setNumRollouts refuses (policy_improvement.cpp:102-106)
        Problem bad2 = p;
        bad2.params.num_reused_rollouts = bad2.params.num_rollouts;
        StompOptimizer o2(&bad2.traj, &bad2.robot, &bad2.params, &bad2.space);
        if (o2.ok() || o2.lastError().find("error -1") == std::string::npos) return 4;
        PolicyImprovementLoop loop;
        if (loop.initialize(std::shared_ptr<Task>()) || loop.runSingleIteration(1)) return 5;
        std::cout << "validate OK\n";
        return 0;
    }
    if (argc < 5) return 2;
    FILE* out = std::fopen(argv[4], "w");
    if (!out) return 2;
    auto opt = std::make_shared<StompOptimizer>(&p.traj, &p.robot, &p.params, &p.space);
    if (!opt->ok()) {
        std::cerr << opt->lastError() << "\n";
        return 6;
    }
    if (mode == "optimize") {
        if (!opt->optimize()) {
            std::cerr << opt->lastError() << "\n";
            return 7;
        }
        const STOMPStatistics& st = opt->getStatistics();
        std::fprintf(out, "%d %d %d %d %d %.17g %.17g %.17g %zu\n", st.iterations, st.success ? 1 : 0,
                     st.success_iteration, st.collision_success_iteration, st.last_improvement_iteration,
                     st.best_cost, st.success_duration, st.collision_success_duration, st.torques.size());
        write_vec(out, st.costs);
        write_vec(out, st.torques);
        for (const auto& row : p.traj.free) write_vec(out, row);
    } else if (mode == "loop" || mode == "unfused_loop") {
        PolicyImprovementLoop loop;
        loop.setUseFusedIteration(mode == "loop");
        if (!loop.initialize(opt)) {
            std::cerr << loop.lastError() << "\n";
            return 8;
        }
        std::shared_ptr<Policy> policy;
        opt->getPolicy(policy);
        if (int rc = run_loop(loop, *opt, policy, out)) return rc;
    } else if (mode == "generic_loop") {
        auto task = std::make_shared<ForwardingTask>(opt);
        PolicyImprovementLoop loop;
        if (!loop.initialize(task)) {
            std::cerr << loop.lastError() << "\n";
            return 8;
        }
        std::shared_ptr<Policy> policy;
        task->getPolicy(policy);
        if (int rc = run_loop(loop, *opt, policy, out)) return rc;
        // every generated rollout and every noiseless rollout went through Task::execute
        const int gen = p.params.num_rollouts + 9 * (p.params.num_rollouts - p.params.num_reused_rollouts);
        if (task->executions != gen + 10) {
            std::cerr << "executions " << task->executions << " expected " << gen + 10 << "\n";
            return 10;
        }
    } else if (mode == "pi_steps") {
        // policy_improvement_loop.cpp:143-202 written out against PolicyImprovement / Policy / Task
        std::shared_ptr<Policy> policy;
        opt->getPolicy(policy);
        PolicyImprovement pi;
        const StompParameters& q = p.params;
        if (!pi.initialize(q.num_rollouts, p.traj.num_points, q.num_reused_rollouts, 1, policy,
                           q.use_cumulative_costs)) {
            std::cerr << pi.lastError() << "\n";
            return 11;
        }
        double w = 0.0;
        opt->getControlCostWeight(w);
        const int J = p.traj.num_joints, N = p.traj.num_points;
        for (int it = 1; it <= 10; ++it) {
            std::vector<double> noise(J);
            for (int i = 0; i < J; ++i) noise[i] = q.noise_stddev[i] * std::pow(q.noise_decay[i], it - 1);
            std::vector<std::vector<VectorXd>> rollouts;
            if (!pi.getRollouts(rollouts, noise)) { std::cerr << pi.lastError() << "\n"; return 12; }
            MatrixXd costs(q.num_rollouts, N);
            for (size_t r = 0; r < rollouts.size(); ++r) {
                VectorXd c;
                if (!opt->execute(rollouts[r], c, it)) return 13;
                for (int t = 0; t < N; ++t) costs((int)r, t) = c[t];
            }
            std::vector<double> totals;
            std::vector<MatrixXd> updates;
            if (!pi.setRolloutCosts(costs, w, totals) || !pi.improvePolicy(updates)) {
                std::cerr << pi.lastError() << "\n";
                return 14;
            }
            if (!policy->updateParameters(updates)) return 15;
            std::vector<VectorXd> theta;
            policy->getParameters(theta);
            VectorXd c;
            if (!opt->execute(theta, c, it)) return 16;
            std::vector<std::vector<VectorXd>> extra(1, theta);
            std::vector<VectorXd> extra_cost(1, c);
            if (!pi.addExtraRollouts(extra, extra_cost)) { std::cerr << pi.lastError() << "\n"; return 17; }
            std::fprintf(out, "%.17g %d %zu\n", opt->lastTrajectoryCost(), opt->lastTrajectoryCollisionFree() ? 1 : 0,
                         rollouts.size());
            for (const auto& row : theta) write_vec(out, row);
            write_vec(out, totals);
        }
    } else if (mode == "pi_steps_eigen") {
        // pi_steps with Eigen-shaped arguments and the node's constructor call shape
        // (stomp_planner_node.cpp:228-234)
        NodePlanningGroup group;
        NodePublisher pub;
        auto node_opt = std::make_shared<StompOptimizer>(&p.traj, &p.robot, &group, &p.params, pub, pub, pub, &p.space,
                                                         Constraints());
        node_opt->setSharedPtr(node_opt);
        if (!node_opt->ok()) return 40;
        std::shared_ptr<Policy> policy;
        node_opt->getPolicy(policy);
        auto* ctp = dynamic_cast<CovariantTrajectoryPolicy*>(policy.get());
        PolicyImprovement pi;
        const StompParameters& q = p.params;
        if (!ctp || !pi.initialize(q.num_rollouts, p.traj.num_points, q.num_reused_rollouts, 1, policy,
                                   q.use_cumulative_costs)) {
            std::cerr << pi.lastError() << "\n";
            return 41;
        }
        double w = 0.0;
        node_opt->getControlCostWeight(w);
        const int J = p.traj.num_joints, N = p.traj.num_points;
        for (int it = 1; it <= 10; ++it) {
            std::vector<double> noise(J);
            for (int i = 0; i < J; ++i) noise[i] = q.noise_stddev[i] * std::pow(q.noise_decay[i], it - 1);
            std::vector<std::vector<EigenLikeVector>> rollouts;
            if (!pi.getRollouts(rollouts, noise)) { std::cerr << pi.lastError() << "\n"; return 42; }
            EigenLikeMatrix costs;
            costs.resize(q.num_rollouts, N);
            for (size_t r = 0; r < rollouts.size(); ++r) {
                EigenLikeVector c;
                if (!node_opt->execute(rollouts[r], c, it)) return 43;
                for (int t = 0; t < N; ++t) costs((long)r, t) = c(t);
            }
            std::vector<double> totals;
            std::vector<EigenLikeMatrix> updates;
            if (!pi.setRolloutCosts(costs, w, totals) || !pi.improvePolicy(updates)) {
                std::cerr << pi.lastError() << "\n";
                return 44;
            }
            if (!ctp->updateParameters(updates)) return 45;
            std::vector<EigenLikeVector> theta;
            ctp->getParameters(theta);
            EigenLikeVector c;
            if (!node_opt->execute(theta, c, it)) return 46;
            std::vector<std::vector<EigenLikeVector>> extra(1, theta);
            std::vector<EigenLikeVector> extra_cost(1, c);
            if (!pi.addExtraRollouts(extra, extra_cost)) { std::cerr << pi.lastError() << "\n"; return 47; }
            std::fprintf(out, "%.17g %d %zu\n", node_opt->lastTrajectoryCost(),
                         node_opt->lastTrajectoryCollisionFree() ? 1 : 0, rollouts.size());
            for (const auto& row : theta) write_vec(out, row.v);
            write_vec(out, totals);
        }
        node_opt->resetSharedPtr();
    } else if (mode == "pi_user") {
        auto policy = std::make_shared<UserPolicy>(*opt, p.traj, p.params);
        if (!policy->ok()) return 23;
        auto task = std::make_shared<UserTask>(opt, policy);
        PolicyImprovementLoop loop;
        if (!loop.initialize(task, p.params)) {
            std::cerr << loop.lastError() << "\n";
            return 24;
        }
        if (int rc = run_loop(loop, *opt, policy, out)) return rc;
    } else if (mode == "pi_user_eigen") {
        // pi_user with the plugins written in the reference's signatures (TaskT / PolicyT)
        auto policy = std::make_shared<EigenUserPolicy>(*opt, p.traj, p.params);
        if (!policy->ok()) return 50;
        auto task = std::make_shared<EigenUserTask>(opt, policy);
        PolicyImprovementLoop loop;
        if (!loop.initialize(task, p.params)) {
            std::cerr << loop.lastError() << "\n";
            return 51;
        }
        if (int rc = run_loop(loop, *opt, policy, out)) return rc;
        // every generated rollout and every noiseless rollout went through the Eigen-shaped execute
        const int gen = p.params.num_rollouts + 9 * (p.params.num_rollouts - p.params.num_reused_rollouts);
        if (task->executions != gen + 10) {
            std::cerr << "executions " << task->executions << " expected " << gen + 10 << "\n";
            return 52;
        }
    } else if (mode == "pi_setnum") {
        // input: K_r for setNumRollouts, and 1 to initialize with the other use_cumulative_costs
        // than the optimizer's (policy_improvement.cpp:64-147): either way the rollout set stays
        // on the device, in an engine of the PolicyImprovement's own
        if (argc < 6) return 2;
        int kr = 0, flip = 0;
        std::ifstream f(argv[5]);
        f >> kr >> flip;
        if (!f) return 2;
        // the caller's tables move after construction (same values, new storage; the old storage
        // kept alive and overwritten): the engines made later for the PolicyImprovement
        // (createSibling) must read the optimizer's own copies, not the caller's old buffers
        std::vector<std::shared_ptr<void>> graveyard;
        auto reseat = [&](auto& v) {
            using V = std::decay_t<decltype(v)>;
            V saved = v;
            for (auto& x : v) std::memset((void*)&x, 0x7f, sizeof x);
            auto old = std::make_shared<V>();
            old->swap(v);
            graveyard.push_back(old);
            v = saved;
        };
        reseat(p.robot.segments);
        reseat(p.robot.joints);
        reseat(p.robot.collision_points);
        reseat(p.robot.inertias);
        reseat(p.params.noise_stddev);
        reseat(p.params.noise_decay);
        reseat(p.traj.start);
        reseat(p.traj.goal);
        std::shared_ptr<Policy> policy;
        opt->getPolicy(policy);
        PolicyImprovement pi;
        const StompParameters& q = p.params;
        const bool cum = flip ? !q.use_cumulative_costs : q.use_cumulative_costs;
        if (!pi.initialize(q.num_rollouts, p.traj.num_points, q.num_reused_rollouts, 1, policy, cum) ||
            !pi.onEngine() || pi.onOwnEngine() != (flip != 0)) {
            std::cerr << "initialize: " << pi.lastError() << "\n";
            return 25;
        }
        if (!pi.setNumRollouts(q.num_rollouts, kr, 1) || !pi.onEngine() ||
            pi.onOwnEngine() != (flip != 0 || kr != q.num_reused_rollouts)) {
            std::cerr << "setNumRollouts: " << pi.lastError() << "\n";
            return 26;
        }
        double w = 0.0;
        opt->getControlCostWeight(w);
        const int J = p.traj.num_joints, N = p.traj.num_points;
        for (int it = 1; it <= 10; ++it) {
            std::vector<double> noise(J);
            for (int i = 0; i < J; ++i) noise[i] = q.noise_stddev[i] * std::pow(q.noise_decay[i], it - 1);
            pi.setNoiseIteration(it);
            std::vector<std::vector<VectorXd>> rollouts;
            if (!pi.getRollouts(rollouts, noise)) { std::cerr << pi.lastError() << "\n"; return 27; }
            MatrixXd costs(q.num_rollouts, N);
            std::vector<VectorXd> c;
            if (!opt->executeBatch(rollouts, c, it)) return 28;
            for (size_t r = 0; r < rollouts.size(); ++r)
                for (int t = 0; t < N; ++t) costs((int)r, t) = c[r][t];
            std::vector<double> totals;
            std::vector<MatrixXd> updates;
            if (!pi.setRolloutCosts(costs, w, totals) || !pi.improvePolicy(updates)) {
                std::cerr << pi.lastError() << "\n";
                return 29;
            }
            if (!policy->updateParameters(updates)) return 30;
            std::vector<VectorXd> theta;
            policy->getParameters(theta);
            VectorXd cx;
            if (!opt->execute(theta, cx, it)) return 31;
            std::vector<std::vector<VectorXd>> extra(1, theta);
            std::vector<VectorXd> extra_cost(1, cx);
            if (!pi.addExtraRollouts(extra, extra_cost)) { std::cerr << pi.lastError() << "\n"; return 32; }
            std::fprintf(out, "%.17g %d %zu\n", opt->lastTrajectoryCost(), opt->lastTrajectoryCollisionFree() ? 1 : 0,
                         rollouts.size());
            for (const auto& row : theta) write_vec(out, row);
            write_vec(out, totals);
        }
    } else if (mode == "control_costs") {
        // in.txt: J x N parameters, then J x N noise
        if (argc < 6) return 2;
        std::ifstream f(argv[5]);
        const int J = p.traj.num_joints, N = p.traj.num_points;
        std::vector<VectorXd> prm(J, VectorXd(N)), nz(J, VectorXd(N));
        for (auto& row : prm) for (double& v : row) f >> v;
        for (auto& row : nz) for (double& v : row) f >> v;
        if (!f) return 2;
        std::shared_ptr<Policy> policy;
        opt->getPolicy(policy);
        std::vector<MatrixXd> R;
        policy->getControlCosts(R);
        double w = 0.0;
        opt->getControlCostWeight(w);
        std::vector<VectorXd> c1, c2;
        // the per-rollout overload as computeRolloutControlCosts calls it (policy_improvement.cpp:484-489)
        if (!policy->computeControlCosts(R, prm, nz, 0.5 * w, c1)) return 18;
        // the time-varying overload: three time steps, parameters, parameters + noise, noise
        std::vector<std::vector<VectorXd>> tv(J, std::vector<VectorXd>(3, VectorXd(N)));
        for (int d = 0; d < J; ++d)
            for (int t = 0; t < N; ++t) {
                tv[d][0][t] = prm[d][t];
                tv[d][1][t] = prm[d][t] + nz[d][t];
                tv[d][2][t] = nz[d][t];
            }
        if (!policy->computeControlCosts(R, tv, w, c2)) return 19;
        for (const auto& row : c1) write_vec(out, row);
        for (const auto& row : c2) write_vec(out, row);
    } else {
        return 2;
    }
    std::fclose(out);
    return 0;
}
