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
// The problem file is whitespace-separated text written by tests/facade_util.py.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
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

int main(int argc, char** argv)
{
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
