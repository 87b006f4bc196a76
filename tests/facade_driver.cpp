// facade_driver.cpp -- drives the C++ facade (include/stomp_motion_planner/stomp_facade.h)
// the way the reference's planner node drives StompOptimizer (stomp_planner_node.cpp:228-234)
// and the way optimize() drives PolicyImprovementLoop (stomp_optimizer.cpp:262-293).
//
// usage: facade_driver <problem.txt> <sdf.bin> <mode> [out.txt]
//   mode validate : argument checks only (no device needed)
//   mode optimize : StompOptimizer::optimize(), writes stats, costs and the best trajectory
//   mode loop     : PolicyImprovementLoop::runSingleIteration 1..10, writes cost and theta
// The problem file is whitespace-separated text written by tests/facade_util.py.
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
    std::vector<float> sdf;
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
    if (!f) return false;
    p.sdf.resize((size_t)n * n * n);
    std::ifstream b(sdf_path, std::ios::binary);
    b.read(reinterpret_cast<char*>(p.sdf.data()), p.sdf.size() * sizeof(float));
    if (!b) return false;
    g.data = p.sdf.data();
    g.data_on_device = 0;
    return true;
}

void write_vec(FILE* out, const std::vector<double>& v)
{
    for (double x : v) std::fprintf(out, "%.17g\n", x);
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
        std::fprintf(out, "%d %d %d %d %d %.17g\n", st.iterations, st.success ? 1 : 0, st.success_iteration,
                     st.collision_success_iteration, st.last_improvement_iteration, st.best_cost);
        write_vec(out, st.costs);
        for (const auto& row : p.traj.free) write_vec(out, row);
    } else if (mode == "loop") {
        PolicyImprovementLoop loop;
        if (!loop.initialize(opt)) {
            std::cerr << loop.lastError() << "\n";
            return 8;
        }
        std::shared_ptr<Policy> policy;
        opt->getPolicy(policy);
        for (int it = 1; it <= 10; ++it) {
            if (!loop.runSingleIteration(it)) {
                std::cerr << loop.lastError() << "\n";
                return 9;
            }
            std::vector<VectorXd> theta;
            policy->getParameters(theta);
            std::fprintf(out, "%.17g %d\n", opt->lastTrajectoryCost(), opt->lastTrajectoryCollisionFree() ? 1 : 0);
            for (const auto& row : theta) write_vec(out, row);
        }
    } else {
        return 2;
    }
    std::fclose(out);
    return 0;
}
