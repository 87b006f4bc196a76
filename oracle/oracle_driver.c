/*
 * oracle/oracle_driver.c -- TEST INFRASTRUCTURE: a standalone C driver of the CPU oracle, so the
 * oracle can be built and run under AddressSanitizer + UndefinedBehaviorSanitizer
 * ("CPU oracle built with -fsanitize=address,undefined"; oracle/Makefile
 * target `sanitize`, run by tests/test_sanitizers.py).  Never part of the product.
 *
 * usage: oracle_driver <problem.txt> <sdf.bin> <out.txt> [threads]
 * The problem file is the text format tests/facade_util.py writes for tests/facade_driver.cpp.
 * The driver runs StompOptimizer::optimize (so_optimize, stomp_optimizer.cpp:249-401), then
 * three more PolicyImprovementLoop iterations (so_iterate, policy_improvement_loop.cpp:143-202)
 * and Task::execute of the first four current rollouts (so_execute, stomp_optimizer.cpp:
 * 1063-1165), and prints every result with %.17g so the caller can compare it bit for bit with
 * the uninstrumented oracle.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "stomp_oracle.h"

static int rd_i(FILE* f, int* v) { return fscanf(f, "%d", v) == 1; }
static int rd_d(FILE* f, double* v) { return fscanf(f, "%lf", v) == 1; }

#define TRY(x)                                              \
    do {                                                    \
        if (!(x)) {                                         \
            fprintf(stderr, "bad problem file: %s\n", #x);  \
            return 2;                                       \
        }                                                   \
    } while (0)

int main(int argc, char** argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: oracle_driver problem.txt sdf.bin out.txt [threads]\n");
        return 2;
    }
    FILE* f = fopen(argv[1], "r");
    if (!f) return 2;
    int J, N, nseg, nsph, n;
    TRY(rd_i(f, &J) && rd_i(f, &N) && rd_i(f, &nseg) && rd_i(f, &nsph) && rd_i(f, &n));
    so_segment* seg = calloc((size_t)nseg, sizeof *seg);
    so_sphere* sph = calloc((size_t)nsph, sizeof *sph);
    so_joint* jnt = calloc((size_t)J, sizeof *jnt);
    so_inertia* inr = calloc((size_t)nseg, sizeof *inr);
    double* start = calloc((size_t)J, sizeof(double));
    double* goal = calloc((size_t)J, sizeof(double));
    double* sd = calloc((size_t)J, sizeof(double));
    double* dc = calloc((size_t)J, sizeof(double));
    for (int s = 0; s < nseg; ++s) {
        TRY(rd_i(f, &seg[s].parent) && rd_i(f, &seg[s].q_index));
        for (int k = 0; k < 9; ++k) TRY(rd_d(f, &seg[s].rot[k]));
        for (int k = 0; k < 3; ++k) TRY(rd_d(f, &seg[s].trans[k]));
        for (int k = 0; k < 3; ++k) TRY(rd_d(f, &seg[s].axis[k]));
    }
    for (int s = 0; s < nsph; ++s) {
        TRY(rd_i(f, &sph[s].segment) && rd_d(f, &sph[s].radius) && rd_d(f, &sph[s].clearance));
        for (int k = 0; k < 3; ++k) TRY(rd_d(f, &sph[s].pos[k]));
    }
    for (int j = 0; j < J; ++j)
        TRY(rd_i(f, &jnt[j].has_limits) && rd_d(f, &jnt[j].min) && rd_d(f, &jnt[j].max) &&
            rd_d(f, &jnt[j].joint_cost));
    for (int j = 0; j < J; ++j) TRY(rd_d(f, &start[j]));
    for (int j = 0; j < J; ++j) TRY(rd_d(f, &goal[j]));
    for (int j = 0; j < J; ++j) TRY(rd_d(f, &sd[j]));
    for (int j = 0; j < J; ++j) TRY(rd_d(f, &dc[j]));
    so_config c;
    memset(&c, 0, sizeof c);
    int cum, K, Kr;
    unsigned long long seed;
    TRY(rd_d(f, &c.discretization) && rd_i(f, &c.max_iterations) && rd_i(f, &c.max_iterations_after_collision_free) &&
        rd_d(f, &c.smoothness_cost_weight) && rd_d(f, &c.obstacle_cost_weight) && rd_d(f, &c.smoothness_costs[0]) &&
        rd_d(f, &c.smoothness_costs[1]) && rd_d(f, &c.smoothness_costs[2]) && rd_d(f, &c.ridge_factor) &&
        rd_i(f, &cum) && rd_i(f, &K) && rd_i(f, &Kr) && fscanf(f, "%llu", &seed) == 1);
    double origin[3], res;
    TRY(rd_d(f, &origin[0]) && rd_d(f, &origin[1]) && rd_d(f, &origin[2]) && rd_d(f, &res));
    int troot, ttip;
    double grav[3];
    TRY(rd_i(f, &troot) && rd_i(f, &ttip) && rd_d(f, &grav[0]) && rd_d(f, &grav[1]) && rd_d(f, &grav[2]));
    for (int s = 0; s < nseg; ++s) {
        TRY(rd_d(f, &inr[s].mass));
        for (int k = 0; k < 3; ++k) TRY(rd_d(f, &inr[s].com[k]));
        for (int k = 0; k < 6; ++k) TRY(rd_d(f, &inr[s].inertia[k]));
    }
    fclose(f);
    const size_t cells = (size_t)n * n * n;
    unsigned short* grid = malloc(cells * sizeof(unsigned short));   /* d2 per voxel */
    FILE* b = fopen(argv[2], "rb");
    if (!b || fread(grid, sizeof(unsigned short), cells, b) != cells) {
        fprintf(stderr, "cannot read the field\n");
        return 2;
    }
    fclose(b);

    c.num_joints = J;
    c.num_time_steps = N;
    c.num_rollouts = K;
    c.num_reused_rollouts = Kr;
    c.num_segments = nseg;
    c.segments = seg;
    c.num_spheres = nsph;
    c.spheres = sph;
    c.joints = jnt;
    c.sdf.nx = c.sdf.ny = c.sdf.nz = n;
    memcpy(c.sdf.origin, origin, sizeof origin);
    c.sdf.resolution = res;
    c.sdf.data = grid;
    c.noise_stddev = sd;
    c.noise_decay = dc;
    c.use_cumulative_costs = cum;
    c.start = start;
    c.goal = goal;
    c.seed = seed;
    c.threads = argc > 4 ? atoi(argv[4]) : 1;
    c.inertias = inr;
    c.torque_root = troot;
    c.torque_tip = ttip;
    memcpy(c.gravity, grav, sizeof grav);

    so_problem* p = so_create(&c);
    if (!p) {
        fprintf(stderr, "so_create: %s\n", so_last_error());
        return 3;
    }
    FILE* out = fopen(argv[3], "w");
    if (!out) return 2;
    so_stats st;
    double* costs = calloc((size_t)c.max_iterations + 1, sizeof(double));
    if (so_optimize(p, &st, costs)) {
        fprintf(stderr, "so_optimize: %s\n", so_last_error());
        return 4;
    }
    fprintf(out, "%d %d %d\n", st.iterations, st.success_iteration, st.collision_success_iteration);
    for (int i = 0; i < st.iterations; ++i) fprintf(out, "%.17g\n", costs[i]);
    double* traj = calloc((size_t)J * N, sizeof(double));
    so_get_best_trajectory(p, traj);
    for (int i = 0; i < J * N; ++i) fprintf(out, "%.17g\n", traj[i]);
    for (int it = st.iterations + 1; it <= st.iterations + 3; ++it) {
        so_iter_out io;
        if (so_iterate(p, it, &io)) {
            fprintf(stderr, "so_iterate: %s\n", so_last_error());
            return 5;
        }
        fprintf(out, "%.17g %d\n", io.cost, io.collision_free);
    }
    so_get_theta(p, traj);
    for (int i = 0; i < J * N; ++i) fprintf(out, "%.17g\n", traj[i]);
    double* params = calloc((size_t)K * J * N, sizeof(double));
    double* ec = calloc((size_t)N, sizeof(double));
    so_get_rollouts(p, "params", params);
    for (int r = 0; r < K && r < 4; ++r) {
        int ecf = 0;
        if (so_execute(p, params + (size_t)r * J * N, ec, &ecf, traj, 1, NULL)) {
            fprintf(stderr, "so_execute: %s\n", so_last_error());
            return 6;
        }
        for (int i = 0; i < N; ++i) fprintf(out, "%.17g\n", ec[i]);
        for (int i = 0; i < J * N; ++i) fprintf(out, "%.17g\n", traj[i]);
        fprintf(out, "%d\n", ecf);
    }
    fclose(out);
    so_destroy(p);
    free(params); free(ec); free(traj); free(costs); free(grid);
    free(seg); free(sph); free(jnt); free(inr); free(start); free(goal); free(sd); free(dc);
    return 0;
}
