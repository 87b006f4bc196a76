/*
 * oracle/stomp_oracle.h -- TEST INFRASTRUCTURE: CPU restatement of the STOMP
 * hot path of kalakris/stomp_motion_planner_icra2011.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 *
 * PARITY UNPINNED: the reference cannot be compiled here (ROS rosbuild, Eigen 2,
 * orocos KDL, boost, arm_navigation distance_field: SURVEY.md section 8c) and
 * ships no unit tests, golden vectors or recorded outputs.  This restatement is
 * pinned only by the reference's constants (DIFF_RULES, params.yaml), by
 * analytic known-answer tests derived from the cited formulas, and by an
 * independent numpy restatement (oracle/numpy_oracle.py).  See DESIGN.md.
 *
 * Structure follows the reference one-to-one:
 *   so_iterate            PolicyImprovementLoop::runSingleIteration  policy_improvement_loop.cpp:143-202
 *   so_execute            StompOptimizer::execute                    stomp_optimizer.cpp:1063-1165
 *   so_optimize           StompOptimizer::optimize                   stomp_optimizer.cpp:249-401
 * Build-defined choices that the reference leaves to third-party code
 * (RNG, KDL frame conventions, distance-field lookup) are documented in
 * DESIGN.md section "Oracle conventions".
 */
#ifndef STOMP_ORACLE_H
#define STOMP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SO_DIFF_RULE_LENGTH 7
#define SO_NUM_DIFF_RULES 3
#define SO_PAD (SO_DIFF_RULE_LENGTH - 1)

/* One kinematic-tree segment in DFS order (parent index < own index).
 * pose(q) = Frame(rot, trans) * Frame(Rot2(axis, q), 0)   (q_index >= 0)
 *         = Frame(rot, trans)                              (fixed segment)
 * frame[s] = frame[parent] * pose(q)  (treefksolverjointposaxis_partial.cpp:125, 168) */
typedef struct {
    int parent;       /* -1 for the root */
    int q_index;      /* group joint index driving this segment, -1 if fixed */
    double rot[9];    /* row-major */
    double trans[3];
    double axis[3];
} so_segment;

/* StompCollisionPoint (stomp_collision_point.cpp:44-55) */
typedef struct {
    int segment;
    double radius;
    double clearance;
    double pos[3];    /* in the segment frame */
} so_sphere;

/* StompJoint limits (stomp_robot_model.cpp:158-164) */
typedef struct {
    int has_limits;
    double min;
    double max;
    double joint_cost;  /* joint_costs/<name>, default 1.0 (stomp_optimizer.cpp:107-109) */
} so_joint;

/* Voxel grid, z fastest: data[(x*ny + y)*nz + z] = d2, the squared cell distance to the nearest
 * obstacle cell (capped).  The distance is sqrt((double)d2) * resolution, the value
 * PropagationDistanceField reads from its sqrt_table_ (third party; distance_square_ per voxel) */
typedef struct {
    int nx, ny, nz;
    double origin[3];
    double resolution;
    const unsigned short* data;
} so_sdf;

/* KDL::RigidBodyInertia(m, cog, Ic) of a segment, in the segment frame; Ic is about the
 * centre of mass, (Ixx, Iyy, Izz, Ixy, Ixz, Iyz) */
typedef struct {
    double mass;
    double com[3];
    double inertia[6];
} so_inertia;

/* motion_planning_msgs::OrientationConstraint as stored by OrientationConstraintEvaluator
 * (constraint_evaluator.cpp:50-73) */
typedef struct {
    int segment;                /* frame_number_ (segmentNameToIndex(link_name)) */
    double orientation[4];      /* nominal quaternion x, y, z, w */
    int body_fixed;             /* type != HEADER_FRAME */
    double absolute_roll_tolerance;
    double absolute_pitch_tolerance;
    double absolute_yaw_tolerance;
    double weight;
} so_orientation_constraint;

typedef struct {
    int num_joints;             /* J */
    int num_time_steps;         /* N (free waypoints) */
    int num_rollouts;           /* K */
    int num_reused_rollouts;    /* K_r */
    int num_segments;
    const so_segment* segments;
    int num_spheres;
    const so_sphere* spheres;
    const so_joint* joints;
    so_sdf sdf;
    double discretization;      /* trajectory_discretization (params.yaml:5) */
    double smoothness_costs[3]; /* vel, acc, jerk (params.yaml:8-10) */
    double ridge_factor;
    double smoothness_cost_weight;
    double obstacle_cost_weight;
    double constraint_cost_weight;
    double torque_cost_weight;  /* > 1e-9: torque term (stomp_optimizer.cpp:1117-1142) */
    const double* noise_stddev; /* J */
    const double* noise_decay;  /* J */
    int use_cumulative_costs;
    const double* start;        /* J */
    const double* goal;         /* J */
    uint64_t seed;
    int max_iterations;
    int max_iterations_after_collision_free;
    int sum_block;              /* canonical blocked sum over rollouts (64); 0 -> 64 */
    int dense;                  /* 1: dense N x N products exactly as the reference (CPU baseline) */
    int threads;                /* OpenMP threads over rollouts (1 = reference) */
    /* torque term: KDL::ChainIdSolver_RNE over getChain(root, tip) (stomp_robot_model.cpp:185-189) */
    const so_inertia* inertias; /* num_segments (NULL: torque term off) */
    int torque_root;            /* chain base segment (exclusive) */
    int torque_tip;             /* chain tip segment (inclusive) */
    double gravity[3];          /* in the frame of torque_root */
    /* path constraints (stomp_optimizer.cpp:195-201, 1107-1115) */
    int num_orientation_constraints;
    const so_orientation_constraint* orientation_constraints;
    /* 1: the reference's written arithmetic order: non-fused dense L z / M eps and sequential
     * rollout sums over all K (instead of the engine's fma chain and 64-rollout blocks);
     * 2: also VectorXd::sum() as Eigen 2's two-lane SSE2 packet reduction;
     * 3: also the C library's exp / sin / cos / atan2 / asin where the reference calls them */
    int ref_arith;
} so_config;

typedef struct so_problem so_problem;

typedef struct {
    double cost;                /* last_trajectory_cost_ of the noiseless rollout */
    int collision_free;         /* last_trajectory_collision_free_ */
    int constraints_satisfied;  /* last_trajectory_constraints_satisfied_ */
} so_iter_out;

/* KDL::ChainIdSolver_RNE::CartToJnt on the torque chain, group joint vectors of length J */
double so_atan2(double y, double x);
double so_asin(double x);
int so_inverse_dynamics(const so_problem* P, const double* q, const double* qd, const double* qdd, double* tau);

typedef struct {
    int iterations;             /* iterations run */
    int success;
    int success_iteration;
    int collision_success_iteration;
    int last_improvement_iteration;
    double best_cost;
} so_stats;

so_problem* so_create(const so_config* cfg);
void so_destroy(so_problem* p);
const char* so_last_error(void);

/* setup products, for stage tests; which: "Rinv","L","M","Qinv","Rall","D0","D1","D2" */
int so_get_matrix(const so_problem* p, const char* which, int joint, double* out);
int so_get_theta(const so_problem* p, double* theta /* J x N */);
int so_set_theta(so_problem* p, const double* theta);
int so_get_pad_positions(const so_problem* p, double* out /* 12 x S x 3 */);

/* Task::execute on one parameter set (J x N, row per joint). iteration_member is the
 * optimizer's iteration_ (0 => padding points count toward the collision flag). */
int so_execute(so_problem* p, const double* params, double* costs, int* collision_free,
               double* traj_out /* J x N clamped free block, may be NULL */, int iteration_member,
               int* constraints_ok /* last_trajectory_constraints_satisfied_, may be NULL */);

/* runSingleIteration(iteration_number); the optimizer's iteration_ is iteration_number-1 */
int so_iterate(so_problem* p, int iteration_number, so_iter_out* out);

/* StompOptimizer::optimize loop (without the final torque statistics) */
int so_optimize(so_problem* p, so_stats* stats, double* costs_per_iteration /* may be NULL */);
int so_get_best_trajectory(const so_problem* p, double* traj /* J x N */);
/* STOMPStatistics.torques of the best trajectory (N); needs the segment inertias */
int so_get_best_torques(const so_problem* p, double* torques /* N */);
int so_get_last_trajectory(const so_problem* p, double* traj /* J x N */);

/* rollout state after so_iterate, for stage tests. which:
 * "params","noise","noise_projected","control_costs","probabilities" -> K x J x N;
 * "state_costs" -> K x N; the extra rollout (addExtraRollouts): "x_params","x_noise",
 * "x_noise_projected","x_control_costs" -> J x N, "x_state_costs" -> N */
int so_get_rollouts(const so_problem* p, const char* which, double* out);
/* the reuse decisions so far: num_reused_rollouts candidate indices per ranking (-1 = the
 * extra rollout), copied up to cap; returns how many there are */
int so_reuse_log(const so_problem* p, int* out, int cap);

/* stage primitives */
void so_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void so_normals(uint64_t seed, int iteration, int joint, int rollout, int n, double* z);
void so_diff_rules(double* out /* 3 x 7: DIFF_RULES, stomp_utils.h:49-56 */);
double so_exp(double x);
double so_log(double x);
void so_sincos(double x, double* s, double* c);
/* sphere world positions for one joint vector q (J): out S x 3 */
int so_sphere_positions(const so_problem* p, const double* q, double* out);
/* distance-field lookup + hinge potential for one sphere (stomp_collision_space.h:193-228) */
double so_sdf_distance(const so_problem* p, double x, double y, double z);
int so_potential(const so_problem* p, int sphere, const double* pos, double* potential);

/* Collision-space voxeliser (oracle/sdf_oracle.c): the shapes of
 * StompCollisionSpace::addCollisionObjectsToPoints (stomp_collision_space.cpp:199-297) and
 * the robot bodies of getVoxelsInBody (:592-650), marked into a grid and turned into the
 * capped, quantised EDT.  Types as stomp_engine.h STOMP_SHAPE_* / STOMP_BODY_*. */
typedef struct {
    int type;
    double position[3];
    double orientation[4];   /* quaternion x, y, z, w */
    double dims[3];
    const double* vertices;  /* BODY_MESH: num_vertices x 3 in the body frame (scale applied); dims[0] = padding */
    int num_vertices;
} so_shape;
/* occ (nx*ny*nz bytes, may be NULL) receives the marked cells; sdf (uint16, may be NULL) the
 * field min(d2, cap^2), cap = ceil(max_expansion / res) <= 255.  Returns the number of points
 * marked (inside the grid), -1 on invalid input. */
long long so_sdf_build_objects(int nx, int ny, int nz, const double* origin, double res, double max_expansion,
                               const so_shape* shapes, int n_shapes, const double* points, long long n_points,
                               unsigned char* occ, unsigned short* sdf);
/* bodies::ConvexMesh's hull as planes: the supporting planes (unit outward normal n, offset d:
 * n.x + d = 0 on the face) of the convex hull of V (nv x 3); planes: room for max_planes x 4.
 * Returns the number of planes, -1 if the vertices span no volume or max_planes is too small. */
int so_hull_planes(const double* V, int nv, double* planes, int max_planes);
/* capped EDT of an occupancy grid alone (the second half of so_sdf_build_objects); -1 when the
 * cap exceeds 255 cells (d2 would not fit 16 bits) */
int so_sdf_from_occupancy(int nx, int ny, int nz, double res, double max_expansion, const unsigned char* occ,
                          unsigned short* sdf);

#ifdef __cplusplus
}
#endif
#endif
