/*
 * stomp_engine.h -- C ABI of the MI355X STOMP noisy-rollout cost engine.
 *
 * Drop-in boundary for the hot path of kalakris/stomp_motion_planner_icra2011
 * (paths relative to /root/reference/stomp_motion_planner/):
 *
 *   stomp_engine_create      replaces StompOptimizer::StompOptimizer + initialize()
 *                            (stomp_optimizer.cpp:50-202) together with
 *                            PolicyImprovementLoop::initialize (policy_improvement_loop.cpp:88-110),
 *                            PolicyImprovement::initialize (policy_improvement.cpp:64-94) and
 *                            CovariantTrajectoryPolicy::initialize/setToMinControlCost
 *                            (covariant_trajectory_policy.cpp:70-148)
 *   stomp_engine_iterate     replaces PolicyImprovementLoop::runSingleIteration
 *                            (policy_improvement_loop.cpp:143-202)
 *   stomp_engine_run         the same iteration, enqueued `count` times with no host sync
 *   stomp_engine_eval        replaces StompOptimizer::execute (stomp_optimizer.cpp:1063-1165),
 *                            batched over rollouts (Task::execute, task.h:70)
 *   stomp_engine_optimize    replaces StompOptimizer::optimize (stomp_optimizer.cpp:249-401)
 *   stomp_engine_get_theta / set_theta
 *                            replace CovariantTrajectoryPolicy::getParameters/setParameters
 *                            (covariant_trajectory_policy.h:200-227)
 *   stomp_sdf_build          builds the distance field that
 *                            StompCollisionSpace::setStartState + PropagationDistanceField
 *                            produce (stomp_collision_space.cpp:154-197), for box and
 *                            z-cylinder obstacles, directly in device memory
 *   stomp_sdf_build_objects  the same fill by the reference's own rules: posed boxes and
 *                            cylinders sampled on its lattice, robot bodies, collision-map
 *                            points (stomp_collision_space.cpp:199-297, 564-650)
 *
 * Conventions: plain pointers and sizes only; host buffers are caller-owned and
 * read/written during the call; device buffers are engine-owned.  Trajectories
 * and parameters are row-major [joint][time step] doubles (J x N).  Every call
 * returns 0 on success (the reference's `true`) or a negative STOMP_E_* code;
 * stomp_engine_last_error() / stomp_last_error() give the message.  Calls on one
 * engine must be serialised by the caller (the reference is single-threaded,
 * stomp_planner_node.cpp:547); distinct engines may run concurrently.
 */
#ifndef STOMP_ENGINE_H
#define STOMP_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STOMP_ENGINE_ABI_VERSION 4

#define STOMP_OK 0
#define STOMP_E_INVALID (-1)   /* bad sizes / arguments */
#define STOMP_E_DEVICE (-2)    /* HIP runtime failure */
#define STOMP_E_UNSUPPORTED (-3)
#define STOMP_E_COMM (-4)      /* RCCL failure */

/* One kinematic-tree segment, DFS order (parent < own index).  Frame of the
 * segment tip: frame[s] = frame[parent] * Frame(rot, trans) * Frame(Rot2(axis, q), 0)
 * with q = joint vector[q_index] (q_index = -1: fixed segment).  Replaces the KDL
 * tree of stomp_robot_model.cpp:81-86 as consumed by
 * treefksolverjointposaxis_partial.cpp:108-178. */
typedef struct stomp_segment {
    int32_t parent;
    int32_t q_index;
    double rot[9];
    double trans[3];
    double axis[3];
} stomp_segment;

/* StompCollisionPoint (stomp_collision_point.h:76-82): sphere in a segment frame */
typedef struct stomp_sphere {
    int32_t segment;
    double radius;
    double clearance;
    double pos[3];
} stomp_sphere;

/* StompJoint limits and joint_costs/<name> (stomp_robot_model.h, stomp_optimizer.cpp:107-109) */
typedef struct stomp_joint {
    int32_t has_limits;
    double min;
    double max;
    double joint_cost;
} stomp_joint;

/* Distance field as PropagationDistanceField holds it (third party; read at
 * stomp_collision_space.h:187-191): data[(x*ny + y)*nz + z] = d2, the integer squared cell
 * distance to the nearest obstacle cell, already capped (<= ceil(max_expansion/res)^2); the
 * distance of a cell is sqrt((double)d2) * resolution, in double, as its sqrt_table_.  A
 * position maps to the cell round((p - origin)/resolution); cells with any index < 1 or
 * >= n-1 read distance 0 (distance_field::getDistanceGradient semantics). */
typedef struct stomp_grid {
    int32_t nx, ny, nz;
    double origin[3];
    double resolution;
    const uint16_t* data;       /* host pointer, or device pointer if data_on_device */
    int32_t data_on_device;     /* 1: engine reads the buffer (caller keeps it alive): in place
                                 * for a field of at most 64 MiB; a larger one (e.g. 512^3) is
                                 * copied once at creation into the engine's 4^3-brick layout
                                 * (STOMP_SDF_LAYOUT=brick|linear overrides the size rule), so a
                                 * caller that rebuilds the field in the same buffer (e.g. with
                                 * stomp_sdf_build_objects between plans) calls
                                 * stomp_engine_refresh_field afterwards */
} stomp_grid;

/* KDL::RigidBodyInertia(m, cog, Ic) of a segment, in the segment frame; Ic about the
 * centre of mass as (Ixx, Iyy, Izz, Ixy, Ixz, Iyz).  Replaces the URDF <inertial> data
 * KDL's ChainIdSolver_RNE reads (stomp_robot_model.cpp:185-189). */
typedef struct stomp_inertia {
    double mass;
    double com[3];
    double inertia[6];
} stomp_inertia;

/* motion_planning_msgs::OrientationConstraint as OrientationConstraintEvaluator stores it
 * (constraint_evaluator.cpp:50-73) */
typedef struct stomp_orientation_constraint {
    int32_t segment;            /* frame_number_ = segmentNameToIndex(link_name) */
    double orientation[4];      /* nominal orientation quaternion (x, y, z, w) */
    int32_t body_fixed;         /* 0: type == HEADER_FRAME, 1: body-fixed */
    double absolute_roll_tolerance;
    double absolute_pitch_tolerance;
    double absolute_yaw_tolerance;
    double weight;
} stomp_orientation_constraint;

typedef struct stomp_engine_desc {
    int32_t abi_version;        /* STOMP_ENGINE_ABI_VERSION */
    int32_t num_joints;         /* J (planning group joints) */
    int32_t num_time_steps;     /* N free waypoints (params.yaml num_time_steps) */
    int32_t num_rollouts;       /* K (params.yaml num_rollouts), whole job */
    int32_t num_reused_rollouts;/* K_r (params.yaml num_reused_rollouts) */
    int32_t num_segments;
    const stomp_segment* segments;
    int32_t num_spheres;
    const stomp_sphere* spheres;
    const stomp_joint* joints;  /* J */
    stomp_grid grid;
    double discretization;      /* trajectory_discretization */
    double smoothness_costs[3]; /* smoothness_cost_{velocity,acceleration,jerk} */
    double ridge_factor;
    double smoothness_cost_weight;
    double obstacle_cost_weight;
    double constraint_cost_weight;
    double torque_cost_weight;  /* > 1e-9: torque term (stomp_optimizer.cpp:1117-1142) */
    const double* noise_stddev; /* J */
    const double* noise_decay;  /* J */
    int32_t use_cumulative_costs;
    const double* start;        /* J */
    const double* goal;         /* J */
    uint64_t seed;              /* Philox key of the noise stream */
    int32_t max_iterations;
    int32_t max_iterations_after_collision_free;
    int32_t device;             /* HIP device ordinal */
    void* stream;               /* hipStream_t to launch on; NULL -> engine-owned stream */
    int32_t rank;               /* rollout shard of this process (0 if world_size == 1) */
    int32_t world_size;         /* processes sharing the K rollouts (1 = no collectives) */
    const void* comm_id;        /* 128-byte RCCL unique id from stomp_comm_unique_id (rank 0) */
    /* torque term: inverse dynamics over the chain torque_root (exclusive) -> torque_tip
     * (inclusive), whose joints must be the group's joints in order (the reference's
     * kdl_tree_.getChain("torso_lift_link", "r_gripper_tool_frame"), stomp_robot_model.cpp:185-189) */
    const stomp_inertia* inertias;  /* num_segments; may be NULL while the torque term is off */
    int32_t torque_root;
    int32_t torque_tip;
    double gravity[3];              /* in the torque_root frame (the reference: 0, 0, -9.8) */
    /* orientation path constraints (stomp_optimizer.cpp:195-201, 1107-1115) */
    int32_t num_orientation_constraints;
    const stomp_orientation_constraint* orientation_constraints;
} stomp_engine_desc;

typedef struct stomp_engine stomp_engine;

typedef struct stomp_iter_out {
    double cost;                /* last_trajectory_cost_ of the noiseless rollout */
    int32_t collision_free;     /* last_trajectory_collision_free_ */
    int32_t constraints_satisfied; /* last_trajectory_constraints_satisfied_ */
} stomp_iter_out;

/* STOMPStatistics (msg/STOMPStatistics.msg): the per-iteration costs go to the
 * costs_per_iteration argument of stomp_engine_optimize, the torques to
 * stomp_engine_get_best_torques.  Durations are seconds from the loop's start to the end of
 * the noiseless rollout of (collision_)success_iteration, on the device wall clock
 * (stomp_optimizer.cpp:251, 306-319); 0 when that iteration never came. */
typedef struct stomp_stats {
    int32_t iterations;
    int32_t success;
    int32_t success_iteration;
    int32_t collision_success_iteration;
    int32_t last_improvement_iteration;
    double best_cost;
    double success_duration;
    double collision_success_duration;
} stomp_stats;

int stomp_engine_create(const stomp_engine_desc* desc, stomp_engine** out);
void stomp_engine_destroy(stomp_engine* e);
const char* stomp_engine_last_error(const stomp_engine* e);
const char* stomp_last_error(void);
/* The 16-hex-digit hash of the sources (and compile flags) this library was built from
 * (stomp_motion_planner_icra2011_amd/_build.py source_hash): the Python binding refuses a library
 * whose hash is not the checkout's, and bench.py reports the hash of the library it timed. */
const char* stomp_engine_source_hash(void);

/* Re-reads the caller's device field (data_on_device = 1) after the caller rebuilt it in place:
 * with the engine's bricked copy the copy is remade (ordered on the engine stream after the work
 * already enqueued there; the caller orders its own rebuild before this call); with the field used
 * in place, nothing to do.  A host field (data_on_device = 0) was uploaded at creation:
 * STOMP_E_UNSUPPORTED. */
int stomp_engine_refresh_field(stomp_engine* e);

int stomp_engine_get_theta(stomp_engine* e, double* theta);
int stomp_engine_set_theta(stomp_engine* e, const double* theta);

int stomp_engine_iterate(stomp_engine* e, int32_t iteration_number, stomp_iter_out* out);
/* run: count iterations enqueued with no host sync.  The last one's noiseless rollout is left
 * pending (it rides in the next rollout launch); synchronize, iterate, set_theta and the
 * trajectory reads evaluate it first. */
int stomp_engine_run(stomp_engine* e, int32_t first_iteration, int32_t count);
/* synchronize, and every other call that waits for the engine's stream: with an RCCL communicator
 * (world_size > 1) the wait is bounded.  An RCCL error, or no completion within
 * STOMP_COMM_TIMEOUT_S seconds (default 300), aborts the communicator (ncclCommAbort) and returns
 * STOMP_E_COMM with a message naming the first collective not complete and the last one posted
 * (kind, iteration and ordinal of each); every later call on the engine returns the same. */
int stomp_engine_synchronize(stomp_engine* e);

/* Batched Task::execute: params E x J x N, costs E x N, collision_free E,
 * traj_out E x J x N (joint-limit-corrected free block, may be NULL).
 * iteration_member is StompOptimizer::iteration_ (0: padding points count for the flag).
 * constraints_satisfied E (last_trajectory_constraints_satisfied_, may be NULL). */
int stomp_engine_eval(stomp_engine* e, const double* params, int32_t num, double* costs,
                      uint8_t* collision_free, double* traj_out, int32_t iteration_member,
                      uint8_t* constraints_satisfied);

int stomp_engine_optimize(stomp_engine* e, stomp_stats* stats, double* costs_per_iteration);
/* STOMPStatistics.torques after optimize (stomp_optimizer.cpp:384-398): per free waypoint,
 * sum_j |tau_j| of the best trajectory by inverse dynamics over the torque chain (N doubles).
 * Needs the segment inertias in the descriptor (also with the torque term off);
 * STOMP_E_UNSUPPORTED without them. */
int stomp_engine_get_best_torques(stomp_engine* e, double* torques);

/* PolicyImprovement (policy_improvement.h:86-126) step by step, for a caller that executes the
 * rollouts with its own Task between the steps (single rank):
 *   get_rollouts        generateRollouts(noise_stddev) + computeProjectedNoise (:158-260): reuse
 *                       ranking, new noise for the generated rows keyed by `iteration` (the
 *                       Philox stream of runSingleIteration(iteration)); the K_gen generated
 *                       parameter sets (K_gen x J x N) and K_gen out
 *   set_rollout_costs   setRolloutCosts (:262-281): state costs of the generated rows (K x N,
 *                       rows >= K_gen ignored), control costs of all K with 0.5 * weight,
 *                       Rollout::getCost of every row (K) out
 *   improve_policy      improvePolicy (:385-401): probabilities and the update M (sum eps P)
 *                       (J x N; row 0 of the reference's per-joint update matrices), theta untouched
 *   add_extra_rollouts  addExtraRollouts (:443-462) of num = 1 rollout: parameters J x N and its
 *                       state costs N; noise against the current theta
 *   reset               setNumRollouts (:96-147) with the engine's own counts: the reuse state
 *                       starts over (the next iteration generates every rollout, a pending extra
 *                       rollout is dropped from the next ranking)
 * Applying the update is Policy::updateParameters: stomp_engine_get_theta / set_theta. */
int stomp_pi_get_rollouts(stomp_engine* e, int32_t iteration, const double* noise_stddev, double* rollouts,
                          int32_t* num_generated);
int stomp_pi_set_rollout_costs(stomp_engine* e, const double* costs, double control_cost_weight, double* totals);
int stomp_pi_improve_policy(stomp_engine* e, double* updates);
int stomp_pi_add_extra_rollouts(stomp_engine* e, int32_t num, const double* params, const double* costs);
int stomp_pi_reset(stomp_engine* e);
int stomp_engine_get_best_trajectory(stomp_engine* e, double* traj);
int stomp_engine_get_last_trajectory(stomp_engine* e, double* traj);

/* Inspection for parity tests.  which: "params","noise","control_costs","probabilities"
 * -> K_local x J x N; "state_costs" -> K_local x N; the extra (noiseless) rollout of
 * addExtraRollouts (policy_improvement.cpp:443-462): "x_params","x_noise","x_control_costs"
 * -> J x N (kept with K_r > 0 only), "x_state_costs" -> N. */
int stomp_engine_get_rollouts(stomp_engine* e, const char* which, double* out);
/* which: "Rinv","L","M","Qinv" (N x N, joint selects Qinv), "R" (free block of the
 * control-cost matrix, CovariantTrajectoryPolicy::getControlCosts,
 * covariant_trajectory_policy.h:235-239), "D0","D1","D2" (the policy's differentiation
 * matrices, (N+12) x (N+12), covariant_trajectory_policy.cpp:204-226).  Host only. */
int stomp_engine_get_matrix(stomp_engine* e, const char* which, int32_t joint, double* out);
/* sphere world positions at the 12 padding points (12 x S x 3) */
int stomp_engine_get_pad_positions(stomp_engine* e, double* out);

/* Per-kernel device time (HIP events on the engine stream), accumulated while enabled.
 * name: "noise", "rollout_cost", "weights", "update", "noiseless", "all". */
int stomp_engine_set_timing(stomp_engine* e, int32_t enable);
int stomp_engine_get_timing(stomp_engine* e, const char* name, double* total_ms, int32_t* launches);
int stomp_engine_local_rollouts(stomp_engine* e, int32_t* first, int32_t* count);
/* The K-sharded decomposition the engine chose: STOMP_SHARD_NONE (one rank),
 * STOMP_SHARD_PARTIALS (all-reduce + two all-gathers of 64-rollout block partials per iteration) or
 * STOMP_SHARD_GATHER (one all-gather of the state-cost rows; every rank weights all K). */
#define STOMP_SHARD_NONE 0
#define STOMP_SHARD_PARTIALS 1
#define STOMP_SHARD_GATHER 2
int stomp_engine_shard_mode(stomp_engine* e, int32_t* mode);
/* How the decomposition was chosen.  info[0] = the mode; when both were possible and none was
 * requested (STOMP_SHARD_MODE unset, world > 1) the engine measured at creation, maxima over the
 * ranks, in microseconds: info[1] = one iteration's compute in gather mode, info[2] = in partials mode
 * (no exchanges), info[3] = the all-reduce(max) of 2 J N doubles, info[4] = the all-gather of the
 * state-cost rows, info[5] = the all-gather of the block partials; zeros otherwise. */
int stomp_engine_shard_info(stomp_engine* e, double* info);
/* The rule applied to those measurements (host only): gather when info[1] + info[4] <=
 * info[2] + info[3] + 2 info[5] (one all-gather against three dependent collectives).
 * measured = info + 1. */
int stomp_shard_decide(const double* measured, int32_t* mode);

/* Distance-field builder (capped exact EDT, stomp_grid's representation):
 *   value = min(d2, ceil(max_expansion/res)^2)   (the cap must be <= 255 cells)
 * d2 = integer squared cell distance to the nearest cell whose centre
 * origin + i*res lies in an obstacle.  boxes: n_boxes x (cx,cy,cz,dx,dy,dz),
 * axis-aligned; cylinders: n_cyl x (cx,cy,cz,radius,length), z-aligned.
 * out_device: device buffer of nx*ny*nz uint16 (z fastest). */
int stomp_sdf_build(int32_t nx, int32_t ny, int32_t nz, const double* origin, double resolution,
                    double max_expansion, const double* boxes, int32_t n_boxes, const double* cylinders,
                    int32_t n_cylinders, uint16_t* out_device, void* stream);

/* An object of the collision space.  Environment objects are sampled as
 * StompCollisionSpace::addCollisionObjectsToPoints does (stomp_collision_space.cpp:199-297):
 *   STOMP_SHAPE_BOX       dims = (dx, dy, dz)
 *   STOMP_SHAPE_CYLINDER  dims = (radius, length, -), axis = the pose's z
 * on the running-sum lattice xlow, xlow + res, ... (x <= xlow + dim + res), each point p
 * mapped through Frame(Rotation::Quaternion(orientation), position) as position - p.
 * Robot bodies (getVoxelsInBody, :592-650; the links addAllBodiesButExcludeLinksToPoints keeps,
 * :564-590, with the caller's padding/scale folded into dims):
 *   STOMP_BODY_SPHERE     dims = (radius, -, -)
 *   STOMP_BODY_BOX        dims = (dx, dy, dz)
 *   STOMP_BODY_CYLINDER   dims = (radius, length, -)
 *   STOMP_BODY_MESH       vertices (num_vertices x 3, the body frame, scale applied), dims =
 *                         (padding, -, -): a robot link's mesh or an environment object of type
 *                         MESH (:216-223 take it through getVoxelsInBody too), as
 *                         bodies::ConvexMesh: the convex hull of the vertices
 * on the lattice position + g * res around the bounding sphere (a mesh's: around its vertices'
 * bounding-box centre), kept where the body contains the point (the reference's ray-crossing
 * parity for these convex bodies). */
#define STOMP_SHAPE_BOX 0
#define STOMP_SHAPE_CYLINDER 1
#define STOMP_BODY_SPHERE 2
#define STOMP_BODY_BOX 3
#define STOMP_BODY_CYLINDER 4
#define STOMP_BODY_MESH 5
typedef struct stomp_shape {
    int32_t type;
    double position[3];
    double orientation[4];      /* quaternion (x, y, z, w), geometry_msgs::Pose order */
    double dims[3];
    const double* vertices;     /* STOMP_BODY_MESH only (host memory), else NULL */
    int32_t num_vertices;
} stomp_shape;

/* The reference's distance-field fill (StompCollisionSpace::setStartState,
 * stomp_collision_space.cpp:154-197) on the device: every object's points and the
 * collision-map points (points: n_points x 3, the "points" namespace, :205-211) mark the cell
 * round((p - origin) * (1/res)) when it lies in the grid (PropagationDistanceField::
 * addPointsToField); value = min(d2, cap^2) with cap = ceil(max_expansion/res) (<= 255) and
 * d2 the integer squared cell distance to the nearest marked cell (stomp_grid's
 * representation).  marked (may be NULL): points that landed inside the grid. */
int stomp_sdf_build_objects(int32_t nx, int32_t ny, int32_t nz, const double* origin, double resolution,
                            double max_expansion, const stomp_shape* shapes, int32_t n_shapes,
                            const double* points, int64_t n_points, uint16_t* out_device, int64_t* marked,
                            void* stream);

/* The differentiation stencils the engine is built on (DIFF_RULES of stomp_utils.h:49-56:
 * velocity, acceleration, jerk; 3 x 7 doubles, row-major).  Host only, no device needed. */
int stomp_diff_rules(double* out);

/* Groups: several engines of one shape (same J, N, K, spheres and model layout; single device,
 * no reuse, no state-cost terms), created on ONE shared stream, advanced in lockstep by shared
 * launches -- one rollout, one weights and one update launch per iteration for the whole group
 * instead of three per engine (a batch of independent planning problems, BASELINE cfg5).  Each
 * engine ends in exactly the state its own stomp_engine_run(first, count) leaves: its θ, rollouts
 * and pending noiseless rollout; the engines' own calls keep working between group runs.
 * stomp_group_synchronize flushes every engine's pending noiseless rollout and waits. */
typedef struct stomp_group stomp_group;
int stomp_stream_create(int32_t device, void** out_stream);
int stomp_stream_destroy(void* stream);
int stomp_group_create(stomp_engine* const* engines, int32_t num_engines, stomp_group** out);
int stomp_group_run(stomp_group* g, int32_t first_iteration, int32_t count);
int stomp_group_synchronize(stomp_group* g);
const char* stomp_group_last_error(const stomp_group* g);
void stomp_group_destroy(stomp_group* g);

/* Device buffers for callers without a HIP runtime of their own (bench, tests). */
int stomp_device_alloc(int32_t device, uint64_t bytes, void** out);
int stomp_device_free(void* p);
int stomp_device_copy_to_host(void* dst, const void* src, uint64_t bytes);
int stomp_device_count(int32_t* count);

/* RCCL unique id for world_size > 1 (call on rank 0, broadcast the 128 bytes). */
int stomp_comm_unique_id(void* out128);
/* Id of an in-process exchange group of world_size ranks: the ranks are engines of THIS
 * process (on one device or several), each created with this id, its rank and world_size and
 * each driven by a host thread of its own; the per-iteration exchanges are device-to-device
 * copies ordered by HIP events instead of RCCL (same results bit for bit). */
int stomp_comm_local_id(int32_t world_size, void* out128);

/* deterministic math + RNG primitives evaluated on the device (parity tests) */
int stomp_device_selftest(const double* x, int32_t n, double* out_exp, double* out_log, double* out_sin,
                          double* out_cos, double* out_sqrt);
int stomp_device_normals(uint64_t seed, int32_t iteration, int32_t joint, int32_t rollout, int32_t n, double* z);

#ifdef __cplusplus
}
#endif
#endif
