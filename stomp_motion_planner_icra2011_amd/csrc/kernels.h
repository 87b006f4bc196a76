// kernels.h -- device data layout and kernel entry points of the STOMP engine.
//
// HBM layout (one engine = one planning problem, K_loc rollouts on this device):
//   theta            [J][N]                fp64  policy parameters (free block)
//   LT, MT           [N(k)][N(i)]          fp64  chol(R^-1) and the projection M, transposed so
//                                                that lanes (i) read consecutive addresses
//   QT               [J][N(k)][N(i)]       fp64  scaled StompCost inverse, column k contiguous
//   params, noise,
//   control, prob    [K_loc][J][N]         fp64  Rollout::parameters_/noise_/control_costs_/probabilities_
//   state            [K_loc][N]            fp64  Rollout::state_costs_
//   sdf              [nx][ny][nz]          u16   distance field as squared cell distances d2 (z
//                                                fastest); distance = sqrt((double)d2) * res
//   psum/u partials  [blocks][J][N]        fp64  per-64-rollout-block sums (RCCL all-gather payload)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace stomp {

constexpr int kMaxJoints = 32;
constexpr int kRunMaxSmall = 16;  // spheres per run (one a-value buffer of the rollout kernel) when N <= 128
constexpr int kRunMaxLarge = 8;   // when N > 128: keeps two rollout WGs per CU at N = 199
constexpr int kSaves = 2;         // saved branch-point FK frames (LDS, one column per waypoint)
constexpr int kSumBlock = 64;     // canonical blocked summation over rollouts
constexpr int kBandBatch = 8;     // rows per load batch of the noise band products
constexpr int kMatPadRows = 16 * kBandBatch;  // zero rows past N in LT / MT (ring look-ahead)
constexpr int kVelTap0 = 2;       // non-zero taps of the velocity rule DIFF_RULES[0]
constexpr int kVelTap1 = 5;       // (stomp_utils.h:54), checked in stomp_engine_create
constexpr int kNoiseJT = 4;       // joint columns per matrix-core block of the rollout kernel's noise phase

inline int run_max(int N) { return N <= 128 ? kRunMaxSmall : kRunMaxLarge; }

// FK program step, executed by every waypoint lane (all fields wave-uniform):
//   seg >= 0: C = base * pose(seg, q)   base: -2 = C itself (chain), -1 = identity (root),
//                                        k >= 0 = saved frame k (branch point)
//             if save >= 0: saved[save] = C
//   then emit spheres [sph_begin, sph_end) from C (seg < 0: emit only).
constexpr int kBaseChain = -2;
constexpr int kBaseRoot = -1;

struct DevSegment {
    int parent, q_index;
    int rot_identity, pad_;     // the fixed rotation is exactly the identity: its products are skipped
    double rot[9];
    double trans[3];
    double axis[3];
};

struct DevSphere {
    int slot;                   // index of its segment's published frame
    // the hinge potential and the collision test as thresholds on the voxel's d2 (made on the
    // host with the potential's own expressions, stomp_collision_space.h:193-228):
    //   potential == 0   <=>  d2 >= zero_lim   (d = sqrt(d2) res - radius >= clearance)
    //   in collision     <=>  d2 <  col_lim    (sqrt(d2) res <= radius)
    int zero_lim, col_lim, pad_;
    double radius, clearance, inv_clearance;
    double pos[3];
};

struct FkOp {
    int seg, base, save, sph_begin, sph_end;
    int slot;                   // publish C as frame slot `slot` (-1: not a sphere segment)
};

struct DevModel {
    int J, N, Nall, S, nops, nseg, nslots, sph_chunk;   // sph_chunk: most spheres on one segment
    int nsaves;                 // saved branch-point frames the FK program uses (0..kSaves, LDS)
    int pad_lds;                // padding-row positions staged in LDS (1) or read from HBM (0)
    int sincos_pre;             // every (sin, cos) of the joint-limited trajectory made before the FK
                                // program by all lanes: sines over traj, cosines in the saved-frame
                                // area (the program's first save comes after its last joint segment)
    int cus;                    // compute units of the device (launch_cost: wide workgroups when a
                                // launch's rollouts fit one per CU)
    int phased_lds;             // dynamic LDS of the phased wide rollout (every slot's frame and every
                                // sphere's a value resident), 0 when it does not fit a CU
    const unsigned long long* img;   // the rollout kernel's LDS table image (RolloutLds from .sph on)
    int img_words;              // 8-byte words of it copied to LDS (up to .pad, or .total with pad_lds)
    const DevSegment* segs;
    const DevSphere* sph;
    const FkOp* ops;
    const int* slot_sph;        // [nslots+1] spheres of slot g: [slot_sph[g], slot_sph[g+1])
    const double* pad_pos;      // [12][S][3]
    const unsigned short* sdf;  // d2 per voxel: [nx][ny][nz] (z fastest), or 4x4x4 bricks (brick)
    int nx, ny, nz;
    int brick;                  // bricks of 4^3 voxels (128 B, one L2 line): brick (bx, by, bz) at
                                // ((bx nby + by) nbz + bz) 64, voxel (x, y, z) & 3 inside at
                                // (x & 3) 16 + (y & 3) 4 + (z & 3)
    int nby, nbz;               // bricks per y / z axis (ceil(n / 4))
    double ox, oy, oz, res, inv_res;
    double ny_d, nz_d;          // ny, nz as doubles (the fp64 cell index of sdf_d2)
    double hi_x, hi_y, hi_z;    // n - 1.5 per axis: round(u) <= n - 2 <=> u < n - 1.5
    const double* start;        // [J]
    const double* goal;         // [J]
    double vel_coef[7];         // invTime * DIFF_RULES[0][k]
    double w_obs, w_con, w_tq;
    int pad_collision;
    const double* QT;           // [J][N][N]
    int* split_cnt;             // [split_cap] pieces done per rollout of the waypoint-split rollout
                                // launch (zero between launches), null: no split launches.  Invariant:
                                // split_cap >= the nro of every split launch (a launch's rollouts,
                                // eval batches included); split_pieces refuses larger launches
    int split_cap;
    int split_max;              // most pieces per rollout (STOMP_DEBUG_SPLIT_MAX, read at creation)
    int x_ctl_inline;           // STOMP_DEBUG_XCTL_INLINE=1: the extra rollout's control rows by its
                                // first piece (CostArgs::x_ctl_block never set)
    // LDS-lean slot-loop layout (rollout_lds lean > 0), chosen at creation when it fits more rollout
    // workgroups on a CU than the full layout and the launch has more workgroups than the full
    // layout's slots (cfg3's N = 199, cfg4's two-arm tree): 1 = the saved branch-point frames in HBM
    // (sv_glob, one [nsaves][12][N] block per rollout workgroup of a launch), no (sin, cos) pre-pass
    // (its cosines parked in the saved-frame area), and the FK / joint-limit tables read from the
    // image in HBM through the scalar cache; 2 = also the sphere table (only with one pair-lane
    // group, N > kBlock / 2, where a run's sphere index is uniform)
    int lean;
    double* sv_glob;
    int sv_rows;                // rollout workgroups sv_glob holds (>= every lean launch's nro)
};


// LDS carve-up of the rollout kernel (bytes).  traj stays resident; the per-slot FK buffers
// follow it and the noise phase's two buffers alias them (they are dead before the first
// frame is published).  From .sph on the layout is a byte image that the engine assembles
// once in HBM (DevModel::img, padding positions last) and each workgroup copies in one pass.
struct RolloutLds {
    size_t traj, fb, sv, av, nzl, nzA, nzB, sph, seg, ops, slot, hl, jlim, pad, total;
};

// The phased layout (k_rollout_phased): fb holds every slot's frame [nslots][12][N], av every
// sphere's a values [S][N] and nzl every pair; the rest as above.

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline int noise_jp(int J) { return (J + kNoiseJT - 1) / kNoiseJT * kNoiseJT; }

__host__ __device__ inline RolloutLds rollout_lds(int J, int N, int S, int max_slot, int nsaves, int nseg, int nops,
                                                  int nslots, int pad_lds, bool phased = false, int lean = 0)
{
    RolloutLds l;
    if (phased) max_slot = S;
    l.traj = 0;
    l.fb = l.traj + (size_t)J * N * sizeof(double);
    l.sv = l.fb + (size_t)(phased ? nslots : 1) * 12 * N * sizeof(double);
    l.av = l.sv + (size_t)(lean ? 0 : nsaves) * 12 * N * sizeof(double);
    l.nzl = l.av + (size_t)max_slot * N * sizeof(double);
    // noise phase: A = z then x (padded), B = eps then the control-cost terms
    const size_t nzw = (size_t)(N + kBandBatch) * noise_jp(J) > (size_t)J * (N + 12)
                           ? (size_t)(N + kBandBatch) * noise_jp(J) : (size_t)J * (N + 12);
    l.nzA = l.fb;
    // phased: in the a-value buffers when they hold both (they are dead until the pairs), so x
    // and the control terms survive the FK program, which prices the row on its idle waves
    if (phased && (size_t)S * N * (sizeof(double) + sizeof(unsigned short)) >= 2 * nzw * sizeof(double)) l.nzA = l.av;
    l.nzB = l.nzA + nzw * sizeof(double);
    size_t end = l.nzl + (size_t)max_slot * N * sizeof(unsigned short);
    if (l.nzB + nzw * sizeof(double) > end) end = l.nzB + nzw * sizeof(double);
    l.sph = align16(end);
    l.seg = align16(l.sph + (size_t)S * sizeof(DevSphere));
    l.ops = align16(l.seg + (size_t)nseg * sizeof(DevSegment));
    l.slot = align16(l.ops + (size_t)nops * sizeof(FkOp));
    l.hl = align16(l.slot + (size_t)(nslots + 1) * sizeof(int));
    l.jlim = align16(l.hl + (size_t)J * sizeof(int));
    l.pad = align16(l.jlim + (size_t)2 * J * sizeof(double));
    l.total = l.pad + (pad_lds ? (size_t)36 * S * sizeof(double) : 0);
    if (lean) {   // only the sphere table (lean 1) stays in LDS; no padding positions
        l.total = lean == 1 ? l.seg : l.sph;
    }
    return l;
}

struct Sigma {
    double v[kMaxJoints];
};

struct NoiseArgs {
    int J, N, Nall, K_loc, first_global, K_gen_global, iteration;
    uint64_t seed;
    Sigma sigma;
    const double* theta;
    const double* LT;
    const double* MT;
    const double* start;
    const double* goal;
    double dcoef[3][7];
    double wr[3];               // 0.5*smoothness_cost_weight * smoothness_costs[rule]
    double* params;
    double* noise;
    double* control;
    int zero_noise;             // extra rollout: params given, noise = 0 (addExtraRollouts); 2: params
                                // are theta, copied into params by the launch
    const int* stop;            // device-resident optimize loop: nonzero -> the launch is a no-op
    int row_begin;              // only rows [row_begin, K_loc) (reused rows after the reuse kernel)
    double* pre_eps;            // [K_loc][J][N] eps = sigma L z made ahead of the rollout launch (k_pregen)
    double* pre_meps;           // [K_loc][J][N] M eps, likewise
    int rows_in_pre;            // pregen rows: leave eps in pre_eps (no noise / params row copies;
                                // the weights read pre_eps, stomp_engine_get_rollouts rebuilds them)
    double* theta_gen;          // with rows_in_pre: rollout 0 keeps the theta the rows were made from
};

// Task::execute batch: blocks [0, num_noisy) evaluate params rows; block num_noisy (if
// x_params) evaluates the noiseless rollout of theta (pipelined from the previous iteration).
struct CostArgs {
    const int* stop;            // nonzero -> no-op (device-resident optimize loop)
    int fused_noise;            // blocks < num_noisy first generate their row (NoiseArgs nz): 1 = normals,
    NoiseArgs nz;               // L z, params, M eps, control costs (k_noise's work); 2 = eps and M eps
                                // from nz.pre_eps / pre_meps (k_pregen), then params and control costs
    const double* params;
    long long stride;
    int num_noisy;
    int member;                 // StompOptimizer::iteration_ for the noisy rows
    double* state_out;          // [num_noisy][N]
    uint8_t* cf_out;            // [num_noisy] or null
    double* traj_out;           // [num_noisy][J][N] or null
    double* total_out;          // [num_noisy] or null
    const double* x_params;     // [J][N] or null
    int x_member;
    int pre_rows;               // > 0: blocks after the rollouts make k_pregen's rows of pre_next (the
    NoiseArgs pre_next;         // next iteration) at low priority in the same dispatch
    int ctl_by_pre;             // with fused_noise 2 and pre_rows >= ctl_rows: pregen block r < ctl_rows also
                                // prices this iteration's row r (computeControlCosts, off the rollout's
                                // critical path) and writes its noise / params rows; the (slot-loop)
                                // rollout workgroups skip both (phased ones price their own rows)
    int ctl_rows;               // rows priced by the pregen blocks (num_noisy; all K of a gather-mode rank)
    int row0;                   // rollout e's row in nz's row buffers is row0 + e (gather mode: the
                                // rank's first global rollout; its state goes to state_out[e])
    double* x_state;
    uint8_t* x_cf;
    double* x_traj;
    double* x_total;
    // K_r > 0: the noiseless rollout is also addExtraRollouts' extra rollout (parameters theta,
    // noise 0; policy_improvement.cpp:443-462): its workgroup writes the copy of theta, the zero
    // noise row and the control costs of theta + 0 (k_noise's zero-noise row) when x_ctl is set
    double* x_ctl;
    double* x_prm;
    double* x_nse;
    int split;                  // set by launch_cost: pieces per rollout of k_rollout_split
    int* split_cnt;
    // blocks after the pregen ones: Rollout::getCost of the previous iteration's K rows (the reuse
    // candidates, tot_state [K][N] / tot_control [K][J][N]) into tot_out [K] (launch_reuse_rows
    // ranks them with the extra rollout's)
    int tot_rows;
    const double* tot_state;
    const double* tot_control;
    double* tot_out;
    // blocks after the totals ones (one device, reuse; launch_reuse_pick): every reuse candidate
    // re-based on nz.theta and priced ahead of the ranking, as the reused rows' kernel would price
    // it (price_candidate): c < spec_rows - 1 the previous row c (spec_src), c = spec_rows - 1
    // the extra rollout (params theta), into spec_params / spec_noise / spec_ctl row c
    int spec_rows;
    const double* spec_src;     // [K][J][N]
    double* spec_params;        // [K + 1][J][N]
    double* spec_noise;
    double* spec_ctl;
    // split launches: the extra rollout's theta copy, zero noise and control costs (x_ctl) made by
    // one block after the pricing blocks instead of by the extra rollout's first piece ahead of its
    // row (set by launch_cost when the launch splits and x_ctl is wanted)
    int x_ctl_block;
};

enum WeightMode { W_FUSED = 0, W_MINMAX = 1, W_PSUM = 2, W_USUM = 3 };

struct WeightArgs {
    const int* stop;            // nonzero -> no-op
    int J, N, K_loc, use_cumulative, mode, tc, nb_total;
    const double* state;        // [K][N]
    const double* control;      // [K][J][N]
    const double* noise;        // [K][J][N]
    const double* cum;          // [K][J][N] cumulative costs or null
    double* prob;               // [K][J][N]
    double* u;                  // [J][N] reduced update before the projection (FUSED)
    double* mm;                 // [2][J][N] (max, -min): MINMAX writes local, PSUM reads global
    double* psum_part;          // [nb_loc][J][N]   PSUM writes
    const double* psum_all;     // [nb_total][J][N] USUM reads
    double* u_part;             // [nb_loc][J][N]   USUM writes
};

// The state-cost terms that StompOptimizer::execute adds after the collision cost
// (stomp_optimizer.cpp:1107-1151): the orientation path constraints (:1107-1115) and the
// torque term (KDL::ChainIdSolver_RNE on the inverse-dynamics chain, :1117-1142).  k_terms runs after k_rollout on the same rollouts,
// reading the joint-limited trajectories k_rollout wrote, and finishes
// costs(t) = (w_obs state + w_con con) + w_tq tq in the reference's order.
constexpr int kMaxChain = 32;

struct ChainSeg {
    DevSegment seg;             // pose(q) of the chain segment (parent = previous chain segment)
    double m, h[3], I[9];       // KDL::RigidBodyInertia about the segment origin (h = m c)
};

// OrientationConstraintEvaluator (constraint_evaluator.cpp:50-73) with the FK path of its
// segment (root first), for one lane per waypoint
struct OcDev {
    int seg, body_fixed, path_len;
    int path[kMaxChain];
    double ninv[9];             // nominal_orientation_inverse_ (bullet inverse, host-computed)
    double rw, pw, yw;          // roll / pitch / yaw weights
    double tol[3];              // absolute roll / pitch / yaw tolerance
    double weight;
};

struct TermsModel {
    int J, N, nchain, torque, noc;
    const ChainSeg* chain;      // [nchain], root side first
    const OcDev* oc;            // [noc]
    const DevSegment* segs;     // the whole tree (constraint FK paths)
    double g[3];                // gravity in the chain root frame
    double cv[7], ca[7];        // invTime * DIFF_RULES[0][k], invTime^2 * DIFF_RULES[1][k]
    const double* start;        // [J]
    const double* goal;         // [J]
    double w_con, w_tq;
};

struct TermsArgs {
    const int* stop;            // nonzero -> no-op
    const double* traj;         // [num_noisy][J][N] joint-limited trajectories
    double* state;              // [num_noisy][N] in: w_obs * collision cost; out: the full costs
    double* total;              // [num_noisy] or null
    int num_noisy;
    uint8_t* cs;                // [num_noisy] constraints satisfied, or null
    const double* x_traj;       // the extra (noiseless) rollout, or null
    double* x_state;
    double* x_total;
    uint8_t* x_cs;
    double* tq_out;             // [N] sum_j |tau_j| of rollout 0 (STOMPStatistics.torques), or null
};

// hipFuncAttributeMaxDynamicSharedMemorySize opt-in for more than the default dynamic LDS:
// remembered per (kernel, current device) once it succeeds, thread-safe (engines on several
// devices or host threads share the kernels).  A failure is left for the launch to report, with
// the message of lds_opt_in_error() (this host thread's last failed opt-in, or "").
hipError_t lds_opt_in(const void* kernel, size_t bytes);
const char* lds_opt_in_error();

size_t terms_lds_bytes(const TermsModel& m);
void launch_terms(const TermsModel& m, const TermsArgs& a, hipStream_t s);

void launch_noise(const NoiseArgs& a, hipStream_t s);
// The reuse step with the reused rows' projection and control costs (policy_improvement.cpp:
// 176-225, 473-482): the K previous rows' totals made by the rollout launch (CostArgs::tot_*),
// then one workgroup per reused row prices the extra rollout, ranks the candidates, copies the
// row of rank rr (params, noise re-based on theta, state) and prices it.  Only when
// launch_reuse_rows_ok.
struct ReuseArgs {
    int K, Kr, K_gen, with_extra;
    const double* costs;        // [K + with_extra] candidate totals (launch_reuse, costs only)
    const double* src_params;   // the previous row set
    const double* src_state;
    const double* x_params;     // the extra (noiseless) rollout
    const double* x_state;
    const double* x_control;
    double* state;              // this iteration's state rows (rows K_gen.. written)
    // launch_reuse_pick: the candidates priced by the rollout launch (CostArgs::spec_*, row K the
    // extra rollout)
    const double* spec_params;
    const double* spec_noise;
    const double* spec_ctl;
};
bool launch_reuse_rows_ok(const NoiseArgs& a, int K, int Kr);
void launch_reuse_rows(const NoiseArgs& a, const ReuseArgs& ra, hipStream_t s);
// The reuse step when the rollout launch priced every candidate ahead (CostArgs::spec_*): one
// workgroup per reused row ranks the candidates (the extra rollout's total made here) and copies
// the chosen candidate's priced params / noise / control rows and its state row.  LDS of one
// pricing block of the rollout launch: price_candidate_lds_bytes.
bool launch_reuse_pick_ok(const NoiseArgs& a, int K, int Kr);
// pieces per rollout of a split rollout launch of nro rollouts and extra_blocks pregen / totals /
// pricing blocks (spec: pricing blocks present), 0 when the launch does not split; only a split
// launch carries pricing blocks
int rollout_split_pieces(const DevModel& m, int nro, int extra_blocks, bool spec);
void launch_reuse_pick(const NoiseArgs& a, const ReuseArgs& ra, hipStream_t s);
// launch_reuse_pick folded into the one-wave-per-column weights (K < 64, no cumulative costs):
// the reused rows' params / noise / control (and ra.state) written column by column as the
// weights read them.  Only when launch_weights_pick_ok.
bool launch_weights_pick_ok(const WeightArgs& a, const ReuseArgs& ra);
void launch_weights_pick(const WeightArgs& a, const ReuseArgs& ra, double* params, double* noise, double* control,
                         hipStream_t s);
size_t price_candidate_lds_bytes(int J, int N);
// the theta-independent part of generateRollouts + computeProjectedNoise for rows [0, rows):
// normals, eps = sigma L z and M eps into a.pre_eps / a.pre_meps (run ahead on a side stream)
void launch_pregen(const NoiseArgs& a, int rows, hipStream_t s);

// StompOptimizer::optimize bookkeeping on the device (stomp_optimizer.cpp:301-344), one launch
// after each iteration's noiseless rollout; sets stop when the loop would break
struct DevTrack {
    int stop, cfi, iterations, success, success_iteration, collision_success_iteration, last_improvement_iteration;
    int pad;
    double best;
    // device wall clock (wall_clock64, hipDeviceAttributeWallClockRate) at the loop's start and
    // when the noiseless rollout of success_iteration / collision_success_iteration finished
    // (STOMPStatistics success_duration / collision_success_duration, stomp_optimizer.cpp:306-319)
    unsigned long long t0, t_success, t_collision_success;
};
// stamps DevTrack::t0 (first launch of an optimize loop)
void launch_track_start(DevTrack* tr, hipStream_t s);
void launch_track(DevTrack* tr, int it, int max_it_cf, const double* total, const uint8_t* cf, const uint8_t* cs,
                  double* costs, const double* last_traj, double* best_traj, int JN, hipStream_t s);
void launch_cost(const DevModel& m, const CostArgs& a, hipStream_t s);
bool cost_supported(const DevModel& m);
size_t rollout_lds_bytes(const DevModel& m, int pad_lds, int lean = 0);   // dynamic LDS of the rollout kernel
size_t rollout_phased_lds_bytes(const DevModel& m);        // of the phased wide rollout, 0: does not fit
size_t rollout_static_lds();                                 // its static LDS
int rollout_blocks_per_cu(size_t lds_total, int lean = 0);   // occupancy (LDS and register limits)
bool rollout_lean_allowed(const DevModel& m, int lean);       // lean 2 needs one pair-lane group
// LDS per CU is 160 KiB (MI355X_MICROARCH.md), but three 49.5 KB rollout workgroups did not
// co-reside on one CU in our residency measurements (tools/stamps.py) while three 46.9 KB
// ones did, so the occupancy model budgets 144 KiB
constexpr size_t kLdsPerCu = 144 * 1024;
constexpr size_t kRolloutLdsMax = 156 * 1024;                // dynamic + static per workgroup
void launch_cumulative(const WeightArgs& a, double* cum, hipStream_t s);
void launch_weights(const WeightArgs& a, hipStream_t s);
int weights_tile(int K_loc);
// theta += M u; with delta: delta = M u and theta untouched
void launch_update(int J, int N, const double* MT, const double* u, const double* u_all, int nb_total,
                   double* theta, const int* stop, hipStream_t s, double* delta = nullptr);
// out[i] = max over r < world of gathered[r][i] (the in-process group's all-reduce(max))
// groups of engines of one shape in shared launches (stomp_group_run)
struct UpdateArgs {
    const double* MT;
    const double* u;
    double* theta;
    const int* stop;
};
void launch_cost_group(const DevModel& m0, const DevModel* ms, const CostArgs* as, int engines, int nro, int npre,
                       hipStream_t s);
int weights_group_tiles(int J, int N, int K_loc);
void launch_weights_group(const WeightArgs* as, int engines, int J, int N, int K_loc, hipStream_t s);
void launch_update_group(int J, int N, const UpdateArgs* as, int engines, hipStream_t s);
void launch_gather_max(const double* gathered, int world, int n, double* out, hipStream_t s);
void launch_pad_fk(const DevModel& m, const double* start, const double* goal, double* pad_pos, int* pad_cf,
                   hipStream_t s);
// src_*: the previous iteration's rows (ranked, copied from); params / noise / state: this
// iteration's rows K_gen.. (written).  The two row sets must be distinct buffers (the copy has no
// staging pass); returns -1 without launching when they alias, -2 when one candidate's cost rows
// (or the ranking's totals) do not fit the LDS.  costs_g: [K + 1] scratch totals, count: a
// counter that is zero between launches (the last workgroup resets it).
int launch_reuse(int K, int J, int N, int Kr, int K_gen, int with_extra, const double* src_params,
                 const double* src_state, const double* src_control, double* params, double* noise, double* state,
                 const double* x_params, const double* x_state, const double* x_control, const double* theta,
                 double* costs_g, int* count, const int* stop, hipStream_t s, bool costs_only = false);
// sharded reuse (world > 1): per-rank totals, the replicated ranking, pack / unpack of the slots
// noise = eps, params = theta_gen + eps of rows left in a pregen buffer (rows_in_pre)
void launch_materialize_rows(int K_loc, int JN, const double* eps, const double* theta_gen, double* noise,
                             double* params, hipStream_t s);
void launch_reuse_totals(int K_loc, int J, int N, const double* state, const double* control, const double* x_state,
                         const double* x_control, double* tot_loc, double* tot_x, const int* stop, hipStream_t s);
void launch_reuse_select(int K, int Kr, int with_extra, const double* tot_all, const double* tot_x, int* sel,
                         const int* stop, hipStream_t s);
void launch_reuse_pack(int Kr, int J, int N, int first, int K_loc, const int* sel, const double* params,
                       const double* state, double* slot, const int* stop, hipStream_t s);
void launch_reuse_unpack(int Kr, int K_gen, int J, int N, int first, int K_loc, const int* sel,
                         const double* slot_all, const double* x_params, const double* x_state, const double* theta,
                         double* params, double* noise, double* state, const int* stop, hipStream_t s);
void launch_sdf_build(int nx, int ny, int nz, int cap2, const int* boxes /*n x 6 idx ranges*/, int nb,
                      const long long* cyl_d2 /*nc x nx x ny*/, const int* cyl_z /*nc x 2*/, int nc,
                      unsigned short* out, hipStream_t s);

// the reference's object voxeliser (k_sdf.hip); shape types as STOMP_SHAPE_* / STOMP_BODY_*
constexpr int kShapeBox = 0, kShapeCylinder = 1, kBodySphere = 2, kBodyBox = 3, kBodyCylinder = 4, kBodyMesh = 5;
struct SdfMarkArgs {
    int n[3];
    double o[3];
    double inv_res;              // 1.0 / res (VoxelGrid oo_resolution)
    unsigned char* occ;          // nx*ny*nz marks
    unsigned long long* marked;  // points that landed inside the grid
};
struct SdfLatticeJob {
    int type;
    int n[3];                    // lattice points per axis
    int off[3];                  // environment objects: offsets of the axis coordinate lists
    int lo[3];                   // robot bodies: first lattice index per axis
    double pos[3];               // lattice centre (the bounding sphere's for bodies)
    double R[9];                 // KDL Rotation::Quaternion (objects) / btMatrix3x3 basis (bodies)
    double dims[3];
    double res;
    double org[3];               // meshes: the body's position (pos is its bounding-sphere centre)
    const double* planes;        // meshes: nplanes x (n, d) of the convex hull, device memory
    int nplanes;
};
void launch_mark_lattice(const SdfLatticeJob& j, const double* axes, const SdfMarkArgs& g, hipStream_t s);
void launch_mark_points(const double* pts, long long np, const SdfMarkArgs& g, hipStream_t s);
void launch_edt(int nx, int ny, int nz, int cap, const unsigned char* occ, unsigned short* a, unsigned short* b,
                unsigned short* field, hipStream_t s);
// the [nx][ny][nz] field re-laid as 4^3 bricks (DevModel::brick) into dst, ceil(n / 4)^3 bricks;
// voxels of the padding bricks past the grid are 0 (never read: the lookup's range test)
void launch_sdf_bricks(const unsigned short* src, unsigned short* dst, int nx, int ny, int nz, hipStream_t s);
inline size_t sdf_brick_cells(int nx, int ny, int nz)
{
    return (size_t)((nx + 3) / 4) * ((ny + 3) / 4) * ((nz + 3) / 4) * 64;
}

}  // namespace stomp
