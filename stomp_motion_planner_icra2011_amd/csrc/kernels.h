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
//   sdf              [nx][ny][nz]          fp32  distance field (z fastest)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace stomp {

constexpr int kMaxJoints = 32;
constexpr int kRunMax = 12;      // spheres processed per FK op (LDS batch)
constexpr int kSlots = 4;        // live FK frames per thread
constexpr int kSumBlock = 64;    // canonical blocked summation over rollouts

struct DevSegment {
    int parent, q_index;
    double rot[9];
    double trans[3];
    double axis[3];
};

struct DevSphere {
    int segment, pad_;
    double radius, clearance, inv_clearance;
    double pos[3];
};

// One FK program step: frame[to] = frame[from] * pose(seg, q) (seg < 0: reuse frame `to`),
// then emit spheres [sph_begin, sph_end) from frame[to].  from = -1: identity parent.
struct FkOp {
    int seg, from, to, sph_begin, sph_end;
};

struct DevModel {
    int J, N, Nall, S, nops;
    const DevSegment* segs;
    const DevSphere* sph;
    const FkOp* ops;
    const double* pad_pos;      // [12][S][3]
    const float* sdf;
    int nx, ny, nz;
    double ox, oy, oz, res;
    const double* start;        // [J]
    const double* goal;         // [J]
    double vel_coef[7];         // invTime * DIFF_RULES[0][k]
    double w_obs, w_con, w_tq;
    int pad_collision;
    const int* has_limits;      // [J]
    const double* jmin;         // [J]
    const double* jmax;         // [J]
    const double* QT;           // [J][N][N]
};

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
    int zero_noise;             // extra rollout: params given, noise = 0 (addExtraRollouts)
};

struct WeightArgs {
    int J, N, K_loc, use_cumulative;
    const double* state;        // [K][N]
    const double* control;      // [K][J][N]
    const double* noise;        // [K][J][N]
    double* cum;                // [K][J][N] scratch (cumulative costs) or null
    double* prob;               // [K][J][N]
    double* u;                  // [J][N] reduced update (before projection)
};

void launch_noise(const NoiseArgs& a, int rollouts_per_block, hipStream_t s);
void launch_rollout_cost(const DevModel& m, const double* params, long long param_stride, int num,
                         double* state_out, uint8_t* cf_out, double* traj_out, double* total_out,
                         int iteration_member, hipStream_t s);
void launch_cumulative(const WeightArgs& a, hipStream_t s);
void launch_weights(const WeightArgs& a, hipStream_t s);
void launch_update(int J, int N, const double* MT, const double* u, double* theta, hipStream_t s);
void launch_pad_fk(const DevModel& m, const double* start, const double* goal, double* pad_pos, int* pad_cf,
                   hipStream_t s);
void launch_reuse(int K, int J, int N, int Kr, int K_gen, int with_extra, double* params, double* noise,
                  double* state, const double* control, const double* x_params, const double* x_state,
                  const double* x_control, const double* theta, double* tmp_params, double* tmp_state,
                  hipStream_t s);
void launch_sdf_build(int nx, int ny, int nz, int cap2, double res, const int* boxes /*n x 6 idx ranges*/,
                      int nb, const long long* cyl_d2 /*nc x nx x ny*/, const int* cyl_z /*nc x 2*/, int nc,
                      float* out, hipStream_t s);

}  // namespace stomp
