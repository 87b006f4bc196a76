// engine.cpp -- host side of the C ABI in include/stomp_engine.h.
//
// One stomp_engine = one planning problem resident on one device: setup matrices,
// distance field, rollout arrays and the policy theta live in HBM for the
// engine's lifetime; an iteration is a fixed sequence of kernel launches on the
// engine stream with no host synchronisation (stomp_engine_run), or with one
// 9-byte read-back (stomp_engine_iterate, the runSingleIteration contract).
#include "stomp_engine.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "kernels.h"
#include "setup.h"

#ifdef STOMP_WITH_RCCL
#include <rccl/rccl.h>
#endif

using namespace stomp;

namespace {

thread_local std::string g_last_error;

enum TimerId { T_NOISE = 0, T_COST, T_WEIGHTS, T_UPDATE, T_NOISELESS, T_REUSE, T_TERMS, T_PREGEN, T_COUNT };
const char* kTimerNames[T_COUNT] = {"noise", "rollout_cost", "weights", "update", "noiseless", "reuse", "state_terms",
                                    "pregen"};

// In-process exchange group: the ranks of one sharded problem as engines of ONE process, each
// driven by its own host thread (one per device, or several on one device).  The collectives are
// device-to-device copies on the ranks' own streams, ordered by HIP events and two host barriers
// per collective (publish -> copy -> done), in place of RCCL.  Created by stomp_comm_local_id.
constexpr char kLocalMagic[8] = {'S', 'T', 'O', 'M', 'P', 'L', 'O', 'C'};

struct LocalGroup {
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    struct Slot {
        const void* src = nullptr;
        hipEvent_t ready = nullptr, done = nullptr;
        int device = 0;
    };
    std::vector<Slot> slot;
    std::vector<char> joined;
    long long phase = 0;    // completed barrier phases
    int arrived = 0;
    // the decomposition every rank must run (gather, K, J, N), set by the first rank to join: a
    // rank that disagrees would post different collectives, so its creation fails instead
    bool has_sig = false;
    long long sig[6] = {0, 0, 0, 0, 0, 0};   // gather, K, J, N, K_r, split_modes (stomp_engine_create)
    bool broken = false;    // a rank timed out: every later barrier fails at once
    // all ranks arrive (or the wait times out: a rank not driven from a thread of its own)
    bool barrier(std::unique_lock<std::mutex>& lk)
    {
        if (broken) return false;
        const long long my = phase;
        if (++arrived == world) {
            arrived = 0;
            ++phase;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return phase != my || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

std::mutex g_groups_mu;
std::map<uint64_t, std::shared_ptr<LocalGroup>> g_groups;   // created, not yet joined by every rank
uint64_t g_next_group = 1;

}  // namespace

struct stomp_engine {
    std::string err;
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int J = 0, N = 0, Nall = 0, K = 0, Kr = 0, K_loc = 0, first = 0, S = 0, nseg = 0;
    int world = 1, rank = 0;
    bool split_modes = false;   // weights in the MINMAX / PSUM / USUM phases (world > 1, or the debug hook)
    // gather mode (world > 1, small K N): every rank makes and prices the noise rows of all K rollouts
    // (counter-based, so no noise moves), evaluates its own K_loc, and one all-gather of the state-cost
    // rows per iteration gives every rank the whole cost matrix for the fused weights and the update
    bool gather = false;
    int rows = 0, row0 = 0;   // rollout rows held per iteration (K_loc, or K in gather mode); own rows' offset
    // the decomposition measured at creation (calibrate_shard_mode): both are possible and none was
    // requested, so the buffers hold all K rows and the ranks time each decomposition's compute and
    // collectives, then pick the faster.  shard_info: mode, T_gather, T_partials (us per iteration
    // without exchanges), L_allreduce, L_allgather_state, L_allgather_partials (us per collective)
    bool calibrate = false;
    double shard_info[6] = {0, 0, 0, 0, 0, 0};
    uint64_t seed = 0;
    double disc = 0.05, w_smooth = 0, w_obs = 0, w_con = 0, w_tq = 0;
    double smooth[3] = {0, 0, 0};
    int use_cum = 0, max_it = 0, max_it_cf = 0;
    std::vector<double> sig_std, sig_dec, start, goal;
    SetupOutput su;
    DevModel model{};
    TermsModel terms{};
    bool terms_on = false;      // torque term / path constraints: k_terms after every k_rollout
    double* d_terms_traj = nullptr;   // [K_loc][J][N] joint-limited trajectories for k_terms
    uint8_t* d_cs = nullptr;          // last_trajectory_constraints_satisfied_ of the noiseless rollout
    DevTrack* d_track = nullptr;      // device-resident optimize loop state; d_track->stop gates every launch
    const int* d_stop = nullptr;
    double* d_opt_costs = nullptr;    // [max_iterations] last_trajectory_cost_ per iteration
    DevTrack* h_track = nullptr;      // pinned read-back slots
    bool tracking = false;            // inside stomp_engine_optimize: k_track after each noiseless rollout
    std::vector<FkOp> ops;
    std::vector<int> sphere_slot;   // published frame slot of each sphere's segment
    int nslots = 0;
    std::vector<void*> allocs;
    double *d_theta = nullptr, *d_LT = nullptr, *d_MT = nullptr, *d_QT = nullptr;
    double *d_params = nullptr, *d_noise = nullptr, *d_control = nullptr, *d_prob = nullptr, *d_state = nullptr;
    // K_r > 0: a second set of rollout rows.  Each reusing iteration swaps the sets, so the
    // previous iteration's rows (ranked and copied by the reuse kernels) stay intact while this
    // iteration's rollout launch writes its generated rows; row_set counts the swaps mod 2
    double *d_params_b = nullptr, *d_noise_b = nullptr, *d_control_b = nullptr, *d_state_b = nullptr;
    int row_set = 0;
    double *d_cum = nullptr, *d_u = nullptr;
    double *d_x_params = nullptr, *d_x_noise = nullptr, *d_x_control = nullptr, *d_x_state = nullptr;
    double *d_last_traj = nullptr, *d_best_traj = nullptr, *d_total = nullptr;
    double *d_pad_pos = nullptr, *d_start = nullptr, *d_goal = nullptr;
    // sharded reuse (world > 1, K_r > 0): per-rank totals, all totals, the extra's total, the
    // chosen rows' slots [Kr][J N + N] and their all-gather [world][Kr][J N + N], the ranking
    double *d_tot_loc = nullptr, *d_tot_all = nullptr, *d_tot_x = nullptr, *d_slot = nullptr, *d_slot_all = nullptr;
    double* d_reuse_costs = nullptr;   // one device: k_reuse's totals [K + 1] and its counter
    int* d_reuse_count = nullptr;
    // one device, reuse: every candidate priced ahead by the rollout launch (CostArgs::spec_*),
    // [K + 1][J][N] each (row K the extra rollout); spec_on: allocated (STOMP_DEBUG_NO_SPEC=1: not)
    double *d_spec_params = nullptr, *d_spec_noise = nullptr, *d_spec_ctl = nullptr;
    bool spec_on = false;
    // the copy of the chosen candidates in the weights launch (STOMP_DEBUG_NO_PICK_FUSE=1: k_reuse_pick)
    bool pick_fuse = true;
    int* d_sel = nullptr;
    uint8_t* d_cf = nullptr;
    uint16_t* d_sdf = nullptr;   // d2 per voxel (the engine's bricked copy when model.brick)
    const uint16_t* d_sdf_caller = nullptr;   // the caller's device field (data_on_device), or null
    int grid_n[3] = {0, 0, 0};
    int* d_pad_cf = nullptr;
    int pad_collision = 0;
    bool reused_next = false, extra_added = false;
    int pending_member = -1;   // iteration_ of a noiseless rollout of theta not evaluated yet
    double *d_mm = nullptr, *d_psum_part = nullptr, *d_psum_all = nullptr, *d_u_part = nullptr, *d_u_all = nullptr;
    int K_gen = 0;
    // pregen (K_r = 0, fused noise phase): the normals, eps = sigma L z and M eps of iteration
    // it + 1 are made by extra low-priority blocks of iteration it's rollout launch; the rollout
    // launch of it + 1 reads them.  Two buffers, by iteration parity: a rollout launch reads one
    // and fills the other.
    bool pre_on = false;
    int pre_it = -1;                  // iteration whose rows are in d_pre_eps / d_pre_meps[it & 1] (enqueued)
    double *d_pre_eps[2] = {nullptr, nullptr}, *d_pre_meps[2] = {nullptr, nullptr};
    // the last iteration left its rows in d_pre_eps (rows_eps) instead of copying them into
    // d_noise / d_params (run / iterate with pregen rows); materialize_rows writes them on demand
    bool rows_in_pre = false;
    const double* rows_eps = nullptr;
    double* d_theta_gen = nullptr;
    double* h_total = nullptr;
    uint8_t* h_cf = nullptr;
    // eval scratch
    int eval_cap = 0;
    double *d_eval_params = nullptr, *d_eval_costs = nullptr, *d_eval_traj = nullptr;
    uint8_t* d_eval_cf = nullptr;
    uint8_t* d_eval_cs = nullptr;
    // timing
    bool timing = false;
    struct Ev {
        int id;
        hipEvent_t a, b;
    };
    std::vector<Ev> evs;
    std::vector<hipEvent_t> pool;
    double tot_ms[T_COUNT] = {0};
    int launches[T_COUNT] = {0};
#ifdef STOMP_WITH_RCCL
    ncclComm_t comm = nullptr;
#endif
    // bounded waits over RCCL (sync_stream): the last collective posted (name, iteration, count),
    // the deadline (STOMP_COMM_TIMEOUT_S, default 300 s), and the aborted communicator's message
    const char* coll_name = "none";
    int coll_it = -1;
    long long coll_count = 0;
    int cur_it = -1;
    double comm_timeout_s = 300.0;
    bool comm_aborted = false;
    std::string comm_msg;
    // STOMP_DEBUG_STALL_COLLECTIVE=n (tests): the n-th collective is withheld and the stream made
    // to wait on h_stall instead (a rank that never posts it); released after the abort
    long long stall_at = 0;
    unsigned* h_stall = nullptr;
    // an event behind each of the last kCollRing collectives: the message names the first one not
    // complete (the stuck one), not only the last one posted
    static constexpr int kCollRing = 32;
    struct CollRec {
        hipEvent_t ev = nullptr;
        const char* name = "";
        int it = -1;
        long long n = 0;
    } coll_ring[kCollRing];
    // PolicyImprovement API (stomp_pi_*): the weight the control-cost rows were priced with,
    // improvePolicy's update (J x N)
    double pi_weight = 0.0;
    double* d_delta = nullptr;
    // STOMPStatistics.torques (stomp_optimizer.cpp:384-398): the torque chain's model whenever
    // inertias are given (also with the torque term off), its per-waypoint output
    bool torque_stats = false;
    TermsModel tq_model{};
    double *d_tq = nullptr, *d_tq_state = nullptr;
    int wall_khz = 0;
    std::shared_ptr<LocalGroup> local;   // in-process exchange group (stomp_comm_local_id), or null
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
    double* d_mm_all = nullptr;          // [world][2][J][N] gathered (max, -min) of a local group
};

namespace {


int fail(stomp_engine* e, int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (e) e->err = buf;
    g_last_error = buf;
    return code;
}

// Every C-ABI entry on an engine runs with the engine's device current (allocations, launches
// and attribute opt-ins land there) and restores the caller's device on return.
struct DeviceGuard {
    int prev = -1, dev;
    explicit DeviceGuard(int d) : dev(d)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
};

#define HIP_TRY(e, x)                                                                          \
    do {                                                                                       \
        hipError_t _st = (x);                                                                  \
        if (_st != hipSuccess)                                                                 \
            return fail((e), STOMP_E_DEVICE, "%s failed: %s", #x, hipGetErrorString(_st));     \
    } while (0)

// hipStreamSynchronize of the engine stream, bounded when collectives are in it: over RCCL the
// wait polls the stream and the communicator's asynchronous error, and after STOMP_COMM_TIMEOUT_S
// seconds without completion (a rank that never posts its side of a collective, a mismatched
// sequence) or on an RCCL error it aborts the communicator (ncclCommAbort also releases RCCL
// kernels still waiting) and fails with STOMP_E_COMM naming the last collective posted.  Every
// later call on the engine fails the same way.
int sync_stream(stomp_engine* e)
{
#ifdef STOMP_WITH_RCCL
    if (e->comm_aborted) return fail(e, STOMP_E_COMM, "%s", e->comm_msg.c_str());
    if (e->comm) {
        const auto t0 = std::chrono::steady_clock::now();
        for (long long n = 0;; ++n) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) return 0;
            if (q != hipErrorNotReady)
                return fail(e, STOMP_E_DEVICE, "hipStreamQuery failed: %s", hipGetErrorString(q));
            ncclResult_t ae = ncclSuccess;
            const ncclResult_t qr = ncclCommGetAsyncError(e->comm, &ae);
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            const bool err = qr != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress);
            if (err || el > e->comm_timeout_s) {
                char buf[400];
                if (err)
                    snprintf(buf, sizeof buf, "rank %d: RCCL error (%s) with collectives in flight",
                             e->rank, ncclGetErrorString(qr != ncclSuccess ? qr : ae));
                else
                    snprintf(buf, sizeof buf, "rank %d: collectives did not complete within %.1f s (STOMP_COMM_TIMEOUT_S)",
                             e->rank, e->comm_timeout_s);
                std::string stuck = "unknown (older than the last 32)";
                for (long long k = std::max(1LL, e->coll_count - stomp_engine::kCollRing + 1); k <= e->coll_count; ++k) {
                    const auto& r = e->coll_ring[k % stomp_engine::kCollRing];
                    if (r.n == k && r.ev && hipEventQuery(r.ev) == hipErrorNotReady) {
                        stuck = std::string(r.name) + " of iteration " + std::to_string(r.it) + " (#" + std::to_string(k) + ")";
                        break;
                    }
                }
                (void)hipGetLastError();
                e->comm_msg = std::string(buf) + "; first collective not complete: " + stuck + "; last posted: " +
                              e->coll_name + " of iteration " + std::to_string(e->coll_it) + " (#" +
                              std::to_string(e->coll_count) + "); communicator aborted";
                // the test hook's wait first: its withheld collective's successors are queued behind
                // it and have not started, so the abort would wait for them
                if (e->h_stall) __atomic_store_n(e->h_stall, 1u, __ATOMIC_SEQ_CST);
                ncclCommAbort(e->comm);
                e->comm = nullptr;
                e->comm_aborted = true;
                (void)hipStreamSynchronize(e->stream);   // the aborted collectives drain
                (void)hipGetLastError();
                return fail(e, STOMP_E_COMM, "%s", e->comm_msg.c_str());
            }
            if (n > 2000) std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
    }
#endif
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    return 0;
}

#define SYNC_TRY(e)                        \
    do {                                   \
        const int _rc = sync_stream(e);    \
        if (_rc) return _rc;               \
    } while (0)

template <class T>
int dev_alloc(stomp_engine* e, T** p, size_t n)
{
    void* q = nullptr;
    if (n == 0) n = 1;
    hipError_t st = hipMalloc(&q, n * sizeof(T));
    if (st != hipSuccess) return fail(e, STOMP_E_DEVICE, "hipMalloc(%zu bytes): %s", n * sizeof(T), hipGetErrorString(st));
    hipMemsetAsync(q, 0, n * sizeof(T), e->stream);
    e->allocs.push_back(q);
    *p = (T*)q;
    return 0;
}

template <class T>
int upload(stomp_engine* e, T** p, const T* src, size_t n)
{
    int rc = dev_alloc(e, p, n);
    if (rc) return rc;
    if (n) HIP_TRY(e, hipMemcpyAsync(*p, src, n * sizeof(T), hipMemcpyHostToDevice, e->stream));
    return 0;
}

hipEvent_t get_event(stomp_engine* e)
{
    if (!e->pool.empty()) {
        hipEvent_t ev = e->pool.back();
        e->pool.pop_back();
        return ev;
    }
    hipEvent_t ev;
    hipEventCreate(&ev);
    return ev;
}

struct Timed {
    stomp_engine* e;
    int id;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    Timed(stomp_engine* e_, int id_, hipStream_t s_ = nullptr) : e(e_), id(id_), s(s_ ? s_ : e_->stream)
    {
        if (e->timing) {
            a = get_event(e);
            b = get_event(e);
            hipEventRecord(a, s);
        }
    }
    ~Timed()
    {
        if (e->timing) {
            hipEventRecord(b, s);
            e->evs.push_back({id, a, b});
        }
    }
};

void collect_timing(stomp_engine* e)
{
    if (e->evs.empty()) return;
    hipStreamSynchronize(e->stream);
    for (auto& v : e->evs) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, v.a, v.b);
        e->tot_ms[v.id] += ms;
        e->launches[v.id] += 1;
        e->pool.push_back(v.a);
        e->pool.push_back(v.b);
    }
    e->evs.clear();
}

// FK program: frames of the segments that carry spheres or are their ancestors, in
// DFS order, each composed from its parent's live slot; sphere runs emitted in list
// order right after their segment's frame (requires sphere segments non-decreasing).
int plan_fk(stomp_engine* e, const stomp_engine_desc* d, std::vector<FkOp>& ops)
{
    const int ns = d->num_segments;
    std::vector<char> needed(ns, 0);
    int prev = -1;
    for (int j = 0; j < d->num_spheres; ++j) {
        int s = d->spheres[j].segment;
        if (s < prev)
            return fail(e, STOMP_E_UNSUPPORTED,
                        "sphere list must be ordered by segment (sphere %d on segment %d after segment %d)", j, s, prev);
        prev = s;
        for (int a = s; a >= 0 && !needed[a]; a = d->segments[a].parent) needed[a] = 1;
    }
    // DFS order: the next needed segment after s is its first needed child, so a chain
    // continues from the running frame C; a segment with several needed children is saved
    // and its later children start from the saved copy.
    std::vector<int> remaining(ns, 0), slot_of(ns, -1);
    for (int s = 0; s < ns; ++s)
        if (needed[s] && d->segments[s].parent >= 0) remaining[d->segments[s].parent]++;
    bool used[kSaves] = {false, false};
    const int runmax = run_max(d->num_time_steps);
    int sph = 0, cur = -1;
    for (int s = 0; s < ns; ++s) {
        if (!needed[s]) continue;
        const int p = d->segments[s].parent;
        int base;
        if (p < 0) base = kBaseRoot;
        else if (p == cur) base = kBaseChain;
        else if (slot_of[p] >= 0) base = slot_of[p];
        else return fail(e, STOMP_E_UNSUPPORTED, "FK planner: parent frame of segment %d not available", s);
        if (p >= 0 && --remaining[p] == 0 && slot_of[p] >= 0) {
            used[slot_of[p]] = false;   // read by this step before any save below overwrites it
            slot_of[p] = -1;
        }
        int save = -1;
        if (remaining[s] >= 2) {
            for (int k = 0; k < kSaves; ++k)
                if (!used[k]) { used[k] = true; save = k; break; }
            if (save < 0) return fail(e, STOMP_E_UNSUPPORTED, "kinematic tree needs more than %d saved frames", kSaves);
            slot_of[s] = save;
        }
        cur = s;
        int b = sph;
        while (sph < d->num_spheres && d->spheres[sph].segment == s) ++sph;
        const int slot = sph > b ? e->nslots++ : -1;
        for (int j = b; j < sph; ++j) e->sphere_slot[j] = slot;
        bool first = true;
        for (int a = b; a < sph || first; a += runmax) {
            FkOp o;
            o.seg = first ? s : -1;
            o.base = first ? base : kBaseChain;
            o.save = first ? save : -1;
            o.slot = first ? slot : -1;
            o.sph_begin = std::min(a, sph);
            o.sph_end = std::min(a + runmax, sph);
            ops.push_back(o);
            first = false;
        }
    }
    return 0;
}

// the torque term's chain (stomp_robot_model.cpp:185-189): segments below torque_root up to
// torque_tip, root side first; its joints must be the group's joints in order.  Returns an
// error message, or nullptr.
const char* torque_chain(const stomp_engine_desc* d, std::vector<int>& path)
{
    path.clear();
    if (!d->inertias) return "torque term needs segment inertias";
    if (d->torque_root < 0 || d->torque_root >= d->num_segments || d->torque_tip < 0 ||
        d->torque_tip >= d->num_segments)
        return "torque chain root/tip out of range";
    for (int sgi = d->torque_tip; sgi != d->torque_root; sgi = d->segments[sgi].parent) {
        if (sgi < 0 || (int)path.size() == kMaxChain) return "torque tip is not below the torque root (or chain too long)";
        path.push_back(sgi);
    }
    std::reverse(path.begin(), path.end());
    int nj = 0;
    for (int sgi : path)
        if (d->segments[sgi].q_index >= 0 && d->segments[sgi].q_index != nj++) return "torque chain joints must be the group joints in order";
    if (nj != d->num_joints) return "torque chain joints must be the group joints in order";
    return nullptr;
}

// OrientationConstraintEvaluator ctor (constraint_evaluator.cpp:50-73): tf::quaternionMsgToTF
// (normalises when |q|^2 is off by more than 0.1), btMatrix3x3(btQuaternion), inverse()
// (bullet LinearMath, double precision), restated as in the oracle
void oc_nominal_inverse(const double* q, double* O)
{
    double x = q[0], y = q[1], z = q[2], w = q[3];
    const double l2 = x * x + y * y + z * z + w * w;
    if (std::fabs(l2 - 1.0) > 0.1f) {
        const double inv = 1.0 / std::sqrt(l2);
        x *= inv; y *= inv; z *= inv; w *= inv;
    }
    const double d = x * x + y * y + z * z + w * w;
    const double s = 2.0 / d;
    const double xs = x * s, ys = y * s, zs = z * s;
    const double wx = w * xs, wy = w * ys, wz = w * zs;
    const double xx = x * xs, xy = x * ys, xz = x * zs;
    const double yy = y * ys, yz = y * zs, zz = z * zs;
    const double M[9] = {1.0 - (yy + zz), xy - wz, xz + wy, xy + wz, 1.0 - (xx + zz), yz - wx,
                         xz - wy, yz + wx, 1.0 - (xx + yy)};
    auto cof = [&](int r1, int c1, int r2, int c2) { return M[3 * r1 + c1] * M[3 * r2 + c2] - M[3 * r1 + c2] * M[3 * r2 + c1]; };
    const double co0 = cof(1, 1, 2, 2), co1 = cof(1, 2, 2, 0), co2 = cof(1, 0, 2, 1);
    const double det = M[0] * co0 + M[1] * co1 + M[2] * co2;
    const double sc = 1.0 / det;
    O[0] = co0 * sc; O[1] = cof(0, 2, 2, 1) * sc; O[2] = cof(0, 1, 1, 2) * sc;
    O[3] = co1 * sc; O[4] = cof(0, 0, 2, 2) * sc; O[5] = cof(0, 2, 1, 0) * sc;
    O[6] = co2 * sc; O[7] = cof(0, 1, 2, 0) * sc; O[8] = cof(0, 0, 1, 1) * sc;
}

void release(stomp_engine* e)
{
    if (!e) return;
    if (e->stream) hipStreamSynchronize(e->stream);
    for (auto& v : e->evs) { hipEventDestroy(v.a); hipEventDestroy(v.b); }
    for (auto ev : e->pool) hipEventDestroy(ev);
    for (void* p : e->allocs) hipFree(p);
    if (e->h_total) hipHostFree(e->h_total);
    if (e->h_cf) hipHostFree(e->h_cf);
    if (e->h_track) hipHostFree(e->h_track);
    if (e->h_stall) hipHostFree(e->h_stall);
    for (auto& r : e->coll_ring)
        if (r.ev) hipEventDestroy(r.ev);
#ifdef STOMP_WITH_RCCL
    if (e->comm) ncclCommDestroy(e->comm);   // null once aborted (sync_stream)
#endif
    if (e->ev_ready) hipEventDestroy(e->ev_ready);
    if (e->ev_done) hipEventDestroy(e->ev_done);
    if (e->own_stream && e->stream) hipStreamDestroy(e->stream);
}

// Task::execute of a launch's rollouts
void launch_rollouts(stomp_engine* e, const CostArgs& ca)
{
    DevModel& m = e->model;
    const int nro = ca.num_noisy + (ca.x_params ? 1 : 0);
    if (m.lean && m.nsaves > 0 && nro > m.sv_rows) {
        // an eval batch with more rollouts than the lean layout's saved-frame blocks: grow them (the
        // old blocks stay allocated until the engine is destroyed, launches before may use them).
        // Without the memory the engine takes the full layout, which is valid for every launch.
        void* q = nullptr;
        if (hipMalloc(&q, sizeof(double) * (size_t)nro * m.nsaves * 12 * m.N) == hipSuccess) {
            e->allocs.push_back(q);
            m.sv_glob = (double*)q;
            m.sv_rows = nro;
        } else {
            (void)hipGetLastError();
            m.lean = 0;
        }
    }
    launch_cost(m, ca, e->stream);
}

// the state-cost terms after the collision cost (k_terms), on the rollouts a k_rollout
// launch with these arguments evaluated; its trajectories must have been written
void launch_terms_for(stomp_engine* e, const CostArgs& ca, uint8_t* cs = nullptr)
{
    if (!e->terms_on) return;
    Timed tm(e, T_TERMS);
    TermsArgs ta{};
    ta.stop = e->d_stop;
    ta.traj = ca.traj_out; ta.state = ca.state_out; ta.total = ca.total_out; ta.num_noisy = ca.num_noisy;
    ta.cs = cs;
    if (ca.x_params) {
        ta.x_traj = ca.x_traj; ta.x_state = ca.x_state; ta.x_total = ca.x_total; ta.x_cs = e->d_cs;
    }
    launch_terms(e->terms, ta, e->stream);
}

// the optimize loop's bookkeeping for the noiseless rollout a launch with these arguments
// evaluated (its iteration_ is ca.x_member)
void track_noiseless(stomp_engine* e, const CostArgs& ca)
{
    if (!e->tracking || !ca.x_params) return;
    launch_track(e->d_track, ca.x_member, e->max_it_cf, e->d_total, e->d_cf, e->d_cs, e->d_opt_costs, e->d_last_traj,
                 e->d_best_traj, e->J * e->N, e->stream);
}

NoiseArgs noise_args(const stomp_engine* e, int it);

// noiseless rollout of the current theta (policy_improvement_loop.cpp:180-182), alone
void launch_noiseless(stomp_engine* e, int member)
{
    CostArgs ca{};
    ca.stop = e->d_stop;
    ca.num_noisy = 0;
    ca.x_params = e->d_theta; ca.x_member = member;
    ca.x_state = e->d_x_state; ca.x_cf = e->d_cf; ca.x_traj = e->d_last_traj; ca.x_total = e->d_total;
    if (e->Kr > 0) {   // it is also the extra rollout of the next reuse ranking
        ca.nz = noise_args(e, member + 1);
        ca.x_ctl = e->d_x_control; ca.x_prm = e->d_x_params; ca.x_nse = e->d_x_noise;
    }
    {
        Timed tm(e, T_NOISELESS);
        launch_rollouts(e, ca);
    }
    launch_terms_for(e, ca);
    track_noiseless(e, ca);
}

// noise / params rows of an iteration that left them in its pregen buffer
void materialize_rows(stomp_engine* e)
{
    if (!e->rows_in_pre) return;
    launch_materialize_rows(e->rows, e->J * e->N, e->rows_eps, e->d_theta_gen, e->d_noise, e->d_params, e->stream);
    e->rows_in_pre = false;
}

int flush_noiseless(stomp_engine* e)
{
    if (e->pending_member >= 0) {
        launch_noiseless(e, e->pending_member);
        e->pending_member = -1;
    }
    return 0;
}


#ifdef STOMP_WITH_RCCL
#define NCCL_TRY(e, x)                                                                       \
    do {                                                                                     \
        ncclResult_t _r = (x);                                                               \
        if (_r != ncclSuccess) return fail((e), STOMP_E_COMM, "%s: %s", #x, ncclGetErrorString(_r)); \
    } while (0)

// a collective about to be posted on the engine stream: recorded for sync_stream's message;
// returns 1 when the STOMP_DEBUG_STALL_COLLECTIVE hook withholds it (the stream then waits on
// h_stall, as behind a rank that never posts it)
int coll_post(stomp_engine* e, const char* name)
{
    e->coll_name = name;
    e->coll_it = e->cur_it;
    ++e->coll_count;
    if (e->stall_at > 0 && e->coll_count == e->stall_at && e->h_stall) {
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, e->h_stall, 0) == hipSuccess &&
            hipStreamWaitValue32(e->stream, dp, 1u, hipStreamWaitValueEq, 0xFFFFFFFFu) == hipSuccess)
            return 1;
        (void)hipGetLastError();
    }
    return 0;
}

// the event behind the collective coll_post just recorded (or withheld)
void coll_mark(stomp_engine* e)
{
    auto& r = e->coll_ring[e->coll_count % stomp_engine::kCollRing];
    if (!r.ev && hipEventCreateWithFlags(&r.ev, hipEventDisableTiming) != hipSuccess) {
        r.ev = nullptr;
        (void)hipGetLastError();
        return;
    }
    r.name = e->coll_name;
    r.it = e->coll_it;
    r.n = e->coll_count;
    (void)hipEventRecord(r.ev, e->stream);
}
#endif

// all-gather of n doubles per rank, rank order, over the in-process group: publish the send
// buffer with an event recorded after its producer; after the first barrier every rank copies
// every rank's buffer behind that rank's event; after the second barrier every rank's stream
// waits for every rank's copies, so no rank overwrites a buffer another still reads
int local_gather(stomp_engine* e, const double* send, double* recv, size_t n)
{
    LocalGroup& g = *e->local;
    HIP_TRY(e, hipEventRecord(e->ev_ready, e->stream));
    std::unique_lock<std::mutex> lk(g.mu);
    g.slot[e->rank].src = send;
    g.slot[e->rank].ready = e->ev_ready;
    g.slot[e->rank].done = e->ev_done;
    if (!g.barrier(lk)) return fail(e, STOMP_E_COMM, "local exchange group: a rank did not arrive (each rank needs a host thread of its own)");
    std::vector<LocalGroup::Slot> sl = g.slot;
    lk.unlock();
    for (int q = 0; q < g.world; ++q) {
        if (q != e->rank) HIP_TRY(e, hipStreamWaitEvent(e->stream, sl[q].ready, 0));
        if (recv + (size_t)q * n != sl[q].src)   // in place (gather mode: the rank's own rows)
            HIP_TRY(e, hipMemcpyAsync(recv + (size_t)q * n, sl[q].src, n * sizeof(double), hipMemcpyDeviceToDevice,
                                      e->stream));
    }
    HIP_TRY(e, hipEventRecord(e->ev_done, e->stream));
    lk.lock();
    if (!g.barrier(lk)) return fail(e, STOMP_E_COMM, "local exchange group: a rank did not arrive");
    lk.unlock();
    for (int q = 0; q < g.world; ++q)
        if (q != e->rank) HIP_TRY(e, hipStreamWaitEvent(e->stream, sl[q].done, 0));
    return 0;
}

// all-reduce(max) in place of n doubles over the ranks (RCCL, or the in-process group; with one
// rank the identity)
int exchange_max(stomp_engine* e, double* buf, size_t n)
{
#ifdef STOMP_WITH_RCCL
    if (e->comm_aborted) return fail(e, STOMP_E_COMM, "%s", e->comm_msg.c_str());
    if (e->comm) {
        if (!coll_post(e, "all-reduce(max)"))
            NCCL_TRY(e, ncclAllReduce(buf, buf, n, ncclFloat64, ncclMax, e->comm, e->stream));
        coll_mark(e);
        return 0;
    }
#endif
    if (e->local) {
        int rc = local_gather(e, buf, e->d_mm_all, n);
        if (rc) return rc;
        launch_gather_max(e->d_mm_all, e->world, (int)n, buf, e->stream);
    }
    return 0;
}

// all-gather of n doubles per rank into recv [world][n] (send may be recv's own slot: in place)
int exchange_gather(stomp_engine* e, const double* send, double* recv, size_t n)
{
#ifdef STOMP_WITH_RCCL
    if (e->comm_aborted) return fail(e, STOMP_E_COMM, "%s", e->comm_msg.c_str());
    if (e->comm) {
        if (!coll_post(e, "all-gather")) NCCL_TRY(e, ncclAllGather(send, recv, n, ncclFloat64, e->comm, e->stream));
        coll_mark(e);
        return 0;
    }
#endif
    if (e->local) return local_gather(e, send, recv, n);
    if (recv != send) HIP_TRY(e, hipMemcpyAsync(recv, send, sizeof(double) * n, hipMemcpyDeviceToDevice, e->stream));
    return 0;
}

// gather mode: every rank's state-cost rows into every rank's [K][N] state buffer (in place;
// with one rank, the STOMP_DEBUG_GATHER_RANKS timing hook, nothing moves)
int exchange_state(stomp_engine* e)
{
    if (e->world == 1) return 0;
    const size_t n = (size_t)e->K_loc * e->N;
    return exchange_gather(e, e->d_state + (size_t)e->row0 * e->N, e->d_state, n);
}

// generateRollouts' sampling arguments of iteration it (policy_improvement_loop.cpp:155-160:
// sigma_d * decay_d^(it - 1))
NoiseArgs noise_args(const stomp_engine* e, int it)
{
    NoiseArgs na{};
    // gather mode: the noise rows of all K rollouts (global ids from 0)
    na.J = e->J; na.N = e->N; na.Nall = e->Nall; na.K_loc = e->rows; na.first_global = e->first - e->row0;
    na.iteration = it; na.seed = e->seed;
    for (int d = 0; d < e->J; ++d) na.sigma.v[d] = e->sig_std[d] * std::pow(e->sig_dec[d], it - 1);
    na.theta = e->d_theta; na.LT = e->d_LT; na.MT = e->d_MT; na.start = e->d_start; na.goal = e->d_goal;
    std::memcpy(na.dcoef, e->su.dcoef, sizeof na.dcoef);
    const double w = 0.5 * e->w_smooth;   // policy_improvement.cpp:487
    for (int r = 0; r < 3; ++r) na.wr[r] = w * e->smooth[r];
    na.params = e->d_params; na.noise = e->d_noise; na.control = e->d_control; na.zero_noise = 0; na.row_begin = 0;
    na.stop = e->d_stop;
    na.pre_eps = e->d_pre_eps[it & 1]; na.pre_meps = e->d_pre_meps[it & 1];
    na.rows_in_pre = 0; na.theta_gen = e->d_theta_gen;
    return na;
}

// k_pregen's arguments for iteration it: no stop flag, so the rows stay valid for pre_it
// whatever the optimize loop decides
NoiseArgs pregen_args(const stomp_engine* e, int it)
{
    NoiseArgs na = noise_args(e, it);
    na.stop = nullptr;
    return na;
}

// generateRollouts bookkeeping (policy_improvement.cpp:167-225): the first call generates all K;
// later ones rank the K previous rollouts and the extra (noiseless) one, keep the best K_r in rows
// K_gen.. with their noise re-based on the current theta, and generate the rest.  With the rows
// sharded over ranks the ranking runs on all-gathered totals and the chosen rows travel in slots
// (k_misc.hip), so every rank ends with exactly its rows of the single-device result.
void swap_row_sets(stomp_engine* e)
{
    std::swap(e->d_params, e->d_params_b);
    std::swap(e->d_noise, e->d_noise_b);
    std::swap(e->d_control, e->d_control_b);
    std::swap(e->d_state, e->d_state_b);
    e->row_set ^= 1;
}

// generateRollouts' bookkeeping: K_gen, and whether the reuse step runs this iteration; when it
// does the row sets swap, so the previous rows are the reuse source (d_*_b) and this iteration's
// rows are written into the other set
bool plan_generate(stomp_engine* e)
{
    e->K_gen = e->K - e->Kr;
    if (!e->reused_next) {
        e->K_gen = e->K;
        if (e->Kr > 0) e->reused_next = true;
        return false;
    }
    swap_row_sets(e);
    return true;
}

// the reuse step: rank the previous rows and the extra (noiseless) rollout, copy the best K_r
// into rows K_gen.. of this iteration's set (the extra rollout's state costs must be evaluated)
int run_reuse(stomp_engine* e)
{
    Timed tm(e, T_REUSE);
    const int with_extra = e->extra_added ? 1 : 0;
    e->extra_added = false;
    if (e->world == 1) {
        if (int rc = launch_reuse(e->K, e->J, e->N, e->Kr, e->K_gen, with_extra, e->d_params_b, e->d_state_b, e->d_control_b,
                         e->d_params, e->d_noise, e->d_state, e->d_x_params, e->d_x_state, e->d_x_control, e->d_theta,
                         e->d_reuse_costs, e->d_reuse_count, e->d_stop, e->stream))
            return fail(e, STOMP_E_INVALID, rc == -1 ? "reuse: the source and destination rollout rows alias"
                                                     : "reuse: the cost rows of one candidate exceed the LDS");
        return 0;
    }
    const size_t slot = (size_t)e->Kr * ((size_t)e->J * e->N + e->N);
    launch_reuse_totals(e->K_loc, e->J, e->N, e->d_state_b, e->d_control_b, e->d_x_state, e->d_x_control,
                        e->d_tot_loc, e->d_tot_x, e->d_stop, e->stream);
    int rc = exchange_gather(e, e->d_tot_loc, e->d_tot_all, (size_t)e->K_loc);
    if (rc) return rc;
    launch_reuse_select(e->K, e->Kr, with_extra, e->d_tot_all, e->d_tot_x, e->d_sel, e->d_stop, e->stream);
    launch_reuse_pack(e->Kr, e->J, e->N, e->first, e->K_loc, e->d_sel, e->d_params_b, e->d_state_b, e->d_slot,
                      e->d_stop, e->stream);
    if ((rc = exchange_gather(e, e->d_slot, e->d_slot_all, slot))) return rc;
    launch_reuse_unpack(e->Kr, e->K_gen, e->J, e->N, e->first, e->K_loc, e->d_sel, e->d_slot_all, e->d_x_params,
                        e->d_x_state, e->d_theta, e->d_params, e->d_noise, e->d_state, e->d_stop, e->stream);
    return 0;
}

// plan + reuse at once (callers that evaluate no rollouts of their own before the ranking)
int begin_generate(stomp_engine* e)
{
    if (!plan_generate(e)) return 0;
    flush_noiseless(e);
    return run_reuse(e);
}

// One runSingleIteration (policy_improvement_loop.cpp:143-202) enqueued on the engine stream.
// pipelined: the noiseless rollout of the updated theta is not launched here but evaluated by
// the next iteration's rollout-cost launch (extra workgroup) or by flush_noiseless().
int enqueue_iteration(stomp_engine* e, int it, bool pipelined)
{
    if (e->comm_aborted) return fail(e, STOMP_E_COMM, "%s", e->comm_msg.c_str());
    e->cur_it = it;
    const int member = it - 1;
    const bool fused = e->J <= 16;   // rollout_project: at most four 4-joint column groups
    // With fused noise the reuse step runs after the rollout launch: the generated rows go to
    // the other row set, and the launch also evaluates the pending noiseless rollout that the
    // ranking needs (so K_r > 0 iterations pipeline like K_r = 0 ones).  Otherwise k_noise
    // makes every row before the launch and the reuse step has to come first.
    if (e->Kr > 0 && !fused) pipelined = false;
    const bool reuse = plan_generate(e);
    const bool reuse_late = reuse && fused;
    if (reuse && !reuse_late) {
        flush_noiseless(e);
        if (int rc = run_reuse(e)) return rc;
    }
    NoiseArgs na = noise_args(e, it);
    na.K_gen_global = e->K_gen;
    // generated rows [0, g1 - g0) of this shard: their noise is made by the rollout kernel
    // itself (fused), k_noise only projects and prices the reused rows after them
    const int g0 = e->first, g1 = std::min(e->first + e->K_loc, e->K_gen);
    const int num_gen = std::max(g1 - g0, 0);
    if (fused) na.row_begin = e->gather ? e->rows : num_gen;
    // the generated rows' eps and M eps come from the pregen buffers (every local row, or with
    // reuse on one device the rows before the reused ones)
    const bool pre = fused && e->pre_on && (num_gen == e->K_loc || (e->Kr > 0 && num_gen > 0));
    if (e->gather && !pre) return fail(e, STOMP_E_INVALID, "gather mode needs the pregen rows");
    // outside the optimize loop and without reuse the rows stay in the pregen buffer: the weights
    // read eps there and nothing else needs the noise / params rows on the device (the reuse step
    // ranks and copies the previous rows, so with K_r > 0 they are written).  The optimize loop
    // keeps the copies: after its stop the pregen blocks of the iterations enqueued past it still
    // overwrite the buffers.
    const bool rows_pre = pre && !e->tracking && e->Kr == 0;
    na.rows_in_pre = rows_pre ? 1 : 0;
    if (!rows_pre) e->rows_in_pre = false;
    if (pre) {
        if (e->pre_it != it) {   // not made ahead by the previous iteration's launches
            Timed tm(e, T_PREGEN);
            launch_pregen(pregen_args(e, it), e->rows, e->stream);
        }
        e->pre_it = -1;
    }
    if (na.row_begin < na.K_loc && !reuse_late) {
        Timed tm(e, T_NOISE);
        launch_noise(na, e->stream);
    }
    // the candidates priced by the rollout launch (launch_reuse_pick) when its blocks still fit
    // the CUs beside the rollouts, pregen and totals blocks (more pricing blocks than idle CUs
    // would lengthen the launch)
    const int spec_nro = num_gen + (e->pending_member >= 0 ? 1 : 0);
    const int spec_extra = (pre ? e->rows : 0) + e->K + (e->K + 1);
    const bool spec = reuse_late && e->spec_on && e->world == 1 && launch_reuse_pick_ok(na, e->K, e->Kr) &&
                      spec_nro + spec_extra <= e->model.cus &&
                      rollout_split_pieces(e->model, spec_nro, spec_extra, true) > 0;
    // Task::execute for the generated rollouts of this shard (+ the pending noiseless rollout)
    {
        CostArgs ca{};
        ca.stop = e->d_stop;
        ca.fused_noise = pre ? 2 : (fused ? 1 : 0);
        ca.nz = na;
        ca.params = e->d_params; ca.stride = (long long)e->J * e->N; ca.num_noisy = num_gen;
        ca.member = member; ca.state_out = e->d_state;
        if (pre) {
            ca.pre_rows = e->rows;
            ca.pre_next = pregen_args(e, it + 1);
            ca.ctl_by_pre = 1;
            ca.ctl_rows = e->Kr > 0 ? num_gen : e->rows;   // the reused rows are priced by k_noise
            ca.row0 = e->row0;
            ca.state_out = e->d_state + (size_t)e->row0 * e->N;
            e->pre_it = it + 1;
        }
        if (reuse_late && e->world == 1 && launch_reuse_rows_ok(na, e->K, e->Kr)) {
            // the reuse candidates' totals (the previous rows, complete) made beside the rollouts
            ca.tot_rows = e->K;
            ca.tot_state = e->d_state_b; ca.tot_control = e->d_control_b; ca.tot_out = e->d_reuse_costs;
            if (spec) {
                // and every candidate re-based on theta and priced, so that the reuse step only
                // ranks and copies
                ca.spec_rows = e->K + 1;
                ca.spec_src = e->d_params_b;
                ca.spec_params = e->d_spec_params; ca.spec_noise = e->d_spec_noise; ca.spec_ctl = e->d_spec_ctl;
            }
        }
        if (e->terms_on) ca.traj_out = e->d_terms_traj;
        if (e->pending_member >= 0) {
            ca.x_params = e->d_theta; ca.x_member = e->pending_member;
            ca.x_state = e->d_x_state; ca.x_traj = e->d_last_traj;
            // the pipelined noiseless rollout's costs.sum() and collision flag are read only by
            // the optimize loop's bookkeeping (k_track); stomp_engine_iterate and the flush
            // evaluate their own, so without tracking the launch skips them
            if (e->tracking) { ca.x_cf = e->d_cf; ca.x_total = e->d_total; }
            if (e->Kr > 0) { ca.x_ctl = e->d_x_control; ca.x_prm = e->d_x_params; ca.x_nse = e->d_x_noise; }
            e->pending_member = -1;
        }
        {
            Timed tm(e, T_COST);
            launch_rollouts(e, ca);
        }
        if (rows_pre) {
            e->rows_in_pre = true;
            e->rows_eps = na.pre_eps;
        }
        launch_terms_for(e, ca);
        // before this iteration's weights / update: a break decided on the previous
        // iteration's noiseless rollout leaves theta where the reference leaves it
        track_noiseless(e, ca);
    }
    if (e->gather)
        if (int rc = exchange_state(e)) return rc;
    // the reuse step folded into the one-wave-per-column weights (launch_weights_pick)
    ReuseArgs pick_ra{};
    bool pick_in_weights = false;
    if (reuse_late) {
        // the previous rows and the extra rollout (evaluated just now) ranked; the reused rows'
        // projection and control costs after them.  On one device the candidates' totals are
        // made by k_reuse and the reused rows' kernel ranks, copies and prices each row itself
        if (e->world == 1 && launch_reuse_rows_ok(na, e->K, e->Kr)) {
            ReuseArgs ra{};
            ra.K = e->K; ra.Kr = e->Kr; ra.K_gen = e->K_gen; ra.with_extra = e->extra_added ? 1 : 0;
            e->extra_added = false;
            ra.costs = e->d_reuse_costs;
            ra.src_params = e->d_params_b; ra.src_state = e->d_state_b;
            ra.x_params = e->d_x_params; ra.x_state = e->d_x_state; ra.x_control = e->d_x_control;
            ra.state = e->d_state;
            Timed tm(e, T_NOISE);
            if (spec) {
                ra.spec_params = e->d_spec_params; ra.spec_noise = e->d_spec_noise; ra.spec_ctl = e->d_spec_ctl;
                // (launch_weights_pick_ok decides at the weights launch; otherwise k_reuse_pick runs there)
                if (e->pick_fuse && !e->split_modes && !e->use_cum) {
                    pick_ra = ra;
                    pick_in_weights = true;
                } else {
                    launch_reuse_pick(na, ra, e->stream);
                }
            } else {
                launch_reuse_rows(na, ra, e->stream);
            }
        } else {
            if (int rc = run_reuse(e)) return rc;
            if (na.row_begin < na.K_loc) {
                Timed tm(e, T_NOISE);
                launch_noise(na, e->stream);
            }
        }
    }
    WeightArgs wa{};
    wa.stop = e->d_stop;
    wa.J = e->J; wa.N = e->N; wa.K_loc = e->rows; wa.use_cumulative = e->use_cum;
    wa.state = e->d_state; wa.control = e->d_control; wa.noise = rows_pre ? na.pre_eps : e->d_noise;
    wa.cum = e->use_cum ? e->d_cum : nullptr; wa.prob = e->d_prob; wa.u = e->d_u;
    wa.tc = weights_tile(e->rows);
    wa.nb_total = e->K / kSumBlock;
    wa.mm = e->d_mm; wa.psum_part = e->d_psum_part; wa.psum_all = e->d_psum_all; wa.u_part = e->d_u_part;
    {
        Timed tm(e, T_WEIGHTS);
        if (e->use_cum) launch_cumulative(wa, e->d_cum, e->stream);
        if (!e->split_modes) {
            wa.mode = W_FUSED;
            if (pick_in_weights && launch_weights_pick_ok(wa, pick_ra)) {
                launch_weights_pick(wa, pick_ra, na.params, na.noise, na.control, e->stream);
            } else {
                if (pick_in_weights) launch_reuse_pick(na, pick_ra, e->stream);
                launch_weights(wa, e->stream);
            }
        } else {
            // the sharded decomposition; with one rank (debug hook) the all-reduce is the
            // identity and the all-gathers are device copies
            const size_t JN = (size_t)e->J * e->N;
            const size_t nb_loc = (size_t)e->K_loc / kSumBlock;
            wa.mode = W_MINMAX;
            launch_weights(wa, e->stream);
            int rc = exchange_max(e, e->d_mm, 2 * JN);
            if (rc) return rc;
            wa.mode = W_PSUM;
            launch_weights(wa, e->stream);
            if ((rc = exchange_gather(e, e->d_psum_part, e->d_psum_all, nb_loc * JN))) return rc;
            wa.mode = W_USUM;
            launch_weights(wa, e->stream);
            if ((rc = exchange_gather(e, e->d_u_part, e->d_u_all, nb_loc * JN))) return rc;
        }
    }
    {
        Timed tm(e, T_UPDATE);
        launch_update(e->J, e->N, e->d_MT, e->d_u, e->split_modes ? e->d_u_all : nullptr, e->K / kSumBlock,
                      e->d_theta, e->d_stop, e->stream);
    }
    if (pipelined) {
        e->pending_member = member;
    } else {
        launch_noiseless(e, member);
    }
    if (e->Kr > 0) {
        // addExtraRollouts (policy_improvement.cpp:443-462): params = theta, noise = 0 — the
        // noiseless rollout of theta, whose workgroup (this iteration's noiseless launch, or the
        // next rollout launch's extra workgroup) also writes the extra rollout's params / noise /
        // control rows (x_ctl) before the next reuse ranking reads them
        e->extra_added = true;
    }
    hipError_t st = hipGetLastError();
    if (st != hipSuccess)
        return fail(e, STOMP_E_DEVICE, "kernel launch failed: %s%s%s", hipGetErrorString(st),
                    lds_opt_in_error()[0] ? "; " : "", lds_opt_in_error());
    return 0;
}

// The K-sharded decomposition from measurements, at the end of stomp_engine_create when
// both are possible and none was requested.  Every rank times, on its own device and stream:
//   T_g  one iteration's rollout launch and fused weights in gather mode (its K_loc rollouts, all K
//        pregen / pricing rows, the weights over all K), no exchange;
//   T_p  the same in partials mode (its K_loc rows, the MINMAX / PSUM / USUM weights phases);
//   L_ar, L_ag, L_agp  the collectives each posts: the all-reduce(max) of 2 J N doubles, the
//        all-gather of the K_loc N state rows, the all-gather of the block partials;
// the maxima over the ranks are taken (one all-reduce), so every rank decides alike:
//   gather  <=>  T_g + L_ag <= T_p + L_ar + 2 L_agp          (stomp_shard_decide)
// The calibration launches leave no state the first iteration reads: theta is untouched, the pregen
// rows are remade (pre_it stays -1), and every row buffer is rewritten by the iterations.
// STOMP_DEBUG_SHARD_LATENCY_US=x adds x us to every measured collective (tests: both selections).
// partials chosen after a calibration that ran in gather mode's layout: the row buffers drop from
// K rows to the rank's K_loc (about world_size times less memory); nothing in them is read again
// (every row is rewritten by the iterations, the pregen rows are remade)
int shrink_rows(stomp_engine* e)
{
    const size_t JN = (size_t)e->J * e->N, KJN = (size_t)e->rows * JN;
    auto re = [&](double*& p, size_t n) -> int {
        if (!p) return 0;
        HIP_TRY(e, hipStreamSynchronize(e->stream));   // the calibration launches used it
        auto it = std::find(e->allocs.begin(), e->allocs.end(), (void*)p);
        if (it != e->allocs.end()) {
            hipFree(*it);
            e->allocs.erase(it);
        }
        p = nullptr;
        return dev_alloc(e, &p, n);
    };
    int rc = 0;
    for (double** p : {&e->d_params, &e->d_noise, &e->d_control, &e->d_prob, &e->d_cum, &e->d_pre_eps[0],
                       &e->d_pre_eps[1], &e->d_pre_meps[0], &e->d_pre_meps[1]})
        if ((rc = re(*p, KJN))) return rc;
    return re(e->d_state, (size_t)e->rows * e->N);
}

int calibrate_shard_mode(stomp_engine* e)
{
    const int J = e->J, N = e->N;
    const size_t JN = (size_t)J * N;
    hipEvent_t ev0 = get_event(e), ev1 = get_event(e);
    auto elapsed_us = [&]() -> double {
        float ms = 0.0f;
        if (hipEventSynchronize(ev1) != hipSuccess || hipEventElapsedTime(&ms, ev0, ev1) != hipSuccess) return -1.0;
        return 1000.0 * ms;
    };
    auto median = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    auto set_mode = [&](bool gather) {
        e->gather = gather;
        e->rows = gather ? e->K : e->K_loc;
        e->row0 = gather ? e->first : 0;
        e->split_modes = !gather;
    };
    // one iteration's compute in the current mode (enqueue_iteration's launches for K_r = 0 with
    // pregen rows, the exchanges left out)
    auto compute = [&]() -> double {
        NoiseArgs na = noise_args(e, 1);
        na.K_gen_global = e->K;
        na.row_begin = e->rows;
        na.rows_in_pre = 1;
        CostArgs ca{};
        ca.stop = e->d_stop;
        ca.fused_noise = 2;
        ca.nz = na;
        ca.params = e->d_params; ca.stride = (long long)JN; ca.num_noisy = e->K_loc;
        ca.member = 0;
        ca.pre_rows = e->rows;
        ca.pre_next = pregen_args(e, 2);
        ca.ctl_by_pre = 1;
        ca.ctl_rows = e->rows;
        ca.row0 = e->row0;
        ca.state_out = e->d_state + (size_t)e->row0 * N;
        WeightArgs wa{};
        wa.stop = e->d_stop;
        wa.J = J; wa.N = N; wa.K_loc = e->rows; wa.use_cumulative = e->use_cum;
        wa.state = e->d_state; wa.control = e->d_control; wa.noise = na.pre_eps;
        wa.cum = e->use_cum ? e->d_cum : nullptr; wa.prob = e->d_prob; wa.u = e->d_u;
        wa.tc = weights_tile(e->rows);
        wa.nb_total = e->K / kSumBlock;
        wa.mm = e->d_mm; wa.psum_part = e->d_psum_part; wa.psum_all = e->d_psum_all; wa.u_part = e->d_u_part;
        hipEventRecord(ev0, e->stream);
        launch_cost(e->model, ca, e->stream);
        if (e->use_cum) launch_cumulative(wa, e->d_cum, e->stream);
        if (!e->split_modes) {
            wa.mode = W_FUSED;
            launch_weights(wa, e->stream);
        } else {
            for (int mode : {W_MINMAX, W_PSUM, W_USUM}) {
                wa.mode = mode;
                launch_weights(wa, e->stream);
            }
        }
        hipEventRecord(ev1, e->stream);
        return elapsed_us();
    };
    auto timed = [&](auto&& f, int reps) -> double {
        f();   // warm
        std::vector<double> v;
        for (int r = 0; r < reps; ++r) v.push_back(f());
        return median(v);
    };
    double m[5];
    set_mode(true);
    m[0] = timed(compute, 3);
    set_mode(false);
    m[1] = timed(compute, 3);
    int rc = 0;
    auto coll = [&](auto&& post) -> double {
        hipEventRecord(ev0, e->stream);
        if (int r = post()) rc = r;
        hipEventRecord(ev1, e->stream);
        return elapsed_us();
    };
    m[2] = timed([&]() { return coll([&]() { return exchange_max(e, e->d_mm, 2 * JN); }); }, 8);
    m[3] = timed([&]() {
        return coll([&]() { return exchange_gather(e, e->d_state + (size_t)e->first * N, e->d_state,
                                                   (size_t)e->K_loc * N); });
    }, 8);
    m[4] = timed([&]() {
        return coll([&]() { return exchange_gather(e, e->d_psum_part, e->d_psum_all,
                                                   (size_t)(e->K_loc / kSumBlock) * JN); });
    }, 8);
    e->pool.push_back(ev0);
    e->pool.push_back(ev1);
    if (rc) return rc;
    for (double x : m)
        if (!(x >= 0.0)) return fail(e, STOMP_E_DEVICE, "decomposition calibration: event timing failed");
    if (const char* lat = std::getenv("STOMP_DEBUG_SHARD_LATENCY_US"))
        for (int k = 2; k < 5; ++k) m[k] += std::atof(lat);
    // every rank decides on the maxima over the ranks
    HIP_TRY(e, hipMemcpyAsync(e->d_mm, m, sizeof m, hipMemcpyHostToDevice, e->stream));
    if ((rc = exchange_max(e, e->d_mm, 5))) return rc;
    HIP_TRY(e, hipMemcpyAsync(m, e->d_mm, sizeof m, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    int32_t mode = 0;
    stomp_shard_decide(m, &mode);
    set_mode(mode == STOMP_SHARD_GATHER);
    if (e->gather) HIP_TRY(e, hipMemsetAsync(e->d_state, 0, sizeof(double) * e->rows * N, e->stream));
    else if ((rc = shrink_rows(e))) return rc;
    e->shard_info[0] = mode;
    for (int k = 0; k < 5; ++k) e->shard_info[1 + k] = m[k];
    return 0;
}

}  // namespace

extern "C" {

const char* stomp_last_error(void) { return g_last_error.c_str(); }

const char* stomp_engine_last_error(const stomp_engine* e) { return e ? e->err.c_str() : g_last_error.c_str(); }
// stomp_engine_source_hash: in the object _build.py generates at link time (build/source_hash.cpp)

// The hinge potential's zero case and the collision test of StompCollisionSpace::
// getCollisionPointPotentialGradient (stomp_collision_space.h:193-228) as thresholds on a voxel's
// squared cell distance d2, whose distance is sqrt((double)d2) * res (the field's sqrt_table_):
//   potential == 0  <=>  d2 >= zero_lim      in collision  <=>  d2 < col_lim
// Every d2 a 16-bit voxel can hold is priced with the reference's expressions (one rounding per
// operation, as the kernel's), and each predicate is checked to switch exactly once, so the
// kernel's integer compares give the same answers as the potential itself.
static bool sphere_thresholds(double radius, double clearance, double res, int* zero_lim, int* col_lim)
{
    if (!(radius >= 0.0 && clearance > 0.0 && std::isfinite(radius) && std::isfinite(clearance))) return false;
    int zl = 65536, cl = 65536;
    bool zseen = false, cseen = false;
    for (int d2 = 0; d2 <= 65535; ++d2) {
        const double dist = std::sqrt((double)d2) * res;
        const double dd = dist - radius;
        const bool zero = dd >= clearance;
        const bool col = dist <= radius;
        if (zero && !zseen) { zl = d2; zseen = true; }
        if (!zero && zseen) return false;
        if (!col && !cseen) { cl = d2; cseen = true; }
        if (col && cseen) return false;
    }
    *zero_lim = zl;
    *col_lim = cl;
    return true;
}

int stomp_engine_create(const stomp_engine_desc* d, stomp_engine** out)
{
    if (!d || !out) return fail(nullptr, STOMP_E_INVALID, "null argument");
    *out = nullptr;
    if (d->abi_version != STOMP_ENGINE_ABI_VERSION)
        return fail(nullptr, STOMP_E_INVALID, "abi_version %d != %d", d->abi_version, STOMP_ENGINE_ABI_VERSION);
    if (d->num_joints <= 0 || d->num_joints > kMaxJoints)
        return fail(nullptr, STOMP_E_INVALID, "num_joints must be in [1, %d]", kMaxJoints);
    if (d->num_time_steps <= 0 || d->num_time_steps > 256)
        return fail(nullptr, STOMP_E_INVALID, "num_time_steps must be in [1, 256]");
    if (d->num_rollouts <= 0) return fail(nullptr, STOMP_E_INVALID, "num_rollouts must be positive");
    if (d->num_reused_rollouts < 0 || d->num_reused_rollouts >= d->num_rollouts)
        return fail(nullptr, STOMP_E_INVALID, "Number of reused rollouts must be strictly less than number of rollouts.");
    if (d->num_orientation_constraints < 0 || (d->num_orientation_constraints > 0 && !d->orientation_constraints))
        return fail(nullptr, STOMP_E_INVALID, "invalid orientation constraints");
    for (int c = 0; c < d->num_orientation_constraints; ++c)
        if (d->orientation_constraints[c].segment < 0 || d->orientation_constraints[c].segment >= d->num_segments)
            return fail(nullptr, STOMP_E_INVALID, "orientation constraint %d: bad segment", c);
    if (d->num_segments <= 0 || !d->segments || (d->num_spheres > 0 && !d->spheres) || !d->joints || !d->noise_stddev ||
        !d->noise_decay || !d->start || !d->goal || !d->grid.data)
        return fail(nullptr, STOMP_E_INVALID, "missing table pointer");
    if (d->grid.nx < 3 || d->grid.ny < 3 || d->grid.nz < 3 || !(d->grid.resolution > 0))
        return fail(nullptr, STOMP_E_INVALID, "invalid grid");
    if ((uint64_t)d->grid.nx * (uint64_t)d->grid.ny * (uint64_t)d->grid.nz > 0xFFFFFFFFull)
        return fail(nullptr, STOMP_E_UNSUPPORTED, "distance field larger than 2^32 cells");
    for (int s = 0; s < d->num_segments; ++s)
        if (d->segments[s].parent >= s || d->segments[s].q_index >= d->num_joints)
            return fail(nullptr, STOMP_E_INVALID, "segment %d: parent must precede it (DFS order), q_index < J", s);
    for (int j = 0; j < d->num_spheres; ++j) {
        if (d->spheres[j].segment < 0 || d->spheres[j].segment >= d->num_segments)
            return fail(nullptr, STOMP_E_INVALID, "sphere %d: bad segment", j);
        int zl, cl;
        if (!sphere_thresholds(d->spheres[j].radius, d->spheres[j].clearance, d->grid.resolution, &zl, &cl))
            return fail(nullptr, STOMP_E_INVALID, "sphere %d: radius / clearance not finite and positive", j);
    }
    if (d->torque_cost_weight > 1e-9) {
        std::vector<int> path;
        if (const char* why = torque_chain(d, path)) return fail(nullptr, STOMP_E_UNSUPPORTED, "%s", why);
    }
    const int world = d->world_size > 0 ? d->world_size : 1;
    if (world > 1) {
        if (!d->comm_id) return fail(nullptr, STOMP_E_INVALID, "world_size > 1 needs a comm_id");
        if (d->rank < 0 || d->rank >= world)
            return fail(nullptr, STOMP_E_INVALID, "rank %d outside [0, world_size %d)", d->rank, world);
        if (d->num_rollouts % (world * kSumBlock) != 0)
            return fail(nullptr, STOMP_E_INVALID, "num_rollouts must be a multiple of 64 * world_size");
#ifndef STOMP_WITH_RCCL
        if (std::memcmp(d->comm_id, kLocalMagic, sizeof kLocalMagic) != 0)
            return fail(nullptr, STOMP_E_UNSUPPORTED, "built without RCCL (use stomp_comm_local_id)");
#endif
    }

    DeviceGuard dg(d->device);
    stomp_engine* e = new stomp_engine();
    e->device = d->device;
    int rc;
    if (hipSetDevice(d->device) != hipSuccess) {
        rc = fail(nullptr, STOMP_E_DEVICE, "hipSetDevice(%d) failed", d->device);
        delete e;
        return rc;
    }
    if (d->stream) {
        e->stream = (hipStream_t)d->stream;
    } else {
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
        e->own_stream = true;
    }
    e->J = d->num_joints; e->N = d->num_time_steps; e->Nall = e->N + 2 * kPad;
    e->K = d->num_rollouts; e->Kr = d->num_reused_rollouts;
    e->world = world; e->rank = world > 1 ? d->rank : 0;
    e->K_loc = e->K / world; e->first = e->rank * e->K_loc;
    if (e->K_loc > kSumBlock * 64) {
        rc = fail(e, STOMP_E_INVALID, "at most %d rollouts per device", kSumBlock * 64);
        g_last_error = e->err; release(e); delete e; return rc;
    }
    // rows made ahead by the previous rollout launch (the fused noise phase takes J <= 16); with
    // reused rollouts on one device too (the generated rows' noise does not depend on the reuse)
    e->pre_on = (e->Kr == 0 || world == 1) && e->J <= 16;
    {
        // the K-sharded decomposition.  gather: one all-gather of the state-cost rows
        // per iteration, every rank making and pricing all K noise rows; partials: three exchanges
        // of 64-rollout block partials (MINMAX / PSUM / USUM weights phases).  Default: gather while
        // the state rows of all K rollouts are at most 1 MiB (cfg2: 396 KB; cfg3's 6.5 MB stay
        // partials), STOMP_SHARD_MODE=gather|partials to choose.  Gather needs the pregen rows in
        // the rollout launch and no reuse.
        const bool can = e->pre_on && e->Kr == 0 && e->K <= kSumBlock * 64;
        const char* sm = std::getenv("STOMP_SHARD_MODE");
        if (world > 1 && sm && std::strcmp(sm, "gather") == 0 && !can) {
            // not honoured silently: a rank falling back to partials would post other collectives
            rc = fail(e, STOMP_E_UNSUPPORTED, "STOMP_SHARD_MODE=gather needs the pregen rows in the rollout launch "
                                              "and no reused rollouts (K_r = %d, J = %d)", e->Kr, e->J);
            g_last_error = e->err; release(e); delete e; return rc;
        }
        // STOMP_DEBUG_GATHER_RANKS=W: a one-device engine times rank 0 of W gather-mode ranks (its
        // K / W rollouts, all K rows made and weighted; nothing exchanged, so results are not the
        // sharded ones: a timing hook)
        const char* sim = std::getenv("STOMP_DEBUG_GATHER_RANKS");
        const int W = (world == 1 && sim) ? std::atoi(sim) : 0;
        if (W > 1 && can && e->K % (W * kSumBlock) == 0) {
            e->gather = true;
            e->K_loc = e->K / W;
        } else if (world > 1 && can) {
            // requested (STOMP_SHARD_MODE), or, where nothing is measured (an in-process group without
            // STOMP_DEBUG_CALIBRATE_LOCAL), gather while the K N state rows fit 1 MiB
            e->gather = sm ? std::strcmp(sm, "gather") == 0 : (size_t)e->K * e->N * sizeof(double) <= (1u << 20);
        }
        // over RCCL, with both decompositions possible and none requested, the choice is measured at
        // the end of creation (calibrate_shard_mode); until then gather mode's layout, which holds every
        // row (shrink_rows gives the buffers back when partials wins)
        // (the in-process exchange group calibrates only on request, STOMP_DEBUG_CALIBRATE_LOCAL=1:
        // its ranks must then be created on host threads of their own, as the measurement exchanges)
        const char* cl = std::getenv("STOMP_DEBUG_CALIBRATE_LOCAL");
        const bool local = world > 1 && std::memcmp(d->comm_id, kLocalMagic, sizeof kLocalMagic) == 0;
        e->calibrate = world > 1 && can && !sm && (!local || (cl && cl[0] == '1'));
        if (e->calibrate) e->gather = true;
        e->rows = e->gather ? e->K : e->K_loc;
        e->row0 = (e->gather && world > 1) ? e->first : 0;
        // STOMP_DEBUG_SHARDED_MODES=1: a one-device engine runs the multi-GPU weights phases
        // (test hook for the MINMAX / PSUM / USUM kernels; needs whole 64-rollout blocks, no reuse)
        const char* dbg = std::getenv("STOMP_DEBUG_SHARDED_MODES");
        e->split_modes = (world > 1 && !e->gather) ||
                         (world == 1 && !e->gather && dbg && dbg[0] == '1' && d->num_rollouts % kSumBlock == 0 &&
                          d->num_reused_rollouts == 0);
    }
    e->S = d->num_spheres; e->nseg = d->num_segments; e->seed = d->seed;
    e->disc = d->discretization; e->w_smooth = d->smoothness_cost_weight; e->w_obs = d->obstacle_cost_weight;
    e->w_con = d->constraint_cost_weight; e->w_tq = d->torque_cost_weight;
    for (int r = 0; r < 3; ++r) e->smooth[r] = d->smoothness_costs[r];
    e->use_cum = d->use_cumulative_costs; e->max_it = d->max_iterations;
    e->max_it_cf = d->max_iterations_after_collision_free;
    e->sig_std.assign(d->noise_stddev, d->noise_stddev + e->J);
    e->sig_dec.assign(d->noise_decay, d->noise_decay + e->J);
    e->start.assign(d->start, d->start + e->J);
    e->goal.assign(d->goal, d->goal + e->J);

#define CREATE_TRY(x)                           \
    do {                                        \
        if ((rc = (x)) != 0) {                  \
            g_last_error = e->err;              \
            release(e);                         \
            delete e;                           \
            return rc;                          \
        }                                       \
    } while (0)

    e->sphere_slot.assign(std::max(e->S, 1), 0);
    CREATE_TRY(plan_fk(e, d, e->ops));
    SetupInput si;
    si.J = e->J; si.N = e->N; si.discretization = e->disc;
    for (int r = 0; r < 3; ++r) si.smoothness_costs[r] = e->smooth[r];
    si.ridge_factor = d->ridge_factor;
    for (int j = 0; j < e->J; ++j) si.joint_cost.push_back(d->joints[j].joint_cost);
    si.start = e->start; si.goal = e->goal;
    std::string msg = compute_setup(si, e->su);
    if (!msg.empty()) CREATE_TRY(fail(e, STOMP_E_INVALID, "%s", msg.c_str()));

    const int J = e->J, N = e->N;
    // LT / MT carry kMatPadRows zero rows past N for the noise kernel's unclamped look-ahead loads
    std::vector<double> LT((size_t)(N + kMatPadRows) * N, 0.0), MT((size_t)(N + kMatPadRows) * N, 0.0),
        QT((size_t)J * N * N);
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < N; ++k) {
            LT[(size_t)k * N + i] = e->su.L[(size_t)i * N + k];
            MT[(size_t)k * N + i] = e->su.M[(size_t)i * N + k];
        }
    for (int j = 0; j < J; ++j)
        for (int i = 0; i < N; ++i)
            for (int k = 0; k < N; ++k)
                QT[((size_t)j * N + k) * N + i] = e->su.Qinv[((size_t)j * N + i) * N + k];
    std::vector<DevSegment> segs(e->nseg);
    for (int s = 0; s < e->nseg; ++s) {
        const stomp_segment& g = d->segments[s];
        segs[s].parent = g.parent; segs[s].q_index = g.q_index;
        std::memcpy(segs[s].rot, g.rot, sizeof g.rot);
        // as the oracle's so_rot_identity: products with it are skipped on both sides
        segs[s].rot_identity = g.rot[0] == 1.0 && g.rot[1] == 0.0 && g.rot[2] == 0.0 && g.rot[3] == 0.0 &&
                               g.rot[4] == 1.0 && g.rot[5] == 0.0 && g.rot[6] == 0.0 && g.rot[7] == 0.0 &&
                               g.rot[8] == 1.0;
        segs[s].pad_ = 0;
        std::memcpy(segs[s].trans, g.trans, sizeof g.trans);
        std::memcpy(segs[s].axis, g.axis, sizeof g.axis);
    }
    std::vector<DevSphere> sph(std::max(e->S, 1));
    for (int j = 0; j < e->S; ++j) {
        const stomp_sphere& g = d->spheres[j];
        sph[j].slot = e->sphere_slot[j];
        sph[j].radius = g.radius; sph[j].clearance = g.clearance;
        sph[j].inv_clearance = 1.0 / g.clearance;   // stomp_collision_point.cpp:50
        std::memcpy(sph[j].pos, g.pos, sizeof g.pos);
        sphere_thresholds(g.radius, g.clearance, d->grid.resolution, &sph[j].zero_lim, &sph[j].col_lim);
        sph[j].pad_ = 0;
    }
    std::vector<int> has_lim(J);
    std::vector<double> jmin(J), jmax(J);
    for (int j = 0; j < J; ++j) {
        has_lim[j] = d->joints[j].has_limits;
        jmin[j] = d->joints[j].min;
        jmax[j] = d->joints[j].max;
    }
    // slots are numbered in sphere order, so each slot owns a contiguous sphere range
    std::vector<int> slot_sph(e->nslots + 1, e->S);
    for (int j = e->S - 1; j >= 0; --j) slot_sph[e->sphere_slot[j]] = j;
    CREATE_TRY(upload(e, &e->d_QT, QT.data(), QT.size()));
    CREATE_TRY(upload(e, &e->d_LT, LT.data(), LT.size()));
    CREATE_TRY(upload(e, &e->d_MT, MT.data(), MT.size()));
    CREATE_TRY(upload(e, &e->d_theta, e->su.theta.data(), e->su.theta.size()));
    CREATE_TRY(upload(e, &e->d_start, e->start.data(), e->start.size()));
    CREATE_TRY(upload(e, &e->d_goal, e->goal.data(), e->goal.size()));
    const size_t ncell = (size_t)d->grid.nx * d->grid.ny * d->grid.nz;
    e->grid_n[0] = d->grid.nx; e->grid_n[1] = d->grid.ny; e->grid_n[2] = d->grid.nz;
    if (d->grid.data_on_device) {
        e->d_sdf = (uint16_t*)d->grid.data;
        e->d_sdf_caller = d->grid.data;
    } else {
        CREATE_TRY(upload(e, &e->d_sdf, d->grid.data, ncell));
    }
    const size_t KJN = (size_t)e->rows * J * N;
    CREATE_TRY(dev_alloc(e, &e->d_params, KJN));
    CREATE_TRY(dev_alloc(e, &e->d_noise, KJN));
    CREATE_TRY(dev_alloc(e, &e->d_control, KJN));
    CREATE_TRY(dev_alloc(e, &e->d_prob, KJN));
    CREATE_TRY(dev_alloc(e, &e->d_state, (size_t)e->rows * N));
    if (e->gather && hipMemsetAsync(e->d_state, 0, sizeof(double) * e->rows * N, e->stream) != hipSuccess)
        CREATE_TRY(fail(e, STOMP_E_DEVICE, "memset failed"));
    if (e->Kr > 0) {
        CREATE_TRY(dev_alloc(e, &e->d_params_b, KJN));
        CREATE_TRY(dev_alloc(e, &e->d_noise_b, KJN));
        CREATE_TRY(dev_alloc(e, &e->d_control_b, KJN));
        CREATE_TRY(dev_alloc(e, &e->d_state_b, (size_t)e->K_loc * N));
    }
    if (e->use_cum) CREATE_TRY(dev_alloc(e, &e->d_cum, KJN));
    CREATE_TRY(dev_alloc(e, &e->d_u, (size_t)J * N));
    if (e->split_modes || e->calibrate) {
        const size_t nb_loc = (size_t)e->K_loc / kSumBlock, nb_tot = (size_t)e->K / kSumBlock;
        CREATE_TRY(dev_alloc(e, &e->d_mm, 2 * (size_t)J * N));
        CREATE_TRY(dev_alloc(e, &e->d_psum_part, nb_loc * J * N));
        CREATE_TRY(dev_alloc(e, &e->d_psum_all, nb_tot * J * N));
        CREATE_TRY(dev_alloc(e, &e->d_u_part, nb_loc * J * N));
        CREATE_TRY(dev_alloc(e, &e->d_u_all, nb_tot * J * N));
    }
    if (e->pre_on)
        for (int b = 0; b < 2; ++b) {
            CREATE_TRY(dev_alloc(e, &e->d_pre_eps[b], KJN));
            CREATE_TRY(dev_alloc(e, &e->d_pre_meps[b], KJN));
        }
    if (e->pre_on) CREATE_TRY(dev_alloc(e, &e->d_theta_gen, (size_t)J * N));
    CREATE_TRY(dev_alloc(e, &e->d_x_params, (size_t)J * N));
    CREATE_TRY(dev_alloc(e, &e->d_x_noise, (size_t)J * N));
    CREATE_TRY(dev_alloc(e, &e->d_x_control, (size_t)J * N));
    CREATE_TRY(dev_alloc(e, &e->d_x_state, (size_t)N));
    CREATE_TRY(dev_alloc(e, &e->d_last_traj, (size_t)J * N));
    CREATE_TRY(dev_alloc(e, &e->d_best_traj, (size_t)J * N));
    CREATE_TRY(dev_alloc(e, &e->d_total, 1));
    CREATE_TRY(dev_alloc(e, &e->d_cf, 1));
    CREATE_TRY(dev_alloc(e, &e->d_cs, 1));
    CREATE_TRY(dev_alloc(e, &e->d_track, 1));
    e->d_stop = &e->d_track->stop;
    CREATE_TRY(dev_alloc(e, &e->d_opt_costs, (size_t)std::max(e->max_it, 1)));
    if (hipHostMalloc((void**)&e->h_track, sizeof(DevTrack) * 4) != hipSuccess)
        CREATE_TRY(fail(e, STOMP_E_DEVICE, "hipHostMalloc failed"));
    if (hipMemsetAsync(e->d_track, 0, sizeof(DevTrack), e->stream) != hipSuccess)
        CREATE_TRY(fail(e, STOMP_E_DEVICE, "memset failed"));
    if (hipMemsetAsync(e->d_cs, 1, 1, e->stream) != hipSuccess) CREATE_TRY(fail(e, STOMP_E_DEVICE, "memset failed"));
    CREATE_TRY(dev_alloc(e, &e->d_pad_cf, 1));
    if (e->world == 1 && e->Kr > 0) {   // k_reuse's per-candidate totals and its counter (zeroed)
        CREATE_TRY(dev_alloc(e, &e->d_reuse_costs, (size_t)e->K + 1));
        CREATE_TRY(dev_alloc(e, &e->d_reuse_count, 1));
        const char* no_spec = std::getenv("STOMP_DEBUG_NO_SPEC");
        if (!(no_spec && std::strcmp(no_spec, "1") == 0)) {
            const size_t n = ((size_t)e->K + 1) * J * N;
            CREATE_TRY(dev_alloc(e, &e->d_spec_params, n));
            CREATE_TRY(dev_alloc(e, &e->d_spec_noise, n));
            CREATE_TRY(dev_alloc(e, &e->d_spec_ctl, n));
            e->spec_on = true;
        }
        const char* no_fuse = std::getenv("STOMP_DEBUG_NO_PICK_FUSE");
        e->pick_fuse = !(no_fuse && std::strcmp(no_fuse, "1") == 0);
    }
    if (e->world > 1 && e->Kr > 0) {
        const size_t slot = (size_t)e->Kr * ((size_t)J * N + N);
        CREATE_TRY(dev_alloc(e, &e->d_tot_loc, (size_t)e->K_loc));
        CREATE_TRY(dev_alloc(e, &e->d_tot_all, (size_t)e->K));
        CREATE_TRY(dev_alloc(e, &e->d_tot_x, 1));
        CREATE_TRY(dev_alloc(e, &e->d_sel, (size_t)e->Kr));
        CREATE_TRY(dev_alloc(e, &e->d_slot, slot));
        CREATE_TRY(dev_alloc(e, &e->d_slot_all, slot * e->world));
    }
    if (hipHostMalloc((void**)&e->h_total, sizeof(double)) != hipSuccess ||
        hipHostMalloc((void**)&e->h_cf, 16) != hipSuccess)
        CREATE_TRY(fail(e, STOMP_E_DEVICE, "hipHostMalloc failed"));

    // the torque term's chain (stomp_robot_model.cpp:185-189): segments below torque_root up to
    // torque_tip, whose joints must be the group's joints in order.  Built whenever the inertias
    // describe a valid chain: the term itself runs only with torque_cost_weight > 1e-9, the
    // final torque statistics of optimize() always (stomp_optimizer.cpp:384-398)
    std::vector<int> tq_path;
    const bool tq_chain = torque_chain(d, tq_path) == nullptr;
    if (tq_chain) {
        std::vector<int>& path = tq_path;
        std::vector<ChainSeg> cs(path.size());
        for (size_t i = 0; i < path.size(); ++i) {
            cs[i].seg = segs[path[i]];
            // KDL::RigidBodyInertia(m, c, Ic): h = m c, I = Ic - m (c c^T - (c.c) 1)
            const stomp_inertia& in = d->inertias[path[i]];
            const double* c = in.com;
            const double* v = in.inertia;
            const double Ic[9] = {v[0], v[3], v[4], v[3], v[1], v[5], v[4], v[5], v[2]};
            const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
            cs[i].m = in.mass;
            for (int a = 0; a < 3; ++a) {
                cs[i].h[a] = in.mass * c[a];
                for (int b = 0; b < 3; ++b) cs[i].I[3 * a + b] = Ic[3 * a + b] - in.mass * (c[a] * c[b] - (a == b ? cc : 0.0));
            }
        }
        ChainSeg* d_chain;
        CREATE_TRY(upload(e, &d_chain, cs.data(), cs.size()));
        TermsModel& t = e->terms;
        t.torque = d->torque_cost_weight > 1e-9 ? 1 : 0;
        t.nchain = (int)cs.size();
        t.chain = d_chain;
        for (int k = 0; k < 3; ++k) t.g[k] = d->gravity[k];
        if (t.torque) e->terms_on = true;
        e->torque_stats = true;
    }
    if (d->num_orientation_constraints > 0) {
        std::vector<OcDev> oc(d->num_orientation_constraints);
        for (int c = 0; c < d->num_orientation_constraints; ++c) {
            const stomp_orientation_constraint& in = d->orientation_constraints[c];
            OcDev& o = oc[c];
            std::vector<int> path;
            for (int sgi = in.segment; sgi >= 0; sgi = d->segments[sgi].parent) path.push_back(sgi);
            if ((int)path.size() > kMaxChain)
                CREATE_TRY(fail(e, STOMP_E_UNSUPPORTED, "constraint segment deeper than %d", kMaxChain));
            std::reverse(path.begin(), path.end());
            o.seg = in.segment; o.body_fixed = in.body_fixed ? 1 : 0; o.path_len = (int)path.size();
            for (size_t k = 0; k < path.size(); ++k) o.path[k] = path[k];
            oc_nominal_inverse(in.orientation, o.ninv);
            o.tol[0] = in.absolute_roll_tolerance; o.tol[1] = in.absolute_pitch_tolerance;
            o.tol[2] = in.absolute_yaw_tolerance; o.weight = in.weight;
            o.rw = o.pw = o.yw = 1.0;   // constraint_evaluator.cpp:66-72
            if (o.tol[1] >= M_PI) o.pw = 0.0;
            if (o.tol[0] >= M_PI) o.rw = 0.0;
            if (o.tol[2] >= M_PI) o.yw = 0.0;
        }
        OcDev* d_oc;
        CREATE_TRY(upload(e, &d_oc, oc.data(), oc.size()));
        e->terms.noc = (int)oc.size();
        e->terms.oc = d_oc;
        e->terms_on = true;
    }
    if (e->terms_on || e->torque_stats) {
        TermsModel& t = e->terms;
        t.J = J; t.N = N;
        const double invTime = 1.0 / e->disc, invTime2 = 1.0 / (e->disc * e->disc);   // stomp_trajectory.h:289, 301
        for (int k = 0; k < 7; ++k) {
            t.cv[k] = invTime * kDiffRules[0][k];
            t.ca[k] = invTime2 * kDiffRules[1][k];
        }
        t.start = e->d_start; t.goal = e->d_goal;
        t.w_con = e->w_con; t.w_tq = e->w_tq;
        if (terms_lds_bytes(t) > 160 * 1024) {
            if (e->terms_on)
                CREATE_TRY(fail(e, STOMP_E_UNSUPPORTED, "state-terms kernel needs %zu B of LDS", terms_lds_bytes(t)));
            e->torque_stats = false;
        }
        if (e->terms_on) CREATE_TRY(dev_alloc(e, &e->d_terms_traj, (size_t)e->K_loc * J * N));
        if (e->torque_stats) {
            e->tq_model = t;
            e->tq_model.torque = 1;
            e->tq_model.noc = 0;   // torques only
            CREATE_TRY(dev_alloc(e, &e->d_tq, (size_t)N));
            CREATE_TRY(dev_alloc(e, &e->d_tq_state, (size_t)N));
        }
    }
    CREATE_TRY(dev_alloc(e, &e->d_delta, (size_t)J * N));
    e->pi_weight = e->w_smooth;
    if (hipDeviceGetAttribute(&e->wall_khz, hipDeviceAttributeWallClockRate, d->device) != hipSuccess) e->wall_khz = 0;

    DevModel& m = e->model;
    m.J = J; m.N = N; m.Nall = e->Nall; m.S = e->S; m.nops = (int)e->ops.size(); m.nseg = e->nseg;
    m.nslots = e->nslots;
    m.sph_chunk = 1;   // the a-value buffer holds the longest sphere run
    for (const FkOp& o : e->ops) m.sph_chunk = std::max(m.sph_chunk, o.sph_end - o.sph_begin);
    {
        if (m.sph_chunk * N > 65535)
            CREATE_TRY(fail(e, STOMP_E_UNSUPPORTED, "%d spheres on one segment x %d waypoints exceed 16-bit pair ids",
                            m.sph_chunk, N));
        m.nsaves = 0;
        for (const FkOp& o : e->ops) m.nsaves = std::max(m.nsaves, o.save + 1);
        // the sincos pre-pass parks the cosines in the saved-frame area: only when that area
        // holds J x N doubles and the first save comes after the last joint segment
        int last_joint = -1, first_save = (int)e->ops.size();
        for (int i = 0; i < (int)e->ops.size(); ++i) {
            const FkOp& o = e->ops[i];
            if (o.seg >= 0 && segs[o.seg].q_index >= 0) last_joint = i;
            if (o.save >= 0 && first_save == (int)e->ops.size()) first_save = i;
        }
        m.sincos_pre = m.nsaves >= 1 && J <= 12 * m.nsaves && first_save > last_joint ? 1 : 0;
        // padding-row positions go to LDS unless that costs a workgroup per CU the launch
        // would use: one rollout launch has K_loc + 1 workgroups over the device's CUs
        const size_t stat = rollout_static_lds();
        const size_t with_pad = rollout_lds_bytes(m, 1) + stat, without = rollout_lds_bytes(m, 0) + stat;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d->device) != hipSuccess || cus <= 0)
            cus = 256;
        m.cus = cus;
        // every workgroup of the launch counts: the rollouts, the noiseless one, the pregen blocks
        // and the reuse candidates' totals blocks beside them (K = 448 with its 449 pregen blocks
        // ran two workgroups per CU at 54.6 us against three at K = 512, 47.1 us: the padding
        // positions took the slot the pregen blocks need)
        const int blocks = e->K_loc + 1 + (e->pre_on ? e->rows : 0) + (e->Kr > 0 && world == 1 ? e->K : 0);
        const int need = (blocks + cus - 1) / cus;
        m.pad_lds = (with_pad <= kRolloutLdsMax &&
                     rollout_blocks_per_cu(with_pad) >= std::min(need, rollout_blocks_per_cu(without))) ? 1 : 0;
        const size_t lds = rollout_lds_bytes(m, m.pad_lds) + stat;
        m.phased_lds = (int)rollout_phased_lds_bytes(m);
        if (getenv("STOMP_DEBUG_PHASED")) fprintf(stderr, "stomp: phased rollout LDS %d B\n", m.phased_lds);
        if (lds > kRolloutLdsMax)
            CREATE_TRY(fail(e, STOMP_E_UNSUPPORTED, "rollout kernel needs %zu B of LDS (J=%d, N=%d, S=%d, %d spheres "
                                                    "on one segment), more than %zu", lds, J, N, e->S, m.sph_chunk,
                            kRolloutLdsMax));
        // the LDS-lean slot-loop layout (DevModel::lean) when it puts more rollout workgroups on a
        // CU and the launch has more workgroups than the full layout's slots: cfg3's N = 199 (71.7
        // KB per workgroup, two per CU; lean 2 46.5 KB, three) and cfg4's two-arm tree (two saved
        // frames, a 12 KB table)
        m.lean = 0;
        const int per_cu_full = rollout_blocks_per_cu(lds);
        int per_cu[3] = {per_cu_full, 0, 0};
        for (int lv = 1; lv <= 2; ++lv)
            if (rollout_lean_allowed(m, lv)) per_cu[lv] = rollout_blocks_per_cu(rollout_lds_bytes(m, 0, lv) + stat, lv);
        if (need > per_cu_full) {
            int best = per_cu_full;
            for (int lv = 1; lv <= 2; ++lv)
                if (per_cu[lv] > best) {
                    best = per_cu[lv];
                    m.lean = lv;
                }
        }
        if (const char* v = getenv("STOMP_DEBUG_LEAN")) {   // tests / A/B: force a layout
            const int lv = atoi(v);
            if (lv >= 0 && lv <= 2 && rollout_lean_allowed(m, lv)) m.lean = lv;
        }
        if (getenv("STOMP_DEBUG_LEAN_PRINT"))
            fprintf(stderr, "stomp: rollout LDS full %zu / lean1 %zu / lean2 %zu B, workgroups per CU %d / %d / %d, "
                            "needed %d, layout lean %d\n", lds, rollout_lds_bytes(m, 0, 1) + stat,
                    rollout_lds_bytes(m, 0, 2) + stat, per_cu[0], per_cu[1], per_cu[2], need, m.lean);
    }
    if (!cost_supported(m)) CREATE_TRY(fail(e, STOMP_E_UNSUPPORTED, "FK program too large (%d ops, %d segments)",
                                            m.nops, m.nseg));
    {
        // the rollout kernel's LDS table image (RolloutLds from .sph on), padding positions last
        const RolloutLds L = rollout_lds(J, N, e->S, m.sph_chunk, m.nsaves, m.nseg, m.nops, m.nslots, 1);
        std::vector<unsigned char> img(L.total - L.sph, 0);
        auto put = [&](size_t off, const void* src, size_t bytes) {
            if (bytes) std::memcpy(img.data() + (off - L.sph), src, bytes);
        };
        std::vector<double> jlim(2 * (size_t)J);
        for (int j = 0; j < J; ++j) { jlim[2 * j] = jmin[j]; jlim[2 * j + 1] = jmax[j]; }
        put(L.sph, sph.data(), sizeof(DevSphere) * e->S);
        put(L.seg, segs.data(), sizeof(DevSegment) * segs.size());
        put(L.ops, e->ops.data(), sizeof(FkOp) * e->ops.size());
        put(L.slot, slot_sph.data(), sizeof(int) * slot_sph.size());
        put(L.hl, has_lim.data(), sizeof(int) * J);
        put(L.jlim, jlim.data(), sizeof(double) * jlim.size());
        unsigned long long* d_img;
        CREATE_TRY(upload(e, &d_img, (const unsigned long long*)img.data(), img.size() / 8));
        if (hipStreamSynchronize(e->stream) != hipSuccess)   // img is pageable and goes out of scope
            CREATE_TRY(fail(e, STOMP_E_DEVICE, "table upload failed"));
        const unsigned char* base = (const unsigned char*)d_img;
        m.img = d_img;
        m.img_words = (int)(((m.pad_lds ? L.total : L.pad) - L.sph) / 8);
        m.sph = (const DevSphere*)(base + (L.sph - L.sph));
        m.segs = (const DevSegment*)(base + (L.seg - L.sph));
        m.ops = (const FkOp*)(base + (L.ops - L.sph));
        m.slot_sph = (const int*)(base + (L.slot - L.sph));
        e->d_pad_pos = (double*)(base + (L.pad - L.sph));
    }
    m.pad_pos = e->d_pad_pos; m.sdf = e->d_sdf;
    {
        // the field as 4^3 bricks (one 128-B line per brick) when it is large: the SDF gathers of
        // neighbouring rollouts' spheres, which differ in x and y as much as in z, then land on
        // shared lines (a z-fastest line holds 64 cells along z only).  STOMP_SDF_LAYOUT =
        // brick | linear overrides.  The engine keeps its own bricked copy; the caller's field
        // ([x][y][z], the ABI's layout) is only read here.
        const char* lay = std::getenv("STOMP_SDF_LAYOUT");
        const bool brick = lay ? std::strcmp(lay, "brick") == 0 : ncell * sizeof(uint16_t) > ((size_t)64 << 20);
        m.brick = 0;
        m.nby = (d->grid.ny + 3) / 4;
        m.nbz = (d->grid.nz + 3) / 4;
        if (brick) {
            uint16_t* bricks = nullptr;
            CREATE_TRY(dev_alloc(e, &bricks, sdf_brick_cells(d->grid.nx, d->grid.ny, d->grid.nz)));
            launch_sdf_bricks(e->d_sdf, bricks, d->grid.nx, d->grid.ny, d->grid.nz, e->stream);
            if (hipStreamSynchronize(e->stream) != hipSuccess)
                CREATE_TRY(fail(e, STOMP_E_DEVICE, "distance-field brick layout failed"));
            if (!d->grid.data_on_device) {   // the linear upload is no longer needed
                auto it = std::find(e->allocs.begin(), e->allocs.end(), (void*)e->d_sdf);
                if (it != e->allocs.end()) {
                    hipFree(*it);
                    e->allocs.erase(it);
                }
            }
            e->d_sdf = bricks;
            m.sdf = bricks;
            m.brick = 1;
        }
    }
    e->terms.segs = m.segs;
    e->tq_model.segs = m.segs;
    m.nx = d->grid.nx; m.ny = d->grid.ny; m.nz = d->grid.nz;
    m.ny_d = (double)m.ny; m.nz_d = (double)m.nz;
    m.hi_x = m.nx - 1.5; m.hi_y = m.ny - 1.5; m.hi_z = m.nz - 1.5;
    m.ox = d->grid.origin[0]; m.oy = d->grid.origin[1]; m.oz = d->grid.origin[2]; m.res = d->grid.resolution;
    m.inv_res = 1.0 / d->grid.resolution;
    m.start = e->d_start; m.goal = e->d_goal;
    const double invTime = 1.0 / e->disc;   // stomp_optimizer.cpp:620
    for (int k = 0; k < 7; ++k) {
        m.vel_coef[k] = invTime * kDiffRules[0][k];
        if ((k < kVelTap0 || k > kVelTap1) && kDiffRules[0][k] != 0.0)
            CREATE_TRY(fail(e, STOMP_E_UNSUPPORTED, "velocity rule tap %d outside the kernel's stencil", k));
    }
    m.w_obs = e->w_obs; m.w_con = e->w_con; m.w_tq = e->w_tq;
    m.QT = e->d_QT;
    // piece counters of the waypoint-split rollout launches (zeroed; the last piece resets its own)
    // one per rollout of any split launch: split_pieces takes nro <= cus / 2 (two pieces or more
    // per rollout), and an eval batch may hold more rows than K_loc + 1
    m.split_cap = std::max(e->K_loc + 2, m.cus / 2 + 1);
    CREATE_TRY(dev_alloc(e, &m.split_cnt, (size_t)m.split_cap));
    if (m.lean && m.nsaves > 0) {   // a [nsaves][12][N] block per rollout workgroup of a launch
        m.sv_rows = e->K_loc + 1;
        CREATE_TRY(dev_alloc(e, &m.sv_glob, (size_t)m.sv_rows * m.nsaves * 12 * N));
    }
    {
        const char* env = std::getenv("STOMP_DEBUG_SPLIT_MAX");
        m.split_max = env ? std::atoi(env) : 0;
        const char* xi = std::getenv("STOMP_DEBUG_XCTL_INLINE");
        m.x_ctl_inline = xi && std::strcmp(xi, "1") == 0 ? 1 : 0;
    }
    m.pad_collision = 0;
    launch_pad_fk(m, e->d_start, e->d_goal, e->d_pad_pos, e->d_pad_cf, e->stream);
    int pad_cf = 0;
    if (hipMemcpyAsync(&pad_cf, e->d_pad_cf, sizeof(int), hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        CREATE_TRY(fail(e, STOMP_E_DEVICE, "padding FK failed: %s", hipGetErrorString(hipGetLastError())));
    m.pad_collision = pad_cf;
    e->pad_collision = pad_cf;
    if (hipMemcpyAsync(e->d_last_traj, e->d_theta, sizeof(double) * J * N, hipMemcpyDeviceToDevice, e->stream) !=
            hipSuccess ||
        hipMemcpyAsync(e->d_best_traj, e->d_theta, sizeof(double) * J * N, hipMemcpyDeviceToDevice, e->stream) !=
            hipSuccess)
        CREATE_TRY(fail(e, STOMP_E_DEVICE, "trajectory copies failed"));

    const bool local_id = world > 1 && std::memcmp(d->comm_id, kLocalMagic, sizeof kLocalMagic) == 0;
    if (local_id) {
        uint64_t gid = 0;
        std::memcpy(&gid, (const char*)d->comm_id + 8, sizeof gid);
        std::shared_ptr<LocalGroup> g;
        {
            std::lock_guard<std::mutex> lk(g_groups_mu);
            auto it = g_groups.find(gid);
            if (it != g_groups.end()) g = it->second;
        }
        if (!g) CREATE_TRY(fail(e, STOMP_E_COMM, "unknown local exchange group (stomp_comm_local_id)"));
        {
            std::lock_guard<std::mutex> lk(g->mu);
            if (g->world != world) CREATE_TRY(fail(e, STOMP_E_COMM, "local group of %d ranks, engine world_size %d",
                                                   g->world, world));
            if (g->joined[e->rank]) CREATE_TRY(fail(e, STOMP_E_COMM, "rank %d joined the local group twice", e->rank));
            // everything that changes the per-iteration exchange sequence: the decomposition, the
            // shapes, the reused rollouts (two more all-gathers) and the weights phases
            const long long sig[6] = {e->gather ? 1 : 0, e->K, J, N, e->Kr, e->split_modes ? 1 : 0};
            if (g->has_sig && std::memcmp(sig, g->sig, sizeof sig) != 0)
                CREATE_TRY(fail(e, STOMP_E_COMM, "rank %d: decomposition (%s, K=%lld, J=%d, N=%d, K_r=%d) differs from the "
                                "group's (%s, K=%lld, J=%lld, N=%lld, K_r=%lld)", e->rank, e->gather ? "gather" : "partials",
                                (long long)e->K, J, N, e->Kr, g->sig[0] ? "gather" : "partials", g->sig[1], g->sig[2],
                                g->sig[3], g->sig[4]));
            std::memcpy(g->sig, sig, sizeof sig);
            g->has_sig = true;
            g->joined[e->rank] = 1;
            g->slot[e->rank].device = e->device;
            for (int q = 0; q < world; ++q)   // copies between the ranks' devices go peer to peer
                if (g->joined[q] && g->slot[q].device != e->device) {
                    (void)hipDeviceEnablePeerAccess(g->slot[q].device, 0);
                    (void)hipGetLastError();   // already enabled is fine
                }
            bool all = true;
            for (int q = 0; q < world; ++q) all = all && g->joined[q];
            if (all) {
                std::lock_guard<std::mutex> lk2(g_groups_mu);
                g_groups.erase(gid);   // every rank holds it now
            }
        }
        e->local = g;
        if (hipEventCreateWithFlags(&e->ev_ready, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_done, hipEventDisableTiming) != hipSuccess)
            CREATE_TRY(fail(e, STOMP_E_DEVICE, "hipEventCreate failed"));
        CREATE_TRY(dev_alloc(e, &e->d_mm_all, (size_t)world * 2 * J * N));
    }
#ifdef STOMP_WITH_RCCL
    if (const char* to = std::getenv("STOMP_COMM_TIMEOUT_S")) {
        const double v = std::atof(to);
        if (v > 0.0) e->comm_timeout_s = v;
    }
    if (const char* st = std::getenv("STOMP_DEBUG_STALL_COLLECTIVE")) {
        e->stall_at = std::atoll(st);
        if (e->stall_at > 0 && hipHostMalloc((void**)&e->h_stall, sizeof(unsigned), hipHostMallocMapped) != hipSuccess)
            CREATE_TRY(fail(e, STOMP_E_DEVICE, "hipHostMalloc (stall hook) failed"));
        if (e->h_stall) *e->h_stall = 0u;
    }
    if (world > 1 && !local_id) {
        ncclUniqueId id;
        std::memcpy(&id, d->comm_id, sizeof id);
        if (ncclCommInitRank(&e->comm, world, id, e->rank) != ncclSuccess)
            CREATE_TRY(fail(e, STOMP_E_COMM, "ncclCommInitRank failed"));
        // every rank must run the same decomposition and shape, or the per-iteration collectives
        // would not pair up (one all-gather against an all-reduce and two all-gathers): one
        // all-reduce(max) of (x, -x) pairs at creation
        // (K_r and the weights phases too: they change the exchange sequence)
        const double sm = e->split_modes ? 1.0 : 0.0;
        const double h[12] = {e->gather ? 1.0 : 0.0, e->gather ? -1.0 : 0.0, (double)e->K, -(double)e->K,
                              (double)J,           -(double)J,            (double)N,    -(double)N,
                              (double)e->Kr,       -(double)e->Kr,        sm,           -sm};
        double* d_sig = nullptr;
        CREATE_TRY(dev_alloc(e, &d_sig, 12));
        double r[12];
        if (hipMemcpyAsync(d_sig, h, sizeof h, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
            (!coll_post(e, "decomposition check (all-reduce(max))") &&
             ncclAllReduce(d_sig, d_sig, 12, ncclFloat64, ncclMax, e->comm, e->stream) != ncclSuccess))
            CREATE_TRY(fail(e, STOMP_E_COMM, "decomposition check across ranks failed"));
        coll_mark(e);
        if (hipMemcpyAsync(r, d_sig, sizeof r, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            CREATE_TRY(fail(e, STOMP_E_COMM, "decomposition check across ranks failed"));
        CREATE_TRY(sync_stream(e));   // bounded: a rank that never gets here fails the others
        for (int k = 0; k < 12; k += 2)
            if (r[k] != -r[k + 1])
                CREATE_TRY(fail(e, STOMP_E_COMM, "ranks disagree on the K-sharded decomposition (gather, K, J, N, K_r, "
                                "weights phases; "
                                "entry %d: max %g, min %g)", k / 2, r[k], -r[k + 1]));
    } else if (e->split_modes && world == 1) {
        // STOMP_DEBUG_RCCL_ONE_RANK=1 (with the sharded-modes hook): a one-rank communicator,
        // so the sharded path's RCCL all-reduce / all-gathers run on a one-GPU box
        const char* one = std::getenv("STOMP_DEBUG_RCCL_ONE_RANK");
        if (one && one[0] == '1') {
            ncclUniqueId id;
            if (ncclGetUniqueId(&id) != ncclSuccess || ncclCommInitRank(&e->comm, 1, id, 0) != ncclSuccess)
                CREATE_TRY(fail(e, STOMP_E_COMM, "one-rank ncclCommInitRank failed"));
        }
    }
#endif
    if (hipStreamSynchronize(e->stream) != hipSuccess) CREATE_TRY(fail(e, STOMP_E_DEVICE, "setup failed"));
    if (e->calibrate) CREATE_TRY(calibrate_shard_mode(e));
    *out = e;
    return 0;
#undef CREATE_TRY
}

void stomp_engine_destroy(stomp_engine* e)
{
    if (!e) return;
    DeviceGuard dg(e->device);
    release(e);
    delete e;
}

int stomp_engine_refresh_field(stomp_engine* e)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    if (!e->d_sdf_caller)
        return fail(e, STOMP_E_UNSUPPORTED, "the distance field was uploaded from the host at creation (data_on_device = 0)");
    if (!e->model.brick) return 0;   // read in place
    DeviceGuard dg(e->device);
    launch_sdf_bricks(e->d_sdf_caller, e->d_sdf, e->grid_n[0], e->grid_n[1], e->grid_n[2], e->stream);
    HIP_TRY(e, hipGetLastError());
    return 0;
}

int stomp_engine_get_theta(stomp_engine* e, double* theta)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    HIP_TRY(e, hipMemcpyAsync(theta, e->d_theta, sizeof(double) * e->J * e->N, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

int stomp_engine_set_theta(stomp_engine* e, const double* theta)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    flush_noiseless(e);   // a pending noiseless rollout belongs to the theta being replaced
    HIP_TRY(e, hipMemcpyAsync(e->d_theta, theta, sizeof(double) * e->J * e->N, hipMemcpyHostToDevice, e->stream));
    SYNC_TRY(e);
    return 0;
}

int stomp_engine_iterate(stomp_engine* e, int32_t it, stomp_iter_out* out)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    flush_noiseless(e);
    int rc = enqueue_iteration(e, it, false);
    if (rc) return rc;
    HIP_TRY(e, hipMemcpyAsync(e->h_total, e->d_total, sizeof(double), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipMemcpyAsync(e->h_cf, e->d_cf, 1, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipMemcpyAsync(e->h_cf + 1, e->d_cs, 1, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    if (out) {
        out->cost = *e->h_total;
        out->collision_free = e->h_cf[0];
        out->constraints_satisfied = e->h_cf[1];
    }
    return 0;
}

int stomp_engine_run(stomp_engine* e, int32_t first_iteration, int32_t count)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    // the last iteration's noiseless rollout stays pending: it rides in the next rollout
    // launch, or is flushed by synchronize, iterate, set_theta and the trajectory reads
    for (int i = 0; i < count; ++i) {
        int rc = enqueue_iteration(e, first_iteration + i, true);
        if (rc) return rc;
    }
    return 0;
}

int stomp_engine_synchronize(stomp_engine* e)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    flush_noiseless(e);
    SYNC_TRY(e);
    return 0;
}

int stomp_engine_eval(stomp_engine* e, const double* params, int32_t num, double* costs, uint8_t* collision_free,
                      double* traj_out, int32_t iteration_member, uint8_t* constraints_satisfied)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    if (num <= 0) return 0;
    const size_t JN = (size_t)e->J * e->N;
    if (num > e->eval_cap) {
        for (void* p : {(void*)e->d_eval_params, (void*)e->d_eval_costs, (void*)e->d_eval_traj, (void*)e->d_eval_cf,
                        (void*)e->d_eval_cs}) {
            if (!p) continue;
            hipFree(p);
            e->allocs.erase(std::remove(e->allocs.begin(), e->allocs.end(), p), e->allocs.end());
        }
        int rc;
        if ((rc = dev_alloc(e, &e->d_eval_params, num * JN))) return rc;
        if ((rc = dev_alloc(e, &e->d_eval_costs, (size_t)num * e->N))) return rc;
        if ((rc = dev_alloc(e, &e->d_eval_traj, num * JN))) return rc;
        if ((rc = dev_alloc(e, &e->d_eval_cf, (size_t)num))) return rc;
        if ((rc = dev_alloc(e, &e->d_eval_cs, (size_t)num))) return rc;
        e->eval_cap = num;
    }
    HIP_TRY(e, hipMemcpyAsync(e->d_eval_params, params, sizeof(double) * num * JN, hipMemcpyHostToDevice, e->stream));
    CostArgs ca{};
    ca.params = e->d_eval_params; ca.stride = (long long)JN; ca.num_noisy = num; ca.member = iteration_member;
    ca.state_out = e->d_eval_costs; ca.cf_out = e->d_eval_cf;
    ca.traj_out = (traj_out || e->terms_on) ? e->d_eval_traj : nullptr;
    {
        Timed tm(e, T_COST);
        launch_rollouts(e, ca);
    }
    if (constraints_satisfied && !e->terms_on) HIP_TRY(e, hipMemsetAsync(e->d_eval_cs, 1, (size_t)num, e->stream));
    launch_terms_for(e, ca, e->d_eval_cs);
    HIP_TRY(e, hipGetLastError());
    HIP_TRY(e, hipMemcpyAsync(costs, e->d_eval_costs, sizeof(double) * num * e->N, hipMemcpyDeviceToHost, e->stream));
    if (collision_free)
        HIP_TRY(e, hipMemcpyAsync(collision_free, e->d_eval_cf, num, hipMemcpyDeviceToHost, e->stream));
    if (constraints_satisfied)
        HIP_TRY(e, hipMemcpyAsync(constraints_satisfied, e->d_eval_cs, num, hipMemcpyDeviceToHost, e->stream));
    if (traj_out)
        HIP_TRY(e, hipMemcpyAsync(traj_out, e->d_eval_traj, sizeof(double) * num * JN, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

// StompOptimizer::optimize loop (stomp_optimizer.cpp:284-359), device-resident: every iteration is
// followed by k_track, which keeps the loop's bookkeeping in HBM and sets the stop flag when the
// reference loop would break; all later launches of the loop then return at once.  The host
// enqueues iterations in chunks, one chunk ahead of the stop flag it reads back, so the stream
// never waits on the host.
int stomp_engine_optimize(stomp_engine* e, stomp_stats* st, double* costs_per_it)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    materialize_rows(e);
    flush_noiseless(e);
    DevTrack init{};
    init.stop = 0; init.cfi = 0; init.iterations = 0; init.success = 0;
    init.success_iteration = -1; init.collision_success_iteration = -1; init.last_improvement_iteration = -1;
    init.best = 0.0;
    e->h_track[3] = init;
    HIP_TRY(e, hipMemcpyAsync(e->d_track, &e->h_track[3], sizeof(DevTrack), hipMemcpyHostToDevice, e->stream));
    launch_track_start(e->d_track, e->stream);   // stomp_optimizer.cpp:251 start_time
    const int max_it = e->max_it;
    // host-side generateRollouts state after each iteration, to restore the one the device stopped at
    struct HostState { bool reused_next, extra_added; int row_set; };
    std::vector<HostState> after((size_t)std::max(max_it, 1));
    const int chunk = 8;
    int next = 0, checked = 0;
    hipEvent_t ev[2] = {get_event(e), get_event(e)};
    int slot_end[2] = {0, 0};
    int inflight = 0, head = 0;
    auto enqueue_chunk = [&](int slot) -> int {
        const int end = std::min(next + chunk, max_it);
        for (; next < end; ++next) {
            // K_r = 0: the noiseless rollout of iteration next rides in the next iteration's
            // rollout launch (pipelined), its k_track right after that launch
            int rc = enqueue_iteration(e, next + 1, true);
            if (rc) return rc;
            after[next] = {e->reused_next, e->extra_added, e->row_set};
        }
        HIP_TRY(e, hipMemcpyAsync(&e->h_track[slot], e->d_track, sizeof(DevTrack), hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(e, hipEventRecord(ev[slot], e->stream));
        slot_end[slot] = next;
        return 0;
    };
    int rc = 0;
    bool stopped = false;
    e->tracking = true;
    while (!stopped && checked < max_it) {
        while (inflight < 2 && next < max_it) {
            if ((rc = enqueue_chunk((head + inflight) & 1))) break;
            ++inflight;
        }
        if (rc || inflight == 0) break;
        HIP_TRY(e, hipEventSynchronize(ev[head]));
        const DevTrack& h = e->h_track[head];
        checked = slot_end[head];
        stopped = h.stop != 0;
        head ^= 1;
        --inflight;
    }
    if (!rc) rc = flush_noiseless(e);   // the last iteration's noiseless rollout and its bookkeeping
    e->tracking = false;
    SYNC_TRY(e);
    e->pool.push_back(ev[0]);
    e->pool.push_back(ev[1]);
    if (rc) return rc;
    DevTrack& t = e->h_track[2];
    HIP_TRY(e, hipMemcpy(&t, e->d_track, sizeof(DevTrack), hipMemcpyDeviceToHost));
    if (t.iterations > 0) {
        e->reused_next = after[t.iterations - 1].reused_next;
        e->extra_added = after[t.iterations - 1].extra_added;
        if (e->row_set != after[t.iterations - 1].row_set) swap_row_sets(e);   // iterations past the stop were no-ops
    }
    if (costs_per_it && t.iterations > 0)
        HIP_TRY(e, hipMemcpy(costs_per_it, e->d_opt_costs, sizeof(double) * t.iterations, hipMemcpyDeviceToHost));
    // later launches (iterate / run / eval) are not gated
    HIP_TRY(e, hipMemsetAsync(e->d_track, 0, sizeof(int), e->stream));
    SYNC_TRY(e);
    stomp_stats s;
    s.iterations = t.iterations;
    s.success = t.success;
    s.success_iteration = t.success_iteration;
    s.collision_success_iteration = t.collision_success_iteration;
    s.last_improvement_iteration = t.last_improvement_iteration;
    s.best_cost = t.best;
    const double tick_s = e->wall_khz > 0 ? 1.0 / (1000.0 * e->wall_khz) : 0.0;
    s.success_duration = t.success_iteration >= 0 ? (double)(t.t_success - t.t0) * tick_s : 0.0;
    s.collision_success_duration =
        t.collision_success_iteration >= 0 ? (double)(t.t_collision_success - t.t0) * tick_s : 0.0;
    if (st) *st = s;
    return 0;
}

int stomp_engine_get_best_torques(stomp_engine* e, double* torques)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    if (!e->torque_stats) return fail(e, STOMP_E_UNSUPPORTED, "no torque chain (segment inertias not given)");
    flush_noiseless(e);
    HIP_TRY(e, hipMemsetAsync(e->d_tq_state, 0, sizeof(double) * e->N, e->stream));
    TermsArgs ta{};
    ta.traj = e->d_best_traj; ta.state = e->d_tq_state; ta.num_noisy = 1; ta.tq_out = e->d_tq;
    launch_terms(e->tq_model, ta, e->stream);
    HIP_TRY(e, hipGetLastError());
    HIP_TRY(e, hipMemcpyAsync(torques, e->d_tq, sizeof(double) * e->N, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

// ---------------------------------------------------------------- PolicyImprovement API
// policy_improvement.h:86-126 step by step on the engine's rollout set, for callers that run
// their own Task::execute between the steps (the fused stomp_engine_iterate does the same work
// in one launch sequence)
int stomp_pi_get_rollouts(stomp_engine* e, int32_t iteration, const double* noise_stddev, double* rollouts,
                          int32_t* num_generated)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    materialize_rows(e);
    if (e->world > 1 || e->gather) return fail(e, STOMP_E_UNSUPPORTED, "the PolicyImprovement API is single-rank");
    if (!noise_stddev) return fail(e, STOMP_E_INVALID, "null noise_stddev");
    flush_noiseless(e);
    if (int rc = begin_generate(e)) return rc;
    NoiseArgs na = noise_args(e, iteration);
    for (int d = 0; d < e->J; ++d) na.sigma.v[d] = noise_stddev[d];   // generateRollouts(noise_stddev)
    na.stop = nullptr;
    na.row_begin = 0;
    na.K_gen_global = e->K_gen;
    {
        Timed tm(e, T_NOISE);
        launch_noise(na, e->stream);
    }
    e->pi_weight = e->w_smooth;
    HIP_TRY(e, hipGetLastError());
    if (rollouts)
        HIP_TRY(e, hipMemcpyAsync(rollouts, e->d_params, sizeof(double) * e->K_gen * e->J * e->N,
                                  hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    if (num_generated) *num_generated = e->K_gen;
    return 0;
}

int stomp_pi_set_rollout_costs(stomp_engine* e, const double* costs, double control_cost_weight, double* totals)
{
    if (!e || !costs) return fail(e, STOMP_E_INVALID, "null argument");
    DeviceGuard dg(e->device);
    materialize_rows(e);
    const int K = e->K, J = e->J, N = e->N;
    // state costs of the generated rows; reused rows keep theirs (policy_improvement.cpp:270-273)
    HIP_TRY(e, hipMemcpyAsync(e->d_state, costs, sizeof(double) * e->K_gen * N, hipMemcpyHostToDevice, e->stream));
    if (control_cost_weight != e->pi_weight) {
        // computeRolloutControlCosts with another weight (:264-266): every row's noise is kept,
        // its projection and control cost recomputed
        NoiseArgs na = noise_args(e, 1);
        na.stop = nullptr; na.row_begin = 0; na.K_gen_global = 0;
        for (int r = 0; r < 3; ++r) na.wr[r] = 0.5 * control_cost_weight * e->smooth[r];
        launch_noise(na, e->stream);
        e->pi_weight = control_cost_weight;
    }
    HIP_TRY(e, hipGetLastError());
    if (totals) {
        // Rollout::getCost (:149-156): state sum, then each joint's control sum
        std::vector<double> st((size_t)K * N), ct((size_t)K * J * N);
        HIP_TRY(e, hipMemcpyAsync(st.data(), e->d_state, sizeof(double) * st.size(), hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(e, hipMemcpyAsync(ct.data(), e->d_control, sizeof(double) * ct.size(), hipMemcpyDeviceToHost, e->stream));
        SYNC_TRY(e);
        for (int r = 0; r < K; ++r) {
            const double* sr = st.data() + (size_t)r * N;
            double c = sr[0];
            for (int t = 1; t < N; ++t) c += sr[t];
            for (int d = 0; d < J; ++d) {
                const double* x = ct.data() + ((size_t)r * J + d) * N;
                double sd = x[0];
                for (int t = 1; t < N; ++t) sd += x[t];
                c += sd;
            }
            totals[r] = c;
        }
    }
    SYNC_TRY(e);
    return 0;
}

int stomp_pi_improve_policy(stomp_engine* e, double* updates)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    materialize_rows(e);
    if (e->world > 1 || e->gather) return fail(e, STOMP_E_UNSUPPORTED, "the PolicyImprovement API is single-rank");
    WeightArgs wa{};
    wa.stop = nullptr;
    wa.J = e->J; wa.N = e->N; wa.K_loc = e->K_loc; wa.use_cumulative = e->use_cum;
    wa.state = e->d_state; wa.control = e->d_control; wa.noise = e->d_noise;
    wa.cum = e->use_cum ? e->d_cum : nullptr; wa.prob = e->d_prob; wa.u = e->d_u;
    wa.tc = weights_tile(e->K_loc);
    wa.nb_total = e->K / kSumBlock;
    wa.mode = W_FUSED;
    {
        Timed tm(e, T_WEIGHTS);
        if (e->use_cum) launch_cumulative(wa, e->d_cum, e->stream);
        launch_weights(wa, e->stream);
    }
    {
        Timed tm(e, T_UPDATE);
        launch_update(e->J, e->N, e->d_MT, e->d_u, nullptr, e->K / kSumBlock, nullptr, nullptr, e->stream, e->d_delta);
    }
    HIP_TRY(e, hipGetLastError());
    if (updates)
        HIP_TRY(e, hipMemcpyAsync(updates, e->d_delta, sizeof(double) * e->J * e->N, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

// setNumRollouts with the engine's counts (policy_improvement.cpp:139-141): rollouts_reused_next_
// and extra_rollouts_added_ cleared
int stomp_pi_reset(stomp_engine* e)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    SYNC_TRY(e);
    e->reused_next = false;
    e->extra_added = false;
    return 0;
}

int stomp_pi_add_extra_rollouts(stomp_engine* e, int32_t num, const double* params, const double* costs)
{
    if (!e || !params || !costs) return fail(e, STOMP_E_INVALID, "null argument");
    DeviceGuard dg(e->device);
    materialize_rows(e);
    if (num != 1) return fail(e, STOMP_E_INVALID, "one extra rollout (the loop's noiseless rollout)");
    const int J = e->J, N = e->N;
    const size_t JN = (size_t)J * N;
    // copyParametersFromPolicy, then noise = parameters - theta (policy_improvement.cpp:446-449, 464-469)
    std::vector<double> th(JN), nz(JN);
    flush_noiseless(e);
    HIP_TRY(e, hipMemcpyAsync(th.data(), e->d_theta, sizeof(double) * JN, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    for (size_t k = 0; k < JN; ++k) nz[k] = params[k] - th[k];
    HIP_TRY(e, hipMemcpyAsync(e->d_x_params, params, sizeof(double) * JN, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(e, hipMemcpyAsync(e->d_x_noise, nz.data(), sizeof(double) * JN, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(e, hipMemcpyAsync(e->d_x_state, costs, sizeof(double) * N, hipMemcpyHostToDevice, e->stream));
    // computeProjectedNoise + computeRolloutControlCosts of the extra row (:452-453)
    NoiseArgs xa = noise_args(e, 1);
    xa.stop = nullptr;
    xa.K_loc = 1; xa.first_global = 0; xa.K_gen_global = 0; xa.zero_noise = 0; xa.row_begin = 0;
    for (int r = 0; r < 3; ++r) xa.wr[r] = 0.5 * e->pi_weight * e->smooth[r];
    xa.params = e->d_x_params; xa.noise = e->d_x_noise; xa.control = e->d_x_control;
    launch_noise(xa, e->stream);
    HIP_TRY(e, hipGetLastError());
    SYNC_TRY(e);   // nz is a pageable host buffer
    e->extra_added = true;
    return 0;
}

int stomp_engine_get_best_trajectory(stomp_engine* e, double* traj)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    flush_noiseless(e);
    HIP_TRY(e, hipMemcpyAsync(traj, e->d_best_traj, sizeof(double) * e->J * e->N, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

int stomp_engine_get_last_trajectory(stomp_engine* e, double* traj)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    flush_noiseless(e);
    HIP_TRY(e, hipMemcpyAsync(traj, e->d_last_traj, sizeof(double) * e->J * e->N, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

int stomp_engine_get_rollouts(stomp_engine* e, const char* which, double* out)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    // this rank's rows (gather mode holds all K: its own start at row0)
    const size_t JN = (size_t)e->J * e->N, KJN = (size_t)e->K_loc * JN, o = (size_t)e->row0 * JN;
    const double* src = nullptr;
    size_t n = KJN;
    if (!std::strcmp(which, "params") || !std::strcmp(which, "noise")) materialize_rows(e);
    if (!std::strcmp(which, "params")) src = e->d_params + o;
    else if (!std::strcmp(which, "noise")) src = e->d_noise + o;
    else if (!std::strcmp(which, "control_costs")) src = e->d_control + o;
    else if (!std::strcmp(which, "probabilities")) src = e->d_prob + o;
    else if (!std::strcmp(which, "state_costs")) { src = e->d_state + (size_t)e->row0 * e->N; n = (size_t)e->K_loc * e->N; }
    else if (!std::strncmp(which, "x_", 2)) {
        // the extra (noiseless) rollout of addExtraRollouts (policy_improvement.cpp:443-462);
        // x_state_costs is written by every noiseless rollout, the others only with reuse
        flush_noiseless(e);
        n = (size_t)e->J * e->N;
        if (!std::strcmp(which, "x_params")) src = e->d_x_params;
        else if (!std::strcmp(which, "x_noise")) src = e->d_x_noise;
        else if (!std::strcmp(which, "x_control_costs")) src = e->d_x_control;
        else if (!std::strcmp(which, "x_state_costs")) { src = e->d_x_state; n = (size_t)e->N; }
        else return fail(e, STOMP_E_INVALID, "unknown rollout field '%s'", which);
    }
    else return fail(e, STOMP_E_INVALID, "unknown rollout field '%s'", which);
    HIP_TRY(e, hipMemcpyAsync(out, src, n * sizeof(double), hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

int stomp_engine_get_matrix(stomp_engine* e, const char* which, int32_t joint, double* out)
{
    const size_t NN = (size_t)e->N * e->N;
    if (!std::strcmp(which, "Rinv")) std::memcpy(out, e->su.Rinv.data(), NN * 8);
    else if (!std::strcmp(which, "L")) std::memcpy(out, e->su.L.data(), NN * 8);
    else if (!std::strcmp(which, "M")) std::memcpy(out, e->su.M.data(), NN * 8);
    else if (!std::strcmp(which, "R")) {
        // free block of the control-cost matrix (CovariantTrajectoryPolicy::getControlCosts)
        for (int i = 0; i < e->N; ++i)
            for (int k = 0; k < e->N; ++k)
                out[(size_t)i * e->N + k] = e->su.Rall[(size_t)(i + kPad) * e->Nall + k + kPad];
    } else if (which[0] == 'D' && which[1] >= '0' && which[1] <= '2' && which[2] == 0) {
        // policy differentiation matrix D_i (Nall x Nall), covariant_trajectory_policy.cpp:204-226
        const int r = which[1] - '0', A = e->Nall;
        std::memset(out, 0, sizeof(double) * A * A);
        for (int i = 0; i < A; ++i)
            for (int j = 0; j < kDiffRuleLength; ++j) {
                const int c = i + j - kDiffRuleLength / 2;
                if (c >= 0 && c < A) out[(size_t)i * A + c] = e->su.dcoef[r][j];
            }
    } else if (!std::strcmp(which, "Qinv")) {
        if (joint < 0 || joint >= e->J) return fail(e, STOMP_E_INVALID, "joint out of range");
        std::memcpy(out, e->su.Qinv.data() + (size_t)joint * NN, NN * 8);
    } else return fail(e, STOMP_E_INVALID, "unknown matrix '%s'", which);
    return 0;
}

int stomp_engine_get_pad_positions(stomp_engine* e, double* out)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    HIP_TRY(e, hipMemcpyAsync(out, e->d_pad_pos, sizeof(double) * 12 * e->S * 3, hipMemcpyDeviceToHost, e->stream));
    SYNC_TRY(e);
    return 0;
}

int stomp_engine_set_timing(stomp_engine* e, int32_t enable)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    collect_timing(e);
    e->timing = enable != 0;
    for (int i = 0; i < T_COUNT; ++i) { e->tot_ms[i] = 0; e->launches[i] = 0; }
    return 0;
}

int stomp_engine_get_timing(stomp_engine* e, const char* name, double* total_ms, int32_t* launches)
{
    if (!e) return fail(nullptr, STOMP_E_INVALID, "null engine");
    DeviceGuard dg(e->device);
    collect_timing(e);
    double t = 0;
    int n = 0;
    bool found = false;
    for (int i = 0; i < T_COUNT; ++i)
        if (!std::strcmp(name, "all") || !std::strcmp(name, kTimerNames[i])) {
            t += e->tot_ms[i];
            n += e->launches[i];
            found = true;
        }
    if (!found) return fail(e, STOMP_E_INVALID, "unknown timer '%s'", name);
    if (total_ms) *total_ms = t;
    if (launches) *launches = n;
    return 0;
}

int stomp_engine_local_rollouts(stomp_engine* e, int32_t* first, int32_t* count)
{
    if (first) *first = e->first;
    if (count) *count = e->K_loc;
    return 0;
}

int stomp_engine_shard_mode(stomp_engine* e, int32_t* mode)
{
    if (!e || !mode) return fail(e, STOMP_E_INVALID, "null argument");
    *mode = e->world == 1 ? STOMP_SHARD_NONE : (e->gather ? STOMP_SHARD_GATHER : STOMP_SHARD_PARTIALS);
    return 0;
}

int stomp_engine_shard_info(stomp_engine* e, double* info)
{
    if (!e || !info) return fail(e, STOMP_E_INVALID, "null argument");
    for (int k = 0; k < 6; ++k) info[k] = e->shard_info[k];
    if (!e->calibrate) info[0] = e->world == 1 ? STOMP_SHARD_NONE : (e->gather ? STOMP_SHARD_GATHER : STOMP_SHARD_PARTIALS);
    return 0;
}

int stomp_shard_decide(const double* measured, int32_t* mode)
{
    if (!measured || !mode) return STOMP_E_INVALID;
    const double gather = measured[0] + measured[3];
    const double partials = measured[1] + measured[2] + 2.0 * measured[4];
    *mode = gather <= partials ? STOMP_SHARD_GATHER : STOMP_SHARD_PARTIALS;
    return 0;
}

int stomp_sdf_build(int32_t nx, int32_t ny, int32_t nz, const double* origin, double res, double max_expansion,
                    const double* boxes, int32_t n_boxes, const double* cyl, int32_t n_cyl, uint16_t* out, void* stream)
{
    if (nx <= 0 || ny <= 0 || nz <= 0 || !(res > 0) || !out) return fail(nullptr, STOMP_E_INVALID, "invalid grid");
    const int n[3] = {nx, ny, nz};
    const double capd = std::ceil(max_expansion / res);
    if (!(capd >= 0) || capd > 255) return fail(nullptr, STOMP_E_UNSUPPORTED, "max_expansion / resolution above 255 cells");
    const int cap = (int)capd;
    const int cap2 = cap * cap;
    auto range = [&](double lo, double hi, int a, int& i0, int& i1) {
        i0 = std::max((int)std::ceil((lo - origin[a]) / res), 0);
        i1 = std::min((int)std::floor((hi - origin[a]) / res), n[a] - 1);
    };
    std::vector<int> br;
    for (int b = 0; b < n_boxes; ++b) {
        const double* q = boxes + 6 * b;
        int r[6];
        bool empty = false;
        for (int a = 0; a < 3; ++a) {
            range(q[a] - q[3 + a] / 2.0, q[a] + q[3 + a] / 2.0, a, r[2 * a], r[2 * a + 1]);
            if (r[2 * a] > r[2 * a + 1]) empty = true;
        }
        if (!empty) br.insert(br.end(), r, r + 6);
    }
    const long long big = 1LL << 40;
    std::vector<long long> cd2;
    std::vector<int> cz;
    for (int c = 0; c < n_cyl; ++c) {
        const double* q = cyl + 5 * c;
        int z0, z1;
        range(q[2] - q[4] / 2.0, q[2] + q[4] / 2.0, 2, z0, z1);
        if (z0 > z1) continue;
        std::vector<std::pair<int, int>> disc;
        for (int i = 0; i < nx; ++i) {
            const double xs = origin[0] + i * res - q[0];
            for (int j = 0; j < ny; ++j) {
                const double ys = origin[1] + j * res - q[1];
                if (xs * xs + ys * ys <= q[3] * q[3]) disc.push_back({i, j});
            }
        }
        if (disc.empty()) continue;
        std::vector<long long> t((size_t)nx * ny, big);
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < ny; ++j) {
                long long best = big;
                for (auto& pq : disc) {
                    long long dx = i - pq.first, dy = j - pq.second;
                    long long v = dx * dx + dy * dy;
                    if (v < best) best = v;
                }
                t[(size_t)i * ny + j] = std::min(best, (long long)cap2);
            }
        cd2.insert(cd2.end(), t.begin(), t.end());
        cz.push_back(z0);
        cz.push_back(z1);
    }
    hipStream_t s = (hipStream_t)stream;
    int* d_b = nullptr;
    long long* d_c = nullptr;
    int* d_z = nullptr;
    if (!br.empty() && hipMalloc(&d_b, br.size() * sizeof(int)) != hipSuccess) return fail(nullptr, STOMP_E_DEVICE, "hipMalloc");
    if (!cd2.empty() && hipMalloc(&d_c, cd2.size() * sizeof(long long)) != hipSuccess) return fail(nullptr, STOMP_E_DEVICE, "hipMalloc");
    if (!cz.empty() && hipMalloc(&d_z, cz.size() * sizeof(int)) != hipSuccess) return fail(nullptr, STOMP_E_DEVICE, "hipMalloc");
    hipError_t cp = hipSuccess;
    if (d_b) cp = hipMemcpyAsync(d_b, br.data(), br.size() * sizeof(int), hipMemcpyHostToDevice, s);
    if (d_c && cp == hipSuccess) cp = hipMemcpyAsync(d_c, cd2.data(), cd2.size() * sizeof(long long), hipMemcpyHostToDevice, s);
    if (d_z && cp == hipSuccess) cp = hipMemcpyAsync(d_z, cz.data(), cz.size() * sizeof(int), hipMemcpyHostToDevice, s);
    if (cp != hipSuccess) {
        if (d_b) hipFree(d_b);
        if (d_c) hipFree(d_c);
        if (d_z) hipFree(d_z);
        return fail(nullptr, STOMP_E_DEVICE, "sdf build: %s", hipGetErrorString(cp));
    }
    launch_sdf_build(nx, ny, nz, cap2, d_b, (int)br.size() / 6, d_c, d_z, (int)cz.size() / 2, out, s);
    hipError_t st = hipStreamSynchronize(s);
    if (d_b) hipFree(d_b);
    if (d_c) hipFree(d_c);
    if (d_z) hipFree(d_z);
    if (st != hipSuccess) return fail(nullptr, STOMP_E_DEVICE, "sdf build: %s", hipGetErrorString(st));
    return 0;
}

// bodies::ConvexMesh's convex hull (third party: qhull in geometric_shapes) as its supporting
// planes, appended to `planes` as (n, d) with unit outward n and n.x + d = 0 on the face; the steps
// of oracle/sdf_oracle.c so_hull_planes, restated in C++ (same expressions, so the same planes):
// merge vertices with identical coordinates (first index kept), incremental hull of the unique
// vertices in index order (first tetrahedron, then each vertex more than eps outside a face
// replaces the faces it sees by a fan over their horizon), faces with the same plane (n . n' >
// 1 - 1e-12, |d - d'| <= eps) merged into facets, each facet's plane spanned by the first
// non-collinear triple of its vertices (|u x w| > 1e-12 |u| |w|) that leaves every hull vertex
// within eps on one side, facets in the order of those triples.  eps = 1e-9 (1 + max |coordinate|).
// O(V log V + V F).  Returns the number of planes (-1: no volume).
namespace hull {
struct Face {
    int v[3];
    double n[3], d;
    int alive;
};
inline const double* at(const double* V, int i) { return V + 3 * (size_t)i; }
inline bool plane3(const double* V, int a, int b, int c, double* n, double* d)
{
    const double* A = at(V, a);
    const double* B = at(V, b);
    const double* C = at(V, c);
    const double u[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]};
    const double w[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]};
    n[0] = u[1] * w[2] - u[2] * w[1];
    n[1] = u[2] * w[0] - u[0] * w[2];
    n[2] = u[0] * w[1] - u[1] * w[0];
    const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    const double lu = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    const double lw = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (!(len > 1e-12 * lu * lw) || !(len > 0.0)) return false;
    n[0] /= len;
    n[1] /= len;
    n[2] /= len;
    *d = -(n[0] * A[0] + n[1] * A[1] + n[2] * A[2]);
    return true;
}
inline double sdist(const double* n, double d, const double* p) { return n[0] * p[0] + n[1] * p[1] + n[2] * p[2] + d; }
inline uint64_t edge_key(int a, int b) { return ((uint64_t)(unsigned)a << 32) | (unsigned)b; }
}  // namespace hull

static int hull_planes(const double* V, int nv, std::vector<double>& planes)
{
    using namespace hull;
    if (nv < 4) return -1;
    double ext = 0.0;
    for (int i = 0; i < 3 * nv; ++i)
        if (std::fabs(V[i]) > ext) ext = std::fabs(V[i]);
    const double eps = 1e-9 * (1.0 + ext);
    // unique vertices
    std::vector<int> ord(nv), uq;
    for (int i = 0; i < nv; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int i, int j) {
        for (int k = 0; k < 3; ++k) {
            const double x = V[3 * (size_t)i + k], y = V[3 * (size_t)j + k];
            if (x != y) return x < y;
        }
        return i < j;
    });
    for (int i = 0; i < nv; ++i) {
        const double* p = at(V, ord[i]);
        if (i > 0) {
            const double* q = at(V, ord[i - 1]);
            if (p[0] == q[0] && p[1] == q[1] && p[2] == q[2]) continue;
        }
        uq.push_back(ord[i]);
    }
    std::sort(uq.begin(), uq.end());
    const int nu = (int)uq.size();
    if (nu < 4) return -1;
    std::vector<unsigned char> onhull(nv, 0);
    std::vector<Face> F;
    std::unordered_map<uint64_t, int> em;
    {
        const int a = uq[0];
        int b = -1, c = -1, e = -1;
        double best = eps;
        for (int i = 1; i < nu; ++i) {
            const double* p = at(V, uq[i]);
            const double* A = at(V, a);
            const double dx = p[0] - A[0], dy = p[1] - A[1], dz = p[2] - A[2];
            const double r = std::sqrt(dx * dx + dy * dy + dz * dz);
            if (r > best) { best = r; b = uq[i]; }
        }
        if (b < 0) return -1;
        best = eps;
        for (int i = 1; i < nu; ++i) {
            const double* A = at(V, a);
            const double* B = at(V, b);
            const double* p = at(V, uq[i]);
            const double u[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]};
            const double w[3] = {p[0] - A[0], p[1] - A[1], p[2] - A[2]};
            const double x[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
            const double r = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]) / std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
            if (r > best) { best = r; c = uq[i]; }
        }
        if (c < 0) return -1;
        double n[3], d;
        if (!plane3(V, a, b, c, n, &d)) return -1;
        best = eps;
        for (int i = 1; i < nu; ++i) {
            const double r = std::fabs(sdist(n, d, at(V, uq[i])));
            if (r > best) { best = r; e = uq[i]; }
        }
        if (e < 0) return -1;
        const int tet[4][3] = {{a, b, c}, {a, e, b}, {b, e, c}, {c, e, a}};
        double ctr[3];
        for (int k = 0; k < 3; ++k) ctr[k] = (at(V, a)[k] + at(V, b)[k] + at(V, c)[k] + at(V, e)[k]) / 4.0;
        for (int f = 0; f < 4; ++f) {
            Face h;
            h.v[0] = tet[f][0]; h.v[1] = tet[f][1]; h.v[2] = tet[f][2];
            if (!plane3(V, h.v[0], h.v[1], h.v[2], h.n, &h.d)) return -1;
            if (sdist(h.n, h.d, ctr) > 0.0) {
                std::swap(h.v[1], h.v[2]);
                if (!plane3(V, h.v[0], h.v[1], h.v[2], h.n, &h.d)) return -1;
            }
            h.alive = 1;
            F.push_back(h);
            for (int k = 0; k < 3; ++k) em[edge_key(h.v[k], h.v[(k + 1) % 3])] = f;
        }
        onhull[a] = onhull[b] = onhull[c] = onhull[e] = 1;
    }
    std::vector<int> vis, hor;
    for (int i = 1; i < nu; ++i) {
        const int p = uq[i];
        if (onhull[p]) continue;
        const double* P = at(V, p);
        vis.clear();
        for (int f = 0; f < (int)F.size(); ++f)
            if (F[f].alive && sdist(F[f].n, F[f].d, P) > eps) vis.push_back(f);
        if (vis.empty()) continue;
        for (int f : vis) F[f].alive = 2;
        hor.clear();
        for (int f : vis)
            for (int k = 0; k < 3; ++k) {
                const int ea = F[f].v[k], eb = F[f].v[(k + 1) % 3];
                const auto it = em.find(edge_key(eb, ea));
                if (it != em.end() && F[it->second].alive == 2) continue;
                hor.push_back(ea);
                hor.push_back(eb);
            }
        for (int f : vis) F[f].alive = 0;
        for (size_t q = 0; q < hor.size(); q += 2) {
            Face h;
            h.v[0] = hor[q]; h.v[1] = hor[q + 1]; h.v[2] = p;
            h.alive = 1;
            if (!plane3(V, h.v[0], h.v[1], h.v[2], h.n, &h.d)) { h.n[0] = h.n[1] = h.n[2] = 0.0; h.d = 0.0; }
            const int id = (int)F.size();
            F.push_back(h);
            for (int k = 0; k < 3; ++k) em[edge_key(h.v[k], h.v[(k + 1) % 3])] = id;
        }
        onhull[p] = 1;
    }
    // facets
    for (const Face& f : F)
        if (f.alive)
            for (int k = 0; k < 3; ++k) onhull[f.v[k]] = 2;
    std::vector<int> hullv;
    for (int i = 0; i < nu; ++i)
        if (onhull[uq[i]] == 2) hullv.push_back(uq[i]);
    struct Facet {
        int t[3];
        double n[3], d;
    };
    std::vector<Facet> fc;
    std::vector<int> grp(F.size(), -1), fv;
    const int nf = (int)F.size();
    for (int f = 0; f < nf; ++f) {
        if (!F[f].alive || grp[f] >= 0) continue;
        fv.clear();
        for (int g = f; g < nf; ++g) {
            if (!F[g].alive || grp[g] >= 0) continue;
            if (g != f && !(F[f].n[0] * F[g].n[0] + F[f].n[1] * F[g].n[1] + F[f].n[2] * F[g].n[2] > 1.0 - 1e-12 &&
                            std::fabs(F[f].d - F[g].d) <= eps))
                continue;
            grp[g] = f;
            for (int k = 0; k < 3; ++k) fv.push_back(F[g].v[k]);
        }
        std::sort(fv.begin(), fv.end());
        fv.erase(std::unique(fv.begin(), fv.end()), fv.end());
        const int mu = (int)fv.size();
        bool found = false;
        for (int x = 0; x < mu && !found; ++x)
            for (int y = x + 1; y < mu && !found; ++y)
                for (int z = y + 1; z < mu && !found; ++z) {
                    double n[3], d;
                    if (!plane3(V, fv[x], fv[y], fv[z], n, &d)) continue;
                    double smax = -1e300, smin = 1e300;
                    for (int q : hullv) {
                        const double sd = sdist(n, d, at(V, q));
                        if (sd > smax) smax = sd;
                        if (sd < smin) smin = sd;
                    }
                    if (smax <= eps) {
                    } else if (smin >= -eps) {
                        n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; d = -d;
                    } else {
                        continue;
                    }
                    fc.push_back(Facet{{fv[x], fv[y], fv[z]}, {n[0], n[1], n[2]}, d});
                    found = true;
                }
    }
    std::sort(fc.begin(), fc.end(), [](const Facet& a, const Facet& b) {
        for (int k = 0; k < 3; ++k)
            if (a.t[k] != b.t[k]) return a.t[k] < b.t[k];
        return false;
    });
    const size_t first = planes.size();
    int np = 0;
    for (const Facet& q : fc) {
        bool dup = false;
        for (int p2 = 0; p2 < np && !dup; ++p2) {
            const double* e = planes.data() + first + 4 * p2;
            dup = q.n[0] * e[0] + q.n[1] * e[1] + q.n[2] * e[2] > 1.0 - 1e-12 && std::fabs(q.d - e[3]) <= eps;
        }
        if (dup) continue;
        planes.insert(planes.end(), {q.n[0], q.n[1], q.n[2], q.d});
        ++np;
    }
    if (np < 4) {
        planes.resize(first);
        return -1;
    }
    return np;
}

// the vertices' bounding-box centre and the largest distance of a vertex from it (bodies::
// ConvexMesh's bounding sphere before the pose; third party, parity unpinned)
static void mesh_box_sphere(const double* V, int nv, double* centre, double* radius)
{
    double lo[3] = {V[0], V[1], V[2]}, hi[3] = {V[0], V[1], V[2]};
    for (int q = 1; q < nv; ++q)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], V[3 * q + a]);
            hi[a] = std::max(hi[a], V[3 * q + a]);
        }
    for (int a = 0; a < 3; ++a) centre[a] = (lo[a] + hi[a]) / 2.0;
    double r2 = 0.0;
    for (int q = 0; q < nv; ++q) {
        const double dx = V[3 * q] - centre[0], dy = V[3 * q + 1] - centre[1], dz = V[3 * q + 2] - centre[2];
        const double s = dx * dx + dy * dy + dz * dz;
        if (s > r2) r2 = s;
    }
    *radius = std::sqrt(r2);
}

// StompCollisionSpace::setStartState's fill (stomp_collision_space.cpp:154-297, 564-650): the
// per-object lattice is set up here (the environment objects' coordinate lists by the reference's
// own running-sum loops), the marking and the EDT run on the device (k_sdf.hip)
int stomp_sdf_build_objects(int32_t nx, int32_t ny, int32_t nz, const double* origin, double res,
                            double max_expansion, const stomp_shape* shapes, int32_t n_shapes, const double* points,
                            int64_t n_points, uint16_t* out, int64_t* marked, void* stream)
{
    if (nx <= 0 || ny <= 0 || nz <= 0 || !(res > 0) || !out || !origin || n_shapes < 0 || n_points < 0 ||
        (n_shapes > 0 && !shapes) || (n_points > 0 && !points))
        return fail(nullptr, STOMP_E_INVALID, "invalid grid or object list");
    const double capd = std::ceil(max_expansion / res);
    if (!(capd >= 0) || capd > 255) return fail(nullptr, STOMP_E_UNSUPPORTED, "max_expansion / resolution above 255 cells");
    const int cap = (int)capd;
    std::vector<double> axes;
    std::vector<double> mesh_planes;   // every mesh's hull planes, 4 doubles each
    std::vector<SdfLatticeJob> jobs;
    const long long kMaxLattice = 1LL << 31;
    for (int s = 0; s < n_shapes; ++s) {
        const stomp_shape& sh = shapes[s];
        SdfLatticeJob j{};
        j.type = sh.type;
        j.res = res;
        for (int a = 0; a < 3; ++a) {
            j.pos[a] = sh.position[a];
            j.dims[a] = sh.dims[a];
        }
        const double qx = sh.orientation[0], qy = sh.orientation[1], qz = sh.orientation[2], qw = sh.orientation[3];
        if (sh.type == STOMP_SHAPE_BOX || sh.type == STOMP_SHAPE_CYLINDER) {
            // KDL::Rotation::Quaternion(x, y, z, w) (:243-246)
            const double x2 = qx * qx, y2 = qy * qy, z2 = qz * qz, w2 = qw * qw;
            const double R[9] = {w2 + x2 - y2 - z2, 2 * qx * qy - 2 * qw * qz, 2 * qx * qz + 2 * qw * qy,
                                 2 * qx * qy + 2 * qw * qz, w2 - x2 + y2 - z2, 2 * qy * qz - 2 * qw * qx,
                                 2 * qx * qz - 2 * qw * qy, 2 * qy * qz + 2 * qw * qx, w2 - x2 - y2 + z2};
            std::memcpy(j.R, R, sizeof R);
            const bool cyl = sh.type == STOMP_SHAPE_CYLINDER;
            const double* p = sh.position;
            const double* d = sh.dims;
            const double low[3] = {cyl ? p[0] - d[0] : p[0] - d[0] / 2.0, cyl ? p[1] - d[0] : p[1] - d[1] / 2.0,
                                   cyl ? p[2] - d[1] / 2.0 : p[2] - d[2] / 2.0};
            const double ext[3] = {cyl ? d[0] * 2.0 : d[0], cyl ? d[0] * 2.0 : d[1], cyl ? d[1] : d[2]};
            long long npts = 1;
            for (int a = 0; a < 3; ++a) {
                j.off[a] = (int)axes.size();
                // for (double x = xlow; x <= xlow + dim + resolution_; x += resolution_) (:255-257, 283-285)
                for (double x = low[a]; x <= low[a] + ext[a] + res; x += res) {
                    axes.push_back(x);
                    if ((long long)axes.size() - j.off[a] > kMaxLattice)
                        return fail(nullptr, STOMP_E_INVALID, "object %d: lattice too large", s);
                }
                j.n[a] = (int)axes.size() - j.off[a];
                npts *= j.n[a];
            }
            if (npts > kMaxLattice) return fail(nullptr, STOMP_E_INVALID, "object %d: lattice too large", s);
        } else if (sh.type >= STOMP_BODY_SPHERE && sh.type <= STOMP_BODY_MESH) {
            // btMatrix3x3::setRotation (bodies::Body::setPose)
            const double dq = qx * qx + qy * qy + qz * qz + qw * qw;
            const double sc = 2.0 / dq;
            const double xs = qx * sc, ys = qy * sc, zs = qz * sc;
            const double wx = qw * xs, wy = qw * ys, wz = qw * zs;
            const double xx = qx * xs, xy = qx * ys, xz = qx * zs;
            const double yy = qy * ys, yz = qy * zs, zz = qz * zs;
            const double B[9] = {1.0 - (yy + zz), xy - wz, xz + wy, xy + wz, 1.0 - (xx + zz), yz - wx,
                                 xz - wy, yz + wx, 1.0 - (xx + yy)};
            std::memcpy(j.R, B, sizeof B);
            const double* d = sh.dims;
            double r;   // bodies::*::computeBoundingSphere
            double centre[3] = {sh.position[0], sh.position[1], sh.position[2]};
            if (sh.type == STOMP_BODY_SPHERE) {
                r = d[0];
            } else if (sh.type == STOMP_BODY_BOX) {
                const double a = d[0] / 2.0, b = d[1] / 2.0, c = d[2] / 2.0;
                r = std::sqrt(a * a + b * b + c * c);
            } else if (sh.type == STOMP_BODY_CYLINDER) {
                const double h = d[1] / 2.0;
                r = std::sqrt(d[0] * d[0] + h * h);
            } else {
                // bodies::ConvexMesh: the convex hull of the vertices as planes, the lattice around
                // the bounding sphere of the vertices' bounding-box centre
                if (!sh.vertices || sh.num_vertices < 4)
                    return fail(nullptr, STOMP_E_INVALID, "mesh %d: needs at least 4 vertices", s);
                const int first = (int)mesh_planes.size() / 4;
                const int np = hull_planes(sh.vertices, sh.num_vertices, mesh_planes);
                if (np < 0) return fail(nullptr, STOMP_E_INVALID, "mesh %d: the vertices span no volume", s);
                j.nplanes = np;
                j.off[0] = first;   // plane offset, resolved to a device pointer below
                double bc[3], rb;
                mesh_box_sphere(sh.vertices, sh.num_vertices, bc, &rb);
                for (int a = 0; a < 3; ++a) {
                    j.org[a] = sh.position[a];
                    centre[a] = B[3 * a] * bc[0] + B[3 * a + 1] * bc[1] + B[3 * a + 2] * bc[2] + sh.position[a];
                    j.pos[a] = centre[a];
                }
                r = rb + d[0];
            }
            long long npts = 1;
            for (int a = 0; a < 3; ++a) {
                const double c = centre[a];
                const double lo = ((c - r) - c) * (1.0 / res), hi = ((c + r) - c) * (1.0 / res);
                if (!(std::fabs(lo) < 1e9 && std::fabs(hi) < 1e9))
                    return fail(nullptr, STOMP_E_INVALID, "body %d: lattice too large", s);
                j.lo[a] = (int)lo;   // worldToGrid truncates (stomp_collision_space.h:230-234)
                j.n[a] = (int)hi - j.lo[a] + 1;
                if (j.n[a] < 0) j.n[a] = 0;
                npts *= j.n[a];
            }
            if (npts > kMaxLattice) return fail(nullptr, STOMP_E_INVALID, "body %d: lattice too large", s);
        } else {
            return fail(nullptr, STOMP_E_INVALID, "object %d: unknown type %d", s, sh.type);
        }
        jobs.push_back(j);
    }
    hipStream_t st = (hipStream_t)stream;
    const size_t cells = (size_t)nx * ny * nz;
    unsigned char* occ = nullptr;
    unsigned short *a = nullptr, *b = nullptr;
    double *d_axes = nullptr, *d_pts = nullptr, *d_planes = nullptr;
    unsigned long long* d_marked = nullptr;
    auto cleanup = [&]() {
        if (occ) hipFree(occ);
        if (a) hipFree(a);
        if (b) hipFree(b);
        if (d_axes) hipFree(d_axes);
        if (d_pts) hipFree(d_pts);
        if (d_planes) hipFree(d_planes);
        if (d_marked) hipFree(d_marked);
    };
    if (hipMalloc(&occ, cells) != hipSuccess || hipMalloc(&a, cells * 2) != hipSuccess ||
        hipMalloc(&b, cells * 2) != hipSuccess || hipMalloc(&d_marked, sizeof(unsigned long long)) != hipSuccess ||
        (!axes.empty() && hipMalloc(&d_axes, axes.size() * sizeof(double)) != hipSuccess) ||
        (!mesh_planes.empty() && hipMalloc(&d_planes, mesh_planes.size() * sizeof(double)) != hipSuccess) ||
        (n_points > 0 && hipMalloc(&d_pts, (size_t)n_points * 3 * sizeof(double)) != hipSuccess)) {
        cleanup();
        return fail(nullptr, STOMP_E_DEVICE, "sdf build: hipMalloc");
    }
    for (SdfLatticeJob& j : jobs)
        if (j.type == kBodyMesh) {
            j.planes = d_planes + 4 * (size_t)j.off[0];
            j.off[0] = 0;
        }
    hipError_t err = hipMemsetAsync(occ, 0, cells, st);
    if (err == hipSuccess) err = hipMemsetAsync(d_marked, 0, sizeof(unsigned long long), st);
    if (err == hipSuccess && d_axes)
        err = hipMemcpyAsync(d_axes, axes.data(), axes.size() * sizeof(double), hipMemcpyHostToDevice, st);
    if (err == hipSuccess && d_planes)
        err = hipMemcpyAsync(d_planes, mesh_planes.data(), mesh_planes.size() * sizeof(double), hipMemcpyHostToDevice,
                             st);
    if (err == hipSuccess && d_pts)
        err = hipMemcpyAsync(d_pts, points, (size_t)n_points * 3 * sizeof(double), hipMemcpyHostToDevice, st);
    if (err != hipSuccess) {
        cleanup();
        return fail(nullptr, STOMP_E_DEVICE, "sdf build: %s", hipGetErrorString(err));
    }
    SdfMarkArgs g{};
    g.n[0] = nx;
    g.n[1] = ny;
    g.n[2] = nz;
    for (int k = 0; k < 3; ++k) g.o[k] = origin[k];
    g.inv_res = 1.0 / res;
    g.occ = occ;
    g.marked = d_marked;
    launch_mark_points(d_pts, n_points, g, st);
    for (const SdfLatticeJob& j : jobs) launch_mark_lattice(j, d_axes, g, st);
    launch_edt(nx, ny, nz, cap, occ, a, b, out, st);
    unsigned long long nm = 0;
    err = hipGetLastError();
    if (err == hipSuccess) err = hipMemcpyAsync(&nm, d_marked, sizeof nm, hipMemcpyDeviceToHost, st);
    if (err == hipSuccess) err = hipStreamSynchronize(st);
    cleanup();
    if (err != hipSuccess) return fail(nullptr, STOMP_E_DEVICE, "sdf build: %s", hipGetErrorString(err));
    if (marked) *marked = (int64_t)nm;
    return 0;
}

int stomp_diff_rules(double* out)
{
    if (!out) return fail(nullptr, STOMP_E_INVALID, "null argument");
    std::memcpy(out, kDiffRules, sizeof(double) * kNumDiffRules * kDiffRuleLength);
    return 0;
}

int stomp_device_alloc(int32_t device, uint64_t bytes, void** out)
{
    if (hipSetDevice(device) != hipSuccess) return fail(nullptr, STOMP_E_DEVICE, "hipSetDevice(%d) failed", device);
    hipError_t st = hipMalloc(out, bytes ? bytes : 1);
    if (st != hipSuccess) return fail(nullptr, STOMP_E_DEVICE, "hipMalloc: %s", hipGetErrorString(st));
    return 0;
}

int stomp_device_free(void* p)
{
    hipError_t st = hipFree(p);
    return st == hipSuccess ? 0 : fail(nullptr, STOMP_E_DEVICE, "hipFree: %s", hipGetErrorString(st));
}

int stomp_device_copy_to_host(void* dst, const void* src, uint64_t bytes)
{
    hipError_t st = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
    return st == hipSuccess ? 0 : fail(nullptr, STOMP_E_DEVICE, "hipMemcpy: %s", hipGetErrorString(st));
}

int stomp_device_count(int32_t* count)
{
    int n = 0;
    hipError_t st = hipGetDeviceCount(&n);
    *count = st == hipSuccess ? n : 0;
    return 0;
}

int stomp_comm_local_id(int32_t world_size, void* out128)
{
    if (world_size < 1 || !out128) return fail(nullptr, STOMP_E_INVALID, "invalid local group arguments");
    auto g = std::make_shared<LocalGroup>();
    g->world = world_size;
    g->slot.resize(world_size);
    g->joined.assign(world_size, 0);
    uint64_t gid;
    {
        std::lock_guard<std::mutex> lk(g_groups_mu);
        gid = g_next_group++;
        g_groups[gid] = g;
    }
    std::memset(out128, 0, 128);
    std::memcpy(out128, kLocalMagic, sizeof kLocalMagic);
    std::memcpy((char*)out128 + 8, &gid, sizeof gid);
    std::memcpy((char*)out128 + 16, &world_size, sizeof world_size);
    return 0;
}

int stomp_comm_unique_id(void* out128)
{
#ifdef STOMP_WITH_RCCL
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return fail(nullptr, STOMP_E_COMM, "ncclGetUniqueId failed");
    std::memcpy(out128, &id, sizeof id);
    return 0;
#else
    (void)out128;
    return fail(nullptr, STOMP_E_UNSUPPORTED, "built without RCCL");
#endif
}


// ===================================================================== engine groups
// Several engines of one shape driven in lockstep by shared launches: per iteration one rollout
// launch covering every engine's rollout workgroups and pregen blocks, one weights launch and one
// update launch (k_rollout_group, k_weights_rows_group, k_update_group), so a batch of independent
// planning problems costs three dispatches per iteration instead of three per problem.  The
// per-engine kernel arguments of a whole run are staged in pinned memory and uploaded once; each
// engine's results are the ones its own stomp_engine_run gives, bit for bit.

int stomp_stream_create(int32_t device, void** out)
{
    if (!out) return fail(nullptr, STOMP_E_INVALID, "null argument");
    DeviceGuard dg(device);
    hipStream_t s = nullptr;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return fail(nullptr, STOMP_E_DEVICE, "hipStreamCreate failed");
    *out = (void*)s;
    return 0;
}

int stomp_stream_destroy(void* stream)
{
    if (stream && hipStreamDestroy((hipStream_t)stream) != hipSuccess)
        return fail(nullptr, STOMP_E_DEVICE, "hipStreamDestroy failed");
    return 0;
}

struct stomp_group {
    std::vector<stomp_engine*> e;
    int device = 0;
    hipStream_t stream = nullptr;
    int nt = 0;                           // weights tiles per engine
    DevModel* d_models = nullptr;         // [P]
    unsigned char* d_args = nullptr;      // [iterations][P] CostArgs, then WeightArgs, then UpdateArgs
    size_t d_cap = 0;
    unsigned char* h_args = nullptr;      // pinned staging of one run's arguments
    size_t h_cap = 0;
    hipEvent_t staged = nullptr;          // the last upload from h_args is done
    std::string err;
};

namespace {
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int gfail(stomp_group* g, int code, const char* msg)
{
    g_last_error = msg;
    if (g) g->err = msg;
    return code;
}
}  // namespace

void stomp_group_destroy(stomp_group* g)
{
    if (!g) return;
    DeviceGuard dg(g->device);
    if (g->staged) {
        hipEventSynchronize(g->staged);
        hipEventDestroy(g->staged);
    }
    if (g->d_models) hipFree(g->d_models);
    if (g->d_args) hipFree(g->d_args);
    if (g->h_args) hipHostFree(g->h_args);
    delete g;
}

int stomp_group_create(stomp_engine* const* engines, int32_t n, stomp_group** out)
{
    if (!engines || n <= 0 || !out) return gfail(nullptr, STOMP_E_INVALID, "invalid group arguments");
    stomp_engine* e0 = engines[0];
    if (!e0) return gfail(nullptr, STOMP_E_INVALID, "null engine");
    const size_t lds0 = rollout_lds_bytes(e0->model, e0->model.pad_lds);
    for (int p = 0; p < n; ++p) {
        stomp_engine* e = engines[p];
        if (!e) return gfail(nullptr, STOMP_E_INVALID, "null engine");
        if (e->device != e0->device || e->stream != e0->stream)
            return gfail(nullptr, STOMP_E_INVALID, "the engines of a group share one device and one stream");
        if (e->J != e0->J || e->N != e0->N || e->K != e0->K || e->S != e0->S ||
            rollout_lds_bytes(e->model, e->model.pad_lds) != lds0 || e->model.brick != e0->model.brick)
            return gfail(nullptr, STOMP_E_INVALID, "the engines of a group have one shape (J, N, K, spheres, model, field layout)");
        if (e->world != 1 || e->Kr != 0 || !e->pre_on || e->terms_on ||
            e->split_modes || e->gather || e->use_cum || e->J > 16)
            return gfail(nullptr, STOMP_E_UNSUPPORTED,
                         "groups run single-device engines without reuse, state-cost terms or cumulative costs");
    }
    const int nt = weights_group_tiles(e0->J, e0->N, e0->K_loc);
    if (nt <= 0) return gfail(nullptr, STOMP_E_UNSUPPORTED, "rollouts per engine beyond the weights tiles");
    DeviceGuard dg(e0->device);
    stomp_group* g = new stomp_group();
    g->e.assign(engines, engines + n);
    g->device = e0->device;
    g->stream = e0->stream;
    g->nt = nt;
    std::vector<DevModel> ms(n);
    for (int p = 0; p < n; ++p) ms[p] = engines[p]->model;
    if (hipMalloc(&g->d_models, sizeof(DevModel) * n) != hipSuccess ||
        hipMemcpy(g->d_models, ms.data(), sizeof(DevModel) * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&g->staged, hipEventDisableTiming) != hipSuccess) {
        stomp_group_destroy(g);
        return gfail(nullptr, STOMP_E_DEVICE, "group allocation failed");
    }
    *out = g;
    return 0;
}

const char* stomp_group_last_error(const stomp_group* g) { return g ? g->err.c_str() : g_last_error.c_str(); }

int stomp_group_run(stomp_group* g, int32_t first, int32_t count)
{
    if (!g) return gfail(nullptr, STOMP_E_INVALID, "null group");
    if (count <= 0) return 0;
    DeviceGuard dg(g->device);
    const int P = (int)g->e.size();
    stomp_engine* e0 = g->e[0];
    for (stomp_engine* e : g->e) {
        // lockstep: the engines enter the run in one pipeline state
        if (e->pending_member != e0->pending_member || e->pre_it != e0->pre_it || e->tracking)
            return gfail(g, STOMP_E_INVALID, "the engines of a group are not at the same iteration state");
    }
    const size_t szc = align256(sizeof(CostArgs) * P), szw = align256(sizeof(WeightArgs) * P),
                 szu = align256(sizeof(UpdateArgs) * P), per = szc + szw + szu;
    const size_t bytes = per * (size_t)count;
    if (g->staged && hipEventSynchronize(g->staged) != hipSuccess)   // h_args free again
        return gfail(g, STOMP_E_DEVICE, "group staging wait failed");
    if (bytes > g->h_cap) {
        if (g->h_args) hipHostFree(g->h_args);
        g->h_args = nullptr;
        g->h_cap = 0;
        if (hipHostMalloc((void**)&g->h_args, bytes) != hipSuccess) return gfail(g, STOMP_E_DEVICE, "hipHostMalloc failed");
        g->h_cap = bytes;
    }
    if (bytes > g->d_cap) {
        if (g->d_args) {
            hipStreamSynchronize(g->stream);
            hipFree(g->d_args);
        }
        g->d_args = nullptr;
        g->d_cap = 0;
        if (hipMalloc(&g->d_args, bytes) != hipSuccess) return gfail(g, STOMP_E_DEVICE, "hipMalloc failed");
        g->d_cap = bytes;
    }
    std::vector<int> nro(count);
    std::vector<char> pregen_first(P, 0);
    for (int i = 0; i < count; ++i) {
        const int it = first + i, member = it - 1;
        CostArgs* cas = (CostArgs*)(g->h_args + per * i);
        WeightArgs* was = (WeightArgs*)(g->h_args + per * i + szc);
        UpdateArgs* uas = (UpdateArgs*)(g->h_args + per * i + szc + szw);
        for (int p = 0; p < P; ++p) {
            stomp_engine* e = g->e[p];
            // enqueue_iteration's pipelined path with pregen rows, arguments only
            int rc = begin_generate(e);   // K_r = 0: every row generated
            if (rc) return rc;
            NoiseArgs na = noise_args(e, it);
            na.K_gen_global = e->K_gen;
            na.row_begin = e->K_loc;
            na.rows_in_pre = 1;
            if (e->pre_it != it) {
                if (i > 0) return gfail(g, STOMP_E_INVALID, "group pregen rows out of step");
                pregen_first[p] = 1;
            }
            CostArgs ca{};
            ca.stop = e->d_stop;
            ca.fused_noise = 2;
            ca.nz = na;
            ca.params = e->d_params; ca.stride = (long long)e->J * e->N; ca.num_noisy = e->K_loc;
            ca.member = member; ca.state_out = e->d_state;
            ca.pre_rows = e->K_loc;
            ca.pre_next = pregen_args(e, it + 1);
            // the grouped launch is throughput-bound: its rollout workgroups price their own rows
            // (pricing in the pregen blocks re-reads theta and eps: cfg5 55.7k vs 53.9-54.5k
            // problem-it/s)
            ca.ctl_by_pre = 0;
            e->pre_it = it + 1;
            if (e->pending_member >= 0) {
                ca.x_params = e->d_theta; ca.x_member = e->pending_member;
                ca.x_state = e->d_x_state; ca.x_cf = e->d_cf; ca.x_traj = e->d_last_traj; ca.x_total = e->d_total;
                e->pending_member = -1;
            }
            const int n_ro = ca.num_noisy + (ca.x_params ? 1 : 0);
            if (p == 0) nro[i] = n_ro;
            else if (n_ro != nro[i]) return gfail(g, STOMP_E_INVALID, "group engines out of step");
            e->rows_in_pre = true;
            e->rows_eps = na.pre_eps;
            cas[p] = ca;
            WeightArgs wa{};
            wa.stop = e->d_stop;
            wa.J = e->J; wa.N = e->N; wa.K_loc = e->K_loc; wa.use_cumulative = 0;
            wa.state = e->d_state; wa.control = e->d_control; wa.noise = na.pre_eps;
            wa.prob = e->d_prob; wa.u = e->d_u;
            wa.tc = weights_tile(e->K_loc);
            wa.nb_total = e->K / kSumBlock;
            wa.mode = W_FUSED;
            was[p] = wa;
            uas[p] = UpdateArgs{e->d_MT, e->d_u, e->d_theta, e->d_stop};
            e->pending_member = member;
        }
    }
    hipStream_t s = g->stream;
    for (int p = 0; p < P; ++p)
        if (pregen_first[p]) launch_pregen(pregen_args(g->e[p], first), g->e[p]->K_loc, s);
    hipError_t err = hipMemcpyAsync(g->d_args, g->h_args, bytes, hipMemcpyHostToDevice, s);
    if (err == hipSuccess) err = hipEventRecord(g->staged, s);
    if (err != hipSuccess) return gfail(g, STOMP_E_DEVICE, "group argument upload failed");
    const int J = e0->J, N = e0->N, K = e0->K_loc;
    for (int i = 0; i < count; ++i) {
        unsigned char* base = g->d_args + per * i;
        // with timing on for the group's first engine, its timers hold the group's launches
        {
            Timed tm(e0, T_COST, s);
            launch_cost_group(e0->model, g->d_models, (const CostArgs*)base, P, nro[i], K, s);
        }
        {
            Timed tm(e0, T_WEIGHTS, s);
            launch_weights_group((const WeightArgs*)(base + szc), P, J, N, K, s);
        }
        {
            Timed tm(e0, T_UPDATE, s);
            launch_update_group(J, N, (const UpdateArgs*)(base + szc + szw), P, s);
        }
    }
    err = hipGetLastError();
    if (err != hipSuccess) return gfail(g, STOMP_E_DEVICE, hipGetErrorString(err));
    return 0;
}

int stomp_group_synchronize(stomp_group* g)
{
    if (!g) return gfail(nullptr, STOMP_E_INVALID, "null group");
    DeviceGuard dg(g->device);
    const int P = (int)g->e.size();
    bool all = true;
    for (stomp_engine* e : g->e) all = all && e->pending_member >= 0 && !e->tracking;
    if (all) {
        // every engine's pending noiseless rollout in one launch (one workgroup per engine)
        const size_t bytes = align256(sizeof(CostArgs) * P);
        if (g->staged && hipEventSynchronize(g->staged) != hipSuccess)
            return gfail(g, STOMP_E_DEVICE, "group staging wait failed");
        if (bytes > g->h_cap || bytes > g->d_cap) {
            all = false;   // the arrays of a run are larger; no run yet: per-engine flushes
        } else {
            CostArgs* cas = (CostArgs*)g->h_args;
            for (int p = 0; p < P; ++p) {
                stomp_engine* e = g->e[p];
                CostArgs ca{};
                ca.stop = e->d_stop;
                ca.num_noisy = 0;
                ca.x_params = e->d_theta; ca.x_member = e->pending_member;
                ca.x_state = e->d_x_state; ca.x_cf = e->d_cf; ca.x_traj = e->d_last_traj; ca.x_total = e->d_total;
                cas[p] = ca;
                e->pending_member = -1;
            }
            hipError_t err = hipMemcpyAsync(g->d_args, g->h_args, bytes, hipMemcpyHostToDevice, g->stream);
            if (err == hipSuccess) err = hipEventRecord(g->staged, g->stream);
            if (err != hipSuccess) return gfail(g, STOMP_E_DEVICE, "group argument upload failed");
            launch_cost_group(g->e[0]->model, g->d_models, (const CostArgs*)g->d_args, P, 1, 0, g->stream);
        }
    }
    for (stomp_engine* e : g->e) flush_noiseless(e);
    if (hipStreamSynchronize(g->stream) != hipSuccess) return gfail(g, STOMP_E_DEVICE, "group synchronize failed");
    return 0;
}

}  // extern "C"
