"""The engine's rank > 0 code path, on one GPU.

The K-sharded multi-GPU iteration: rank r owns global rollouts
[r K/W, (r+1) K/W) (first_global, K_loc).  Two decompositions:
  partials: each rank generates exactly its rows of the counter-based noise, and the ranks
    exchange (1) all-reduce(max) of [max S, -min S], (2) all-gather of the per-64-rollout-block
    exp sums, (3) all-gather of the per-block eps * P sums;
  gather (STOMP_SHARD_MODE=gather, K_r = 0): every rank makes and prices the noise rows of all K
    rollouts, evaluates its own, and one all-gather of the state-cost rows gives every rank the
    whole cost matrix;
then every rank applies delta theta = M u redundantly (policy_improvement.cpp:322-383).  Here the W ranks are W engines
of one process on device 0, each driven by its own host thread, exchanging through the
engine's in-process group (stomp_comm_local_id: device copies ordered by HIP events, in place
of RCCL).  Every rank must reproduce its slice of the single-process oracle BIT FOR BIT:
probabilities, state costs, parameters, and the (replicated) theta and noiseless rollout.
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest

from oracle import pyoracle as po
from stomp_motion_planner_icra2011_amd import engine as eng
from stomp_motion_planner_icra2011_amd import problem as pb

pytestmark = pytest.mark.gpu
THREADS = int(os.environ.get("OMP_NUM_THREADS") or 8)


MODES = ["partials", "gather"]


def make_ranks(p, world, mode=None, monkeypatch=None):
    if mode is not None:
        monkeypatch.setenv("STOMP_SHARD_MODE", mode)
    gid = eng.comm_local_id(world)
    return [eng.Engine(p, rank=r, world_size=world, comm_id=gid) for r in range(world)]


def on_threads(engines, fn):
    with cf.ThreadPoolExecutor(len(engines)) as ex:
        futs = [ex.submit(fn, r, e) for r, e in enumerate(engines)]
        return [f.result(timeout=300) for f in futs]


@pytest.mark.parametrize("world,K,Kr,mode", [(2, 256, 0, "partials"), (4, 256, 0, "partials"), (2, 256, 0, "gather"),
                                             (4, 256, 0, "gather"), (2, 128, 64, None), (4, 256, 90, None),
                                             (8, 512, 200, None)])
def test_ranks_iterate_bitwise(world, K, Kr, mode, monkeypatch):
    """Kr > 0: the reuse ranking over all ranks' rows (all-gathered totals), the chosen rows moved
    to their destination shard (policy_improvement.cpp:176-225); 90 and 200 reused rows straddle
    shard boundaries (partials: gather mode needs K_r = 0)"""
    p = pb.make_problem(grid_n=64, num_rollouts=K, num_reused_rollouts=Kr)
    engines = make_ranks(p, world, mode, monkeypatch)
    K_loc = K // world
    for r, e in enumerate(engines):
        assert (e.first, e.K_loc) == (r * K_loc, K_loc)
        assert e.shard_mode == (mode or "partials")
    o = po.Oracle(p, threads=THREADS)
    iters = range(1, 6)

    def drive(r, e):
        rec = []
        for it in iters:
            c = e.iterate(it)
            rec.append(dict(cost=c, theta=e.theta(), last=e.last_trajectory(),
                            **{f: e.rollouts(f) for f in ("probabilities", "state_costs", "params", "noise",
                                                           "control_costs")}))
        return rec

    recs = on_threads(engines, drive)
    for k, it in enumerate(iters):
        oc = o.iterate(it)
        full = {f: o.rollouts(f) for f in ("probabilities", "state_costs", "params", "noise", "control_costs")}
        for r in range(world):
            rec = recs[r][k]
            assert rec["cost"] == oc, (it, r)
            np.testing.assert_array_equal(rec["theta"], o.theta(), err_msg=f"theta it {it} rank {r}")
            np.testing.assert_array_equal(rec["last"], o.last_trajectory())
            for f, v in full.items():
                np.testing.assert_array_equal(rec[f], v[r * K_loc:(r + 1) * K_loc], err_msg=f"{f} it {it} rank {r}")
    for e in engines:
        e.close()


@pytest.mark.parametrize("mode", MODES)
def test_eight_ranks_cfg2_strong_scaling_shape(mode, monkeypatch):
    # the 8-GPU decomposition of the headline config: K = 512 over 8 ranks (64 rollouts, one
    # block each), enqueued by run() with no host sync inside the chunk
    p = pb.make_problem(grid_n=128, num_rollouts=512, num_reused_rollouts=0)
    engines = make_ranks(p, 8, mode, monkeypatch)
    o = po.Oracle(p, threads=THREADS)

    def drive(r, e):
        e.run(1, 6)
        e.synchronize()
        th, last = e.theta(), e.last_trajectory()
        c = e.iterate(7)
        return th, last, c, e.rollouts("probabilities"), e.theta()

    res = on_threads(engines, drive)
    for it in range(1, 7):
        o.iterate(it)
    th6, last6 = o.theta(), o.last_trajectory()
    oc = o.iterate(7)
    prob = o.rollouts("probabilities")
    for r, (th, last, c, pr, th7) in enumerate(res):
        np.testing.assert_array_equal(th, th6, err_msg=f"rank {r}")
        np.testing.assert_array_equal(last, last6)
        assert c == oc
        np.testing.assert_array_equal(pr, prob[64 * r:64 * (r + 1)])
        np.testing.assert_array_equal(th7, o.theta())
    for e in engines:
        e.close()


@pytest.mark.parametrize("Kr,after_cf,mode", [(0, 1000, "partials"), (0, 1000, "gather"), (0, 3, "gather"),
                                              (64, 1000, None), (40, 3, None)])
def test_ranks_optimize_loop(Kr, after_cf, mode, monkeypatch):
    # the device-resident optimize loop on every rank (identical stop decisions), with and
    # without reuse across the shards
    p = pb.make_problem(grid_n=64, num_rollouts=128, num_reused_rollouts=Kr, max_iterations=30,
                        max_iterations_after_collision_free=after_cf)
    engines = make_ranks(p, 2, mode, monkeypatch)
    o = po.Oracle(p, threads=THREADS)
    ost, ocosts = o.optimize()

    def drive(r, e):
        st, costs = e.optimize()
        return st.iterations, costs, e.best_trajectory()

    for its, costs, best in on_threads(engines, drive):
        assert its == ost.iterations
        np.testing.assert_array_equal(costs, ocosts)
        np.testing.assert_array_equal(best, o.best_trajectory())
    for e in engines:
        e.close()


@pytest.mark.parametrize("mode", MODES)
def test_ranks_with_state_terms_bitwise(mode, monkeypatch):
    # the state-cost terms (torque, orientation constraint; k_terms) on a rank's own rows: in
    # gather mode they land at the rank's offset of the all-K state buffer before the all-gather
    p = pb.make_problem(grid_n=64, num_rollouts=128, num_reused_rollouts=0, torque_cost_weight=0.001,
                        orientation_constraints=[pb.upright_constraint()])
    engines = make_ranks(p, 2, mode, monkeypatch)
    o = po.Oracle(p, threads=THREADS)

    def drive(r, e):
        rec = []
        for it in range(1, 4):
            c = e.iterate(it)
            rec.append((c, e.theta(), e.rollouts("state_costs"), e.rollouts("probabilities")))
        return rec

    recs = on_threads(engines, drive)
    for k, it in enumerate(range(1, 4)):
        oc = o.iterate(it)
        st, pr = o.rollouts("state_costs"), o.rollouts("probabilities")
        for r in range(2):
            c, th, s, pp = recs[r][k]
            assert c == oc, (it, r)
            np.testing.assert_array_equal(th, o.theta(), err_msg=f"theta it {it} rank {r}")
            np.testing.assert_array_equal(s, st[64 * r:64 * (r + 1)])
            np.testing.assert_array_equal(pp, pr[64 * r:64 * (r + 1)])
    for e in engines:
        e.close()


@pytest.mark.parametrize("world,latency_us", [(2, 0.0), (4, 0.0), (4, 5000.0)])
def test_decomposition_measured_at_creation(world, latency_us, monkeypatch):
    # no STOMP_SHARD_MODE: the ranks time both decompositions' compute and their collectives at
    # creation and take the maxima over the ranks (stomp_engine_shard_info); every rank picks the same
    # one by stomp_shard_decide's rule.  A synthetic 5 ms per collective makes the one-exchange gather
    # mode the choice; either way the iterations after the calibration are the oracle's bit for bit
    monkeypatch.setenv("STOMP_DEBUG_CALIBRATE_LOCAL", "1")
    monkeypatch.setenv("STOMP_DEBUG_SHARD_LATENCY_US", str(latency_us))
    monkeypatch.delenv("STOMP_SHARD_MODE", raising=False)
    p = pb.make_problem(grid_n=64, num_rollouts=256, num_reused_rollouts=0)
    gid = eng.comm_local_id(world)
    with cf.ThreadPoolExecutor(world) as ex:   # the calibration exchanges: one host thread per rank
        engines = list(ex.map(lambda r: eng.Engine(p, rank=r, world_size=world, comm_id=gid), range(world)))
    modes = {e.shard_mode for e in engines}
    assert len(modes) == 1, modes
    info = engines[0].shard_info
    assert info is not None and all(e.shard_info == info for e in engines)
    assert engines[0].shard_mode == eng.shard_decide(**info)
    if latency_us > 0:
        assert engines[0].shard_mode == "gather"
    o = po.Oracle(p, threads=THREADS)
    K_loc = 256 // world

    def drive(r, e):
        out = []
        for it in range(1, 4):
            out.append((e.iterate(it), e.theta(), e.rollouts("state_costs")))
        return out

    recs = on_threads(engines, drive)
    for k, it in enumerate(range(1, 4)):
        oc = o.iterate(it)
        for r in range(world):
            c, th, st = recs[r][k]
            assert c == oc, (it, r)
            np.testing.assert_array_equal(th, o.theta())
            np.testing.assert_array_equal(st, o.rollouts("state_costs")[r * K_loc:(r + 1) * K_loc])
    for e in engines:
        e.close()


def test_gather_request_not_honoured_fails(monkeypatch):
    # STOMP_SHARD_MODE=gather with reused rollouts cannot run gather mode: creation fails instead of
    # silently falling back to partials (a rank on the other mode would post other collectives)
    p = pb.make_problem(grid_n=32, num_rollouts=128, num_reused_rollouts=64)
    monkeypatch.setenv("STOMP_SHARD_MODE", "gather")
    with pytest.raises(RuntimeError, match="STOMP_SHARD_MODE=gather"):
        eng.Engine(p, rank=0, world_size=2, comm_id=eng.comm_local_id(2))


def test_ranks_disagreeing_on_the_decomposition_fail(monkeypatch):
    p = pb.make_problem(grid_n=32, num_rollouts=128, num_reused_rollouts=0)
    gid = eng.comm_local_id(2)
    monkeypatch.setenv("STOMP_SHARD_MODE", "gather")
    e0 = eng.Engine(p, rank=0, world_size=2, comm_id=gid)
    monkeypatch.setenv("STOMP_SHARD_MODE", "partials")
    with pytest.raises(RuntimeError, match="differs from the group"):
        eng.Engine(p, rank=1, world_size=2, comm_id=gid)
    del e0


def test_ranks_disagreeing_on_reused_rollouts_fail(monkeypatch):
    # K_r changes the exchange sequence (the sharded reuse posts two more all-gathers): ranks that
    # differ only in num_reused_rollouts are refused at creation, not left to post unmatched
    # collectives
    gid = eng.comm_local_id(2)
    monkeypatch.setenv("STOMP_SHARD_MODE", "partials")
    e0 = eng.Engine(pb.make_problem(grid_n=32, num_rollouts=128, num_reused_rollouts=0), rank=0, world_size=2,
                    comm_id=gid)
    with pytest.raises(RuntimeError, match="differs from the group"):
        eng.Engine(pb.make_problem(grid_n=32, num_rollouts=128, num_reused_rollouts=64), rank=1, world_size=2,
                   comm_id=gid)
    del e0


def test_cfg3_eight_rank_split_bitwise():
    # cfg3's real 8-GPU decomposition (BASELINE configs[2]): K = 4096 over 8 ranks, K_loc = 512,
    # N = 199, 256^3 device-built field, partials mode (its 6.5 MB of state rows are past gather
    # mode's 1 MiB), three iterations; every rank's slice of the oracle's rows bit for bit
    p = pb.make_problem(dof=7, waypoints=200, grid_n=256, num_rollouts=4096, num_reused_rollouts=0,
                        build_grid=False)
    n = p.grid.n
    buf = eng.DeviceBuffer(2 * n ** 3)
    eng.sdf_build_device(p, buf.ptr)
    p.sdf = buf.to_numpy(np.uint16, (n, n, n))
    gid = eng.comm_local_id(8)
    engines = [eng.Engine(p, rank=r, world_size=8, comm_id=gid, sdf_device_ptr=buf.ptr) for r in range(8)]
    assert all(e.shard_mode == "partials" and e.K_loc == 512 for e in engines)
    o = po.Oracle(p, threads=THREADS)

    def drive(r, e):
        rec = []
        for it in (1, 2, 3):
            c = e.iterate(it)
            rec.append((c, e.theta(), e.last_trajectory(), e.rollouts("state_costs"), e.rollouts("probabilities")))
        return rec

    recs = on_threads(engines, drive)
    for k, it in enumerate((1, 2, 3)):
        oc = o.iterate(it)
        st, pr = o.rollouts("state_costs"), o.rollouts("probabilities")
        for r in range(8):
            c, th, last, est, epr = recs[r][k]
            assert c == oc, (it, r)
            np.testing.assert_array_equal(th, o.theta(), err_msg=f"theta it {it} rank {r}")
            np.testing.assert_array_equal(last, o.last_trajectory())
            np.testing.assert_array_equal(est, st[512 * r:512 * (r + 1)], err_msg=f"state it {it} rank {r}")
            np.testing.assert_array_equal(epr, pr[512 * r:512 * (r + 1)], err_msg=f"prob it {it} rank {r}")
    for e in engines:
        e.close()
    buf.free()
