"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Bar: the engine and the oracle share one floating-point contract (fp64, one
rounding per operation, fixed summation orders, deterministic elementary
functions), so every stage is compared BIT FOR BIT (assert_array_equal).  The
north-star tolerance for the final trajectory, 1e-5 absolute, is asserted on
top for the multi-iteration runs.
"""
import numpy as np
import pytest

from stomp_motion_planner_icra2011_amd import problem as pb
from stomp_motion_planner_icra2011_amd import engine as eng
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu

TOL_FINAL = 1e-5  # north_star: final trajectory within 1e-5


def make(dof=7, waypoints=100, grid_n=64, K=10, Kr=0, **kw):
    return pb.make_problem(dof=dof, waypoints=waypoints, grid_n=grid_n, num_rollouts=K, num_reused_rollouts=Kr, **kw)


def test_device_math_bitwise():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-10, 0, 4000), rng.uniform(-20, 20, 4000), rng.uniform(0, 1, 2000),
                        [0.0, -0.0, 1.0, 2.0 ** -53, 1e-300, 6.283185307179586, 3.141592653589793]])
    e, l, s, c, q = eng.device_math(x)
    for i in range(0, len(x), 97):
        v = float(x[i])
        assert e[i] == po.dexp(v)
        if v > 0:
            assert l[i] == po.dlog(v)
            assert q[i] == np.sqrt(v)
        ss, cc = po.dsincos(v)
        assert s[i] == ss and c[i] == cc


def test_device_sqrt_correctly_rounded():
    rng = np.random.default_rng(2)
    x = np.abs(rng.standard_normal(100000)) * 10.0 ** rng.integers(-6, 6, 100000)
    _, _, _, _, q = eng.device_math(x)
    np.testing.assert_array_equal(q, np.sqrt(x))


def test_device_normals_bitwise():
    for (it, d, r, n) in [(1, 0, 0, 99), (7, 3, 511, 99), (500, 6, 4095, 199), (2, 13, 17, 1)]:
        np.testing.assert_array_equal(eng.device_normals(0x53544F4D50000000, it, d, r, n),
                                      po.normals(0x53544F4D50000000, it, d, r, n))


def test_setup_matrices_bitwise():
    p = make()
    o, e = po.Oracle(p), eng.Engine(p)
    for m in ("Rinv", "L", "M"):
        np.testing.assert_array_equal(e.matrix(m), o.matrix(m))
    for j in range(p.J):
        np.testing.assert_array_equal(e.matrix("Qinv", j), o.matrix("Qinv", j))
    np.testing.assert_array_equal(e.theta(), o.theta())
    np.testing.assert_array_equal(e.pad_positions(), o.pad_positions())


@pytest.mark.parametrize("dof", [7, 14])
def test_execute_bitwise(dof):
    p = make(dof=dof)
    o, e = po.Oracle(p), eng.Engine(p)
    rng = np.random.default_rng(3)
    th = o.theta()
    # large perturbations: exercise joint limits, collisions and out-of-grid spheres
    params = th[None] + rng.standard_normal((6, p.J, p.N)).cumsum(axis=2) * 0.05
    params[0] = th
    params[5] += 3.0
    costs, cf, traj = e.execute(params, iteration_member=1)
    for r in range(params.shape[0]):
        oc, ocf, otr = o.execute(params[r], iteration_member=1)
        np.testing.assert_array_equal(costs[r], oc)
        np.testing.assert_array_equal(traj[r], otr)
        assert bool(cf[r]) == ocf
    c0, cf0, _ = e.execute(params[0], iteration_member=0)
    oc0, ocf0, _ = o.execute(params[0], iteration_member=0)
    np.testing.assert_array_equal(c0, oc0)
    assert cf0 == ocf0


def test_execute_more_rows_than_rollouts_bitwise():
    # Task::execute batches larger than K + 1 (the facade's executeBatch with several extra
    # rollouts): K = 20 and 40 rows run the waypoint-split launch with 40 rollouts, one piece
    # counter each (the counters were sized K + 2); twice, so the counters' reset by the
    # last piece is exercised too
    p = make(K=20)
    o, e = po.Oracle(p), eng.Engine(p)
    rng = np.random.default_rng(11)
    th = o.theta()
    for rep in range(2):
        params = th[None] + rng.standard_normal((40, p.J, p.N)).cumsum(axis=2) * 0.05
        params[7] += 2.0   # joint limits and collisions
        costs, cf, traj = e.execute(params, iteration_member=1)
        for r in range(params.shape[0]):
            oc, ocf, otr = o.execute(params[r], iteration_member=1)
            np.testing.assert_array_equal(costs[r], oc, err_msg=f"rep {rep} row {r}")
            np.testing.assert_array_equal(traj[r], otr)
            assert bool(cf[r]) == ocf, (rep, r)


@pytest.mark.parametrize("grid_n,K", [(64, 20), (66, 10)])
def test_brick_layout_bitwise(monkeypatch, grid_n, K):
    # the distance field re-laid as 4^3 bricks inside the engine (the default past 64 MiB, 512^3):
    # same voxels, same lookups, so every iteration is bit-identical; 66 is not a multiple of 4
    # (padding bricks)
    monkeypatch.setenv("STOMP_SDF_LAYOUT", "brick")
    p = make(K=K, grid_n=grid_n)
    o, e = po.Oracle(p), eng.Engine(p)
    for it in range(1, 6):
        _compare_iteration(o, e, it)
    rng = np.random.default_rng(5)
    params = o.theta()[None] + rng.standard_normal((4, p.J, p.N)).cumsum(axis=2) * 0.08
    costs, cf, _ = e.execute(params, iteration_member=1)
    for r in range(4):
        oc, ocf, _ = o.execute(params[r], iteration_member=1)
        np.testing.assert_array_equal(costs[r], oc)
        assert bool(cf[r]) == ocf


@pytest.mark.parametrize("dof,waypoints,lean", [(7, 200, 2), (7, 200, 1), (14, 100, 1), (7, 100, 1)])
def test_lean_layout_bitwise(monkeypatch, capfd, dof, waypoints, lean):
    # the LDS-lean slot-loop layout (DevModel::lean: saved branch-point frames in HBM, the FK and
    # joint-limit tables through the scalar cache, no (sin, cos) pre-pass; lean 2 also the sphere
    # table), forced at K = 300 (more rollouts than CUs, so the launch takes the slot loop):
    # bit-identical to the oracle, and an eval batch larger than the saved-frame blocks made at
    # creation grows them
    monkeypatch.setenv("STOMP_DEBUG_LEAN", str(lean))
    monkeypatch.setenv("STOMP_DEBUG_LEAN_PRINT", "1")
    p = make(dof=dof, waypoints=waypoints, K=300)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    assert f"layout lean {lean}" in capfd.readouterr().err
    for it in range(1, 4):
        _compare_iteration(o, e, it)
    rng = np.random.default_rng(9)
    params = o.theta()[None] + rng.standard_normal((320, p.J, p.N)).cumsum(axis=2) * 0.05
    costs, cf, _ = e.execute(params, iteration_member=1)
    for r in range(0, 320, 37):
        oc, ocf, _ = o.execute(params[r], iteration_member=1)
        np.testing.assert_array_equal(costs[r], oc)
        assert bool(cf[r]) == ocf


def test_refresh_field_after_an_in_place_rebuild(monkeypatch):
    # a device field the engine copies into its bricked layout (the default past 64 MiB; forced
    # here at 64^3): after the caller rebuilds its buffer in place, stomp_engine_refresh_field
    # remakes the copy, so the engine plans against the new field -- bit for bit the oracle of
    # the new scene.  Without the refresh the engine keeps the field it was created with.
    monkeypatch.setenv("STOMP_SDF_LAYOUT", "brick")
    shelf, empty = make(K=16), make(K=16)
    empty.boxes, empty.cylinders = [], []
    empty.sdf = pb.build_sdf(empty.grid, [], [])
    buf = eng.DeviceBuffer(2 * 64 ** 3)
    eng.sdf_build_device(shelf, buf.ptr)
    e = eng.Engine(empty, sdf_device_ptr=buf.ptr)
    stale = eng.Engine(empty, sdf_device_ptr=buf.ptr)
    eng.sdf_build_device(empty, buf.ptr)     # the scene changed: the shelf and the pole are gone
    e.refresh_field()
    o_new, o_old = po.Oracle(empty), po.Oracle(shelf)
    for it in range(1, 4):
        _compare_iteration(o_new, e, it)
        o_old.iterate(it)
        stale.iterate(it)
    np.testing.assert_array_equal(stale.theta(), o_old.theta())
    assert not np.array_equal(e.theta(), stale.theta())


def test_slot_loop_runs_between_other_calls_bitwise():
    # K + 1 > CUs (the slot-loop launches of cfg2), pipelined runs interleaved with get_theta,
    # iterate, execute and set_theta: the pending noiseless rollout and the pregen rows made ahead
    # stay consistent across the calls
    p = make(K=320, grid_n=64)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    e.run(1, 4)
    for it in range(1, 5):
        o.iterate(it)
    np.testing.assert_array_equal(e.theta(), o.theta())          # get_theta flushes
    e.run(5, 3)
    for it in range(5, 8):
        o.iterate(it)
    _compare_iteration(o, e, 8)                                     # iterate after a run
    e.run(9, 2)
    e.synchronize()
    for it in range(9, 11):
        o.iterate(it)
    costs, cf, _ = e.execute(o.theta()[None], iteration_member=1)   # execute after a run
    oc, ocf, _ = o.execute(o.theta(), iteration_member=1)
    np.testing.assert_array_equal(costs[0], oc)
    np.testing.assert_array_equal(e.last_trajectory(), o.last_trajectory())
    th = o.theta() + 0.01
    e.set_theta(th)
    o.set_theta(th)
    e.run(11, 3)
    for it in range(11, 14):
        o.iterate(it)
    np.testing.assert_array_equal(e.theta(), o.theta())
    for f in ("state_costs", "probabilities"):
        np.testing.assert_array_equal(e.rollouts(f), o.rollouts(f), err_msg=f)


def _compare_iteration(o, e, it):
    oc = o.iterate(it)
    ec = e.iterate(it)
    assert ec[0] == oc[0] and ec[1] == oc[1], (it, ec, oc)
    for f in ("params", "noise", "control_costs", "state_costs", "probabilities"):
        np.testing.assert_array_equal(e.rollouts(f), o.rollouts(f), err_msg=f"iteration {it} field {f}")
    np.testing.assert_array_equal(e.theta(), o.theta(), err_msg=f"theta after iteration {it}")
    np.testing.assert_array_equal(e.last_trajectory(), o.last_trajectory())


@pytest.mark.parametrize("K,Kr", [(10, 0), (10, 5), (20, 10), (130, 0)])
def test_iterations_bitwise(K, Kr):
    p = make(K=K, Kr=Kr)
    o, e = po.Oracle(p), eng.Engine(p)
    for it in range(1, 11):
        _compare_iteration(o, e, it)


@pytest.mark.parametrize("mode", ["fused", "pick", "no_spec"])
@pytest.mark.parametrize("dof,K,Kr", [(7, 20, 10), (14, 16, 6), (7, 12, 11), (7, 63, 30), (7, 96, 40), (7, 130, 129)])
def test_reused_rows_priced_ahead_or_after_bitwise(monkeypatch, mode, dof, K, Kr):
    # the reuse step on one device: every candidate priced by the rollout launch and the chosen
    # one copied in the weights launch (K < 64: k_weights_wave_pick) or by its own launch
    # (STOMP_DEBUG_NO_PICK_FUSE=1, and K >= 64: k_reuse_pick), or (STOMP_DEBUG_NO_SPEC=1) the
    # chosen row priced after the ranking (k_noise_rows<REUSE>); K_r = K - 1 reaches the
    # lowest-ranked candidates; K = 63 fills the wave with the extra rollout's lane; K > 64
    # takes reuse_choice's ranking through the shared sel[] array (k_noise.hip), at K = 96 in the
    # split launch with its pricing blocks, at K = 130 (131 rollouts: no split) in the slot loop
    monkeypatch.setenv("STOMP_DEBUG_NO_SPEC", "1" if mode == "no_spec" else "0")
    monkeypatch.setenv("STOMP_DEBUG_NO_PICK_FUSE", "1" if mode == "pick" else "0")
    p = make(dof=dof, K=K, Kr=Kr)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    for it in range(1, 7):
        _compare_iteration(o, e, it)


def test_per_joint_noise_schedule_bitwise():
    # params.yaml:19-26 gives noise_stddev / noise_decay per joint (policy_improvement_loop.cpp:155-160)
    sig = [2.0, 1.5, 3.0, 0.5, 2.5, 1.0, 4.0]
    dec = [0.999, 0.995, 1.0, 0.99, 0.999, 0.98, 0.995]
    p = make(K=20, Kr=10, noise_stddev=sig, noise_decay=dec)
    o, e = po.Oracle(p), eng.Engine(p)
    for it in range(1, 6):
        _compare_iteration(o, e, it)


def test_cumulative_costs_bitwise():
    p = make(K=16, use_cumulative_costs=True)
    o, e = po.Oracle(p), eng.Engine(p)
    for it in range(1, 4):
        _compare_iteration(o, e, it)


def test_cfg2_shape_one_iteration_bitwise():
    # BASELINE cfg2 workload shape (K=512, N=99, J=7) on a 128^3 field
    p = make(K=512, grid_n=128)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    _compare_iteration(o, e, 1)
    _compare_iteration(o, e, 2)


@pytest.mark.parametrize("dof,waypoints,Kr", [(14, 100, 4), (7, 40, 0), (7, 65, 3), (7, 129, 0)])
def test_fused_noise_shapes_bitwise(dof, waypoints, Kr):
    # the rollout kernel's fused noise phase: two 8-joint tiles (14 DOF), one or two waypoint
    # halves per wave (N = 39, 64, 128), reused rows priced by k_noise beside it
    p = make(dof=dof, waypoints=waypoints, K=16, Kr=Kr)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    for it in range(1, 4):
        _compare_iteration(o, e, it)


@pytest.mark.parametrize("K,cum", [(128, False), (192, True)])
def test_sharded_weight_phases_bitwise(monkeypatch, K, cum):
    # the multi-GPU weights decomposition (MINMAX -> all-reduce -> PSUM -> all-gather -> USUM ->
    # all-gather -> update from block partials) on one device, collectives as identities/copies
    monkeypatch.setenv("STOMP_DEBUG_SHARDED_MODES", "1")
    p = make(K=K, Kr=0, use_cumulative_costs=cum)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    for it in range(1, 4):
        _compare_iteration(o, e, it)


def test_sharded_weight_phases_through_rccl_bitwise(monkeypatch):
    # the same decomposition with the collectives issued through RCCL on a one-rank
    # communicator (ncclAllReduce max, two ncclAllGather), as the multi-GPU engine issues them
    monkeypatch.setenv("STOMP_DEBUG_SHARDED_MODES", "1")
    monkeypatch.setenv("STOMP_DEBUG_RCCL_ONE_RANK", "1")
    p = make(K=128, Kr=0)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    for it in range(1, 4):
        _compare_iteration(o, e, it)
    e.run(4, 20)
    for it in range(4, 24):
        o.iterate(it)
    np.testing.assert_array_equal(e.theta(), o.theta())


def test_stuck_collective_fails_within_the_deadline(monkeypatch):
    # A rank that never posts its side of a collective, modelled on a one-rank RCCL communicator:
    # STOMP_DEBUG_STALL_COLLECTIVE=5 withholds the fifth collective (iteration 2's first
    # all-gather of the sharded weights phases) and makes the stream wait behind it.  The bounded
    # wait aborts the communicator after STOMP_COMM_TIMEOUT_S and fails with STOMP_E_COMM naming
    # that collective; later calls fail the same way instead of hanging.
    import time
    monkeypatch.setenv("STOMP_DEBUG_SHARDED_MODES", "1")
    monkeypatch.setenv("STOMP_DEBUG_RCCL_ONE_RANK", "1")
    monkeypatch.setenv("STOMP_COMM_TIMEOUT_S", "2")
    monkeypatch.setenv("STOMP_DEBUG_STALL_COLLECTIVE", "5")
    p = make(K=128, Kr=0)
    e = eng.Engine(p)
    t0 = time.time()
    with pytest.raises(RuntimeError) as ei:
        e.run(1, 3)
        e.synchronize()
    dt = time.time() - t0
    msg = str(ei.value)
    assert "error -4" in msg and "did not complete within 2.0 s" in msg, msg
    assert "first collective not complete: all-gather of iteration 2 (#5)" in msg, msg
    assert "communicator aborted" in msg, msg
    assert dt < 20, dt
    with pytest.raises(RuntimeError, match="communicator aborted"):
        e.run(4, 1)


def test_waypoints_200_dual_arm_bitwise():
    p = make(dof=14, waypoints=200, K=64)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    for it in range(1, 3):
        _compare_iteration(o, e, it)


def test_optimize_100_iterations():
    p = make(K=20, Kr=10, max_iterations=100, max_iterations_after_collision_free=100)
    o, e = po.Oracle(p), eng.Engine(p)
    ost, ocosts = o.optimize()
    est, ecosts = e.optimize()
    assert est.iterations == ost.iterations
    assert est.success_iteration == ost.success_iteration
    assert est.collision_success_iteration == ost.collision_success_iteration
    assert est.last_improvement_iteration == ost.last_improvement_iteration
    np.testing.assert_array_equal(ecosts, ocosts)
    eb, ob = e.best_trajectory(), o.best_trajectory()
    assert np.max(np.abs(eb - ob)) <= TOL_FINAL
    np.testing.assert_array_equal(eb, ob)


def test_run_matches_iterate():
    p = make(K=64)
    e1, e2 = eng.Engine(p), eng.Engine(p)
    for it in range(1, 6):
        e1.iterate(it)
    e2.run(1, 5)
    e2.synchronize()
    np.testing.assert_array_equal(e1.theta(), e2.theta())


def test_out_of_order_iterations_bitwise():
    """The engine makes the next iteration's noise rows ahead (pregen blocks of the rollout
    launch, ping-pong buffers keyed by iteration parity).  Iteration numbers that skip, repeat
    or go back, with set_theta / execute calls in between, must discard those rows."""
    p = make(K=64)
    o, e = po.Oracle(p), eng.Engine(p)
    th = o.theta()
    for it in (1, 2, 5, 6, 6, 3, 10, 12, 11):
        if it == 3:
            nt = th + 0.01
            o.set_theta(nt)
            e.set_theta(nt)
        if it == 10:
            c, cf, _ = e.execute(th[None], iteration_member=4)
            oc, ocf, _ = o.execute(th, iteration_member=4)
            np.testing.assert_array_equal(c[0], oc)
        _compare_iteration(o, e, it)


def test_run_chunks_match_iterate():
    """run() chunks that continue, restart and skip iteration numbers, against iterate()."""
    p = make(K=128)
    e1, e2 = eng.Engine(p), eng.Engine(p)
    seq = [(1, 3), (4, 2), (4, 1), (9, 3)]
    for first, n in seq:
        for it in range(first, first + n):
            e1.iterate(it)
        e2.run(first, n)
    e2.synchronize()
    np.testing.assert_array_equal(e1.theta(), e2.theta())
    # run leaves its last noiseless rollout pending: a trajectory read evaluates it, and so does
    # set_theta before replacing the theta it belongs to
    e1.iterate(12)
    e2.run(12, 1)
    np.testing.assert_array_equal(e1.last_trajectory(), e2.last_trajectory())
    e1.iterate(13)
    e2.run(13, 1)
    th = e1.theta()
    e2.set_theta(th + 0.02)
    e1.set_theta(th + 0.02)
    np.testing.assert_array_equal(e1.last_trajectory(), e2.last_trajectory())
    e1.iterate(14)
    e2.run(14, 1)
    e2.synchronize()
    np.testing.assert_array_equal(e1.theta(), e2.theta())
    np.testing.assert_array_equal(e1.last_trajectory(), e2.last_trajectory())


def test_sdf_build_device_bitwise():
    for n in (32, 64, 96):
        p = make(grid_n=n)
        buf = eng.DeviceBuffer(2 * n ** 3)
        eng.sdf_build_device(p, buf.ptr)
        np.testing.assert_array_equal(buf.to_numpy(np.uint16, (n, n, n)), p.sdf)


def test_engine_on_device_sdf():
    p = make(grid_n=64)
    buf = eng.DeviceBuffer(2 * 64 ** 3)
    eng.sdf_build_device(p, buf.ptr)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    o = po.Oracle(p)
    for it in range(1, 4):
        _compare_iteration(o, e, it)


def _golden(name):
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", name + ".npz"))


def test_golden_cfg1_iterate_10_5():
    g = _golden("cfg1_iterate_10_5")
    e = eng.Engine(make(grid_n=128, K=10, Kr=5))
    for it in range(1, 11):
        c, cf = e.iterate(it)
        assert c == g["costs"][it - 1] and cf == bool(g["cf"][it - 1])
        np.testing.assert_array_equal(e.theta(), g["theta"][it - 1])
    np.testing.assert_array_equal(e.rollouts("state_costs"), g["state_costs"])
    np.testing.assert_array_equal(e.rollouts("probabilities"), g["probabilities"])


def test_golden_cfg1_optimize():
    # cfg1 (K = 20, K_r = 10, 128^3): the north-star check on best_group_trajectory_
    g = _golden("cfg1_optimize_20_10")
    e = eng.Engine(make(grid_n=128, K=20, Kr=10, max_iterations=100))
    st, costs = e.optimize()
    np.testing.assert_array_equal(costs, g["costs"])
    best = e.best_trajectory()
    np.testing.assert_array_equal(best, g["best"])
    assert np.abs(best - g["best"]).max() <= TOL_FINAL
    assert [st.iterations, st.success, st.success_iteration, st.collision_success_iteration,
            st.last_improvement_iteration] == list(g["stats"])
    assert st.best_cost == g["best_cost"][0]


@pytest.mark.parametrize("waypoints,K,Kr,dof", [(200, 20, 10, 7), (30, 12, 4, 7), (200, 16, 0, 14), (12, 8, 3, 7)])
def test_waypoint_split_shapes_bitwise(waypoints, K, Kr, dof):
    # the split body at other shapes: N = 199 (four or more pieces: one FK wave each), a short
    # trajectory (pieces of a few waypoints, the halo clamped at both ends), 14 DOF, with and
    # without the fused reuse step
    p = make(dof=dof, waypoints=waypoints, K=K, Kr=Kr, grid_n=64)
    o, e = po.Oracle(p), eng.Engine(p)
    for it in range(1, 5):
        _compare_iteration(o, e, it)


def test_reuse_ranking_past_the_fused_path_bitwise():
    # K + 1 > 1024 candidates: the reuse step takes k_reuse (one workgroup per candidate, the last
    # ranks and copies) and k_noise_rows without the fused ranking; K <= 1023 takes the fused path
    # (the rollout launch's totals blocks, the reused rows' kernel ranks and copies)
    p = make(K=1088, Kr=100, grid_n=64)
    o, e = po.Oracle(p, threads=8), eng.Engine(p)
    for it in range(1, 4):
        _compare_iteration(o, e, it)


@pytest.mark.parametrize("pieces", [1, 2, 3, 8, 40])
@pytest.mark.parametrize("K,Kr,dof", [(20, 10, 7), (64, 0, 7), (16, 0, 14)])
def test_waypoint_split_pieces_bitwise(monkeypatch, pieces, K, Kr, dof):
    # k_rollout_split: a rollout's waypoints over `pieces` workgroups (1: the phased one-workgroup
    # body), the velocity halo, the per-joint control rows dealt over the pieces, the last
    # piece's costs.sum() and collision flag: the oracle's rows and totals bit for bit
    monkeypatch.setenv("STOMP_DEBUG_SPLIT_MAX", str(pieces))
    p = make(dof=dof, K=K, Kr=Kr, grid_n=64)
    o, e = po.Oracle(p), eng.Engine(p)
    for it in range(1, 5):
        _compare_iteration(o, e, it)
    # a batch of rows through stomp_engine_eval (per-rollout totals and flags: every piece counts)
    rng = np.random.default_rng(pieces)
    rows = o.theta()[None] + 0.3 * rng.standard_normal((3,) + o.theta().shape)
    costs, cf, traj = e.execute(rows, 3)
    for i in range(3):
        co, cfo, tro = o.execute(rows[i], 3)
        np.testing.assert_array_equal(costs[i], co)
        np.testing.assert_array_equal(traj[i], tro)
        assert bool(cf[i]) == cfo


def test_golden_execute_cases():
    g = _golden("execute_cases")
    for dof in (7, 14):
        e = eng.Engine(make(dof=dof, grid_n=64, K=10))
        c, cf, tr = e.execute(g[f"params_{dof}"], 1)
        np.testing.assert_array_equal(c, g[f"costs_{dof}"])
        np.testing.assert_array_equal(tr, g[f"traj_{dof}"])
        np.testing.assert_array_equal(cf, g[f"cf_{dof}"])


@pytest.mark.parametrize("K,Kr,after_cf", [(20, 10, 3), (10, 0, 1), (20, 10, 1000), (16, 8, 1)])
def test_device_optimize_loop_stops_like_the_reference(K, Kr, after_cf):
    # the device-resident loop (k_track + stop flag, chunks enqueued ahead) must stop at the
    # reference's iteration (stomp_optimizer.cpp:340-344), leave theta as the last executed
    # iteration did, and let plain iterations continue from there
    p = make(K=K, Kr=Kr, max_iterations=37, max_iterations_after_collision_free=after_cf)
    o, e = po.Oracle(p), eng.Engine(p)
    ost, ocosts = o.optimize()
    est, ecosts = e.optimize()
    assert (est.iterations, est.success, est.success_iteration, est.collision_success_iteration,
            est.last_improvement_iteration) == (ost.iterations, ost.success, ost.success_iteration,
                                                ost.collision_success_iteration, ost.last_improvement_iteration)
    assert est.best_cost == ost.best_cost
    np.testing.assert_array_equal(ecosts, ocosts)
    np.testing.assert_array_equal(e.best_trajectory(), o.best_trajectory())
    np.testing.assert_array_equal(e.last_trajectory(), o.last_trajectory())
    np.testing.assert_array_equal(e.theta(), o.theta())
    # the extra (noiseless) rollout the next iteration's reuse ranking reads: priced on the
    # iteration the loop stops at too (addExtraRollouts runs before the break)
    fields = ("x_params", "x_noise", "x_control_costs", "x_state_costs") if Kr > 0 else ("x_state_costs",)
    for f in fields:
        np.testing.assert_array_equal(e.rollouts(f), o.rollouts(f), err_msg=f)
    for it in range(est.iterations + 1, est.iterations + 3):
        _compare_iteration(o, e, it)


@pytest.mark.parametrize("K,Kr", [(16, 6), (130, 0)])
def test_policy_improvement_api_bitwise(K, Kr):
    # the stomp_pi_* entry points driven as policy_improvement_loop.cpp:143-202 drives
    # PolicyImprovement, with Task::execute through stomp_engine_eval in between
    p = make(K=K, Kr=Kr)
    o, e = po.Oracle(p), eng.Engine(p)
    pr = p.params
    w = pr.smoothness_cost_weight
    for it in range(1, 8):
        sig = np.full(p.J, pr.noise_stddev * pr.noise_decay ** (it - 1))
        rollouts = e.pi_get_rollouts(it, sig)
        costs, _, _ = e.execute(rollouts, iteration_member=it - 1)
        if it == 2:   # another weight re-prices every row; the loop's weight restores it
            e.pi_set_rollout_costs(costs, 2.0 * w)
        totals = e.pi_set_rollout_costs(costs, w)
        upd = e.pi_improve_policy()
        th = e.theta() + 1.0 * upd   # CovariantTrajectoryPolicy::updateParameters
        e.set_theta(th)
        c, cf, _ = e.execute(th, iteration_member=it - 1)
        e.pi_add_extra_rollout(th, c)
        oc, ocf = o.iterate(it)
        assert cf == ocf
        np.testing.assert_array_equal(th, o.theta(), err_msg=f"theta it {it}")
        for f in ("params", "noise", "control_costs", "state_costs", "probabilities"):
            np.testing.assert_array_equal(e.rollouts(f), o.rollouts(f), err_msg=f"it {it} {f}")
        st, ct = o.rollouts("state_costs"), o.rollouts("control_costs")
        want = []
        for k in range(K):
            v = float(st[k][0])
            for x in st[k][1:]:
                v += float(x)
            for row in ct[k]:
                sd = float(row[0])
                for x in row[1:]:
                    sd += float(x)
                v += sd
            want.append(v)
        np.testing.assert_array_equal(totals, want)
        if Kr:
            for f in ("x_params", "x_noise", "x_control_costs", "x_state_costs"):
                np.testing.assert_array_equal(e.rollouts(f), o.rollouts(f), err_msg=f"it {it} {f}")


def test_optimize_statistics_torques_and_durations():
    # STOMPStatistics.torques of the best trajectory (stomp_optimizer.cpp:384-398) and the
    # (collision_)success durations (:306-319)
    p = make(K=20, Kr=10, grid_n=128, max_iterations=60, max_iterations_after_collision_free=1000)
    o, e = po.Oracle(p), eng.Engine(p)
    ost, _ = o.optimize()
    est, _ = e.optimize()
    np.testing.assert_array_equal(e.best_torques(), o.best_torques())
    assert est.success_iteration == ost.success_iteration
    if est.collision_success_iteration >= 0:
        assert 0.0 < est.collision_success_duration < 30.0
    if est.success_iteration >= 0:
        assert est.collision_success_duration <= est.success_duration < 30.0
    else:
        assert est.success_duration == 0.0
