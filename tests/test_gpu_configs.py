"""GPU parity at the BASELINE.json workloads themselves (not scaled-down shapes).

Every config the bench reports is run here through the C ABI and compared with the CPU
oracle on the same inputs, BIT FOR BIT (assert_array_equal), plus the north-star 1e-5
bound on best_group_trajectory_ for the optimize runs:

  cfg2  7-DOF, N=99, K=512, 256^3 device-built SDF: 10 iterations, every rollout field,
        then StompOptimizer::optimize for 100 iterations
  cfg3  7-DOF, N=199, 256^3: the per-GPU shard shape K=512, the whole K=4096 iteration on one
        device (plain and through the sharded weights phases), and StompOptimizer::optimize
        over 25 iterations of the whole K=4096
  cfg4  14-DOF, N=99, K=1024, 512^3 device-built SDF (the HBM-bound field): 3 iterations
        field by field, then StompOptimizer::optimize over 25 iterations
  cfg5  the bench's own shape: 64 planning problems (K=128 each, distinct start / goal / seed)
        as ONE engine group (stomp_group_run, shared launches) on one device SDF; and 8
        problems on separate engine streams, enqueued interleaved

The distance field is built on the device by stomp_sdf_build (as bench.py does) and copied
to the host for the oracle.  Reference: policy_improvement_loop.cpp:143-202.
"""
import os

import numpy as np
import pytest

from oracle import pyoracle as po
from stomp_motion_planner_icra2011_amd import engine as eng
from stomp_motion_planner_icra2011_amd import problem as pb

pytestmark = pytest.mark.gpu

TOL_FINAL = 1e-5  # north_star: final trajectory within 1e-5
THREADS = int(os.environ.get("OMP_NUM_THREADS") or 8)
FIELDS = ("params", "noise", "control_costs", "state_costs", "probabilities")


def problem_on_device_sdf(**kw):
    """make_problem without the numpy SDF; the field is built on the device and copied back."""
    p = pb.make_problem(build_grid=False, **kw)
    n = p.grid.n
    buf = eng.DeviceBuffer(2 * n ** 3)
    eng.sdf_build_device(p, buf.ptr)
    p.sdf = buf.to_numpy(np.uint16, (n, n, n))
    return p, buf


def compare_iteration(o, e, it, fields=FIELDS):
    oc = o.iterate(it)
    ec = e.iterate(it)
    assert ec == oc, (it, ec, oc)
    for f in fields:
        np.testing.assert_array_equal(e.rollouts(f), o.rollouts(f), err_msg=f"iteration {it} field {f}")
    np.testing.assert_array_equal(e.theta(), o.theta(), err_msg=f"theta after iteration {it}")
    np.testing.assert_array_equal(e.last_trajectory(), o.last_trajectory())


@pytest.fixture(scope="module")
def cfg2():
    p, buf = problem_on_device_sdf(dof=7, waypoints=100, grid_n=256, num_rollouts=512, num_reused_rollouts=0,
                                   max_iterations=100)
    yield p, buf
    buf.free()


def test_cfg2_sdf_matches_host_build(cfg2):
    p, _ = cfg2
    np.testing.assert_array_equal(p.sdf, pb.build_sdf(p.grid, p.boxes, p.cylinders))


def test_cfg2_ten_iterations_bitwise(cfg2):
    p, buf = cfg2
    o = po.Oracle(p, threads=THREADS)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    for it in range(1, 11):
        compare_iteration(o, e, it)


def test_cfg2_run_matches_oracle(cfg2):
    # the bench's own call: iterations enqueued by stomp_engine_run with no host sync
    p, buf = cfg2
    o = po.Oracle(p, threads=THREADS)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    e.run(1, 25)
    e.synchronize()
    for it in range(1, 26):
        o.iterate(it)
    np.testing.assert_array_equal(e.theta(), o.theta())
    np.testing.assert_array_equal(e.last_trajectory(), o.last_trajectory())
    for f in FIELDS:
        np.testing.assert_array_equal(e.rollouts(f), o.rollouts(f), err_msg=f)


def test_cfg2_optimize_100_iterations(cfg2):
    p, buf = cfg2
    o = po.Oracle(p, threads=THREADS)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    ost, ocosts = o.optimize()
    est, ecosts = e.optimize()
    assert est.iterations == ost.iterations == 100
    assert (est.success, est.success_iteration, est.collision_success_iteration, est.last_improvement_iteration) == \
        (ost.success, ost.success_iteration, ost.collision_success_iteration, ost.last_improvement_iteration)
    np.testing.assert_array_equal(ecosts, ocosts)
    eb, ob = e.best_trajectory(), o.best_trajectory()
    assert np.max(np.abs(eb - ob)) <= TOL_FINAL
    np.testing.assert_array_equal(eb, ob)


@pytest.fixture(scope="module")
def sdf256_n199():
    p, buf = problem_on_device_sdf(dof=7, waypoints=200, grid_n=256, num_rollouts=512, num_reused_rollouts=0)
    yield p, buf
    buf.free()


def test_cfg3_shard_shape_bitwise(sdf256_n199):
    # one GPU's shard of cfg3 at N = 8: K = 512, N = 199, J = 7
    p, buf = sdf256_n199
    assert p.N == 199
    o = po.Oracle(p, threads=THREADS)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    for it in range(1, 6):
        compare_iteration(o, e, it)


@pytest.mark.parametrize("sharded", [False, True])
def test_cfg3_whole_iteration_on_one_device(sdf256_n199, monkeypatch, sharded):
    # the whole cfg3 iteration (K = 4096, N = 199) on one device; with the sharded weights
    # phases (MINMAX / PSUM / USUM over 64 block partials) as the 8-GPU run computes them
    if sharded:
        monkeypatch.setenv("STOMP_DEBUG_SHARDED_MODES", "1")
    base, buf = sdf256_n199
    p = pb.make_problem(dof=7, waypoints=200, grid_n=256, num_rollouts=4096, num_reused_rollouts=0,
                        build_grid=False)
    p.sdf = base.sdf
    o = po.Oracle(p, threads=THREADS)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    for it in range(1, 3):
        compare_iteration(o, e, it, fields=("state_costs", "probabilities"))
    np.testing.assert_array_equal(e.rollouts("params"), o.rollouts("params"))


@pytest.mark.parametrize("K,reused", [(2049, 0), (3001, 300)])
def test_half_width_weights_tiles_bitwise(sdf256_n199, K, reused):
    # K in (2048, 4096]: the weights update runs the two-column row tiles (ragged K, with and
    # without reuse), every rollout field bit for bit
    base, buf = sdf256_n199
    p = pb.make_problem(dof=7, waypoints=100, grid_n=256, num_rollouts=K, num_reused_rollouts=reused,
                        build_grid=False)
    p.sdf = base.sdf
    o = po.Oracle(p, threads=THREADS)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    for it in range(1, 4):
        compare_iteration(o, e, it)


def optimize_matches(o, e, iterations):
    """StompOptimizer::optimize (stomp_optimizer.cpp:249-401) on both sides: the same statistics,
    the same per-iteration costs, and best_group_trajectory_ within the north-star 1e-5 and bit
    for bit."""
    ost, ocosts = o.optimize()
    est, ecosts = e.optimize()
    assert est.iterations == ost.iterations == iterations
    assert (est.success, est.success_iteration, est.collision_success_iteration, est.last_improvement_iteration) == \
        (ost.success, ost.success_iteration, ost.collision_success_iteration, ost.last_improvement_iteration)
    np.testing.assert_array_equal(ecosts, ocosts)
    eb, ob = e.best_trajectory(), o.best_trajectory()
    assert np.max(np.abs(eb - ob)) <= TOL_FINAL
    np.testing.assert_array_equal(eb, ob)
    np.testing.assert_array_equal(e.theta(), o.theta())


def test_cfg3_optimize_whole_K(sdf256_n199):
    # cfg3's whole K = 4096 rollouts at N = 199 through the device-resident optimize loop
    base, buf = sdf256_n199
    p = pb.make_problem(dof=7, waypoints=200, grid_n=256, num_rollouts=4096, num_reused_rollouts=0,
                        build_grid=False, max_iterations=25, max_iterations_after_collision_free=1000)
    p.sdf = base.sdf
    o = po.Oracle(p, threads=THREADS)
    e = eng.Engine(p, sdf_device_ptr=buf.ptr)
    optimize_matches(o, e, 25)
    e.close()


def test_cfg4_dual_arm_512_grid_bitwise():
    p, buf = problem_on_device_sdf(dof=14, waypoints=100, grid_n=512, num_rollouts=1024, num_reused_rollouts=0,
                                   max_iterations=25, max_iterations_after_collision_free=1000)
    try:
        assert p.J == 14 and len(p.spheres) > 90
        o = po.Oracle(p, threads=THREADS)
        e = eng.Engine(p, sdf_device_ptr=buf.ptr)
        for it in range(1, 4):
            compare_iteration(o, e, it)
        e.close()
        # the optimize loop from a fresh start, 25 iterations
        o = po.Oracle(p, threads=THREADS)
        e = eng.Engine(p, sdf_device_ptr=buf.ptr)
        optimize_matches(o, e, 25)
        e.close()
    finally:
        buf.free()


def test_cfg5_bench_shape_one_group():
    # bench.py --workload cfg5 on one GPU: 64 problems (K = 128, 256^3), one engine group on one
    # stream, the problems' offsets / seeds drawn as bench_problems draws them; two runs
    base, buf = problem_on_device_sdf(dof=7, waypoints=100, grid_n=256, num_rollouts=128, num_reused_rollouts=0)
    s = eng.Stream()
    engines, oracles = [], []
    try:
        P = 64
        rng = np.random.default_rng(1234)
        offsets = rng.uniform(-0.15, 0.15, (P, 2, base.J))
        for i in range(P):
            d = offsets[i]
            p = pb.make_problem(dof=7, waypoints=100, grid_n=256, num_rollouts=128, num_reused_rollouts=0,
                                build_grid=False, seed=base.seed + 1 + i, start=list(base.start + d[0]),
                                goal=list(base.goal + d[1]))
            p.sdf = base.sdf
            engines.append(eng.Engine(p, sdf_device_ptr=buf.ptr, stream=s.ptr))
            oracles.append(po.Oracle(p, threads=THREADS))
        group = eng.EngineGroup(engines)
        for first, count in ((1, 5), (6, 4)):
            group.run(first, count)
            group.synchronize()
            for o in oracles:
                for it in range(first, first + count):
                    o.iterate(it)
            for i, (e, o) in enumerate(zip(engines, oracles)):
                np.testing.assert_array_equal(e.theta(), o.theta(), err_msg=f"problem {i}")
                np.testing.assert_array_equal(e.last_trajectory(), o.last_trajectory(), err_msg=f"problem {i}")
                np.testing.assert_array_equal(e.rollouts("state_costs"), o.rollouts("state_costs"),
                                              err_msg=f"problem {i}")
                np.testing.assert_array_equal(e.rollouts("probabilities"), o.rollouts("probabilities"),
                                              err_msg=f"problem {i}")
        assert not np.array_equal(engines[0].theta(), engines[63].theta())
        group.close()
    finally:
        for e in engines:
            e.close()
        s.close()
        buf.free()


def test_cfg5_eight_problems_on_separate_streams():
    # bench.py --problems 8: one engine (own stream) per problem, one shared device SDF,
    # every problem's iterations enqueued as one run before any is synchronised
    base, buf = problem_on_device_sdf(dof=7, waypoints=100, grid_n=256, num_rollouts=128, num_reused_rollouts=0)
    try:
        rng = np.random.default_rng(1234)
        probs, engines, oracles = [], [], []
        for i in range(8):
            d = rng.uniform(-0.15, 0.15, (2, base.J))
            p = pb.make_problem(dof=7, waypoints=100, grid_n=256, num_rollouts=128, num_reused_rollouts=0,
                                build_grid=False, seed=base.seed + 1 + i, start=list(base.start + d[0]),
                                goal=list(base.goal + d[1]))
            p.sdf = base.sdf
            probs.append(p)
            engines.append(eng.Engine(p, sdf_device_ptr=buf.ptr))
            oracles.append(po.Oracle(p, threads=THREADS))
        for first, count in ((1, 6), (7, 4)):
            for e in engines:
                e.run(first, count)
            for e in engines:
                e.synchronize()
            for o in oracles:
                for it in range(first, first + count):
                    o.iterate(it)
            for i, (e, o) in enumerate(zip(engines, oracles)):
                np.testing.assert_array_equal(e.theta(), o.theta(), err_msg=f"problem {i}")
                np.testing.assert_array_equal(e.last_trajectory(), o.last_trajectory(), err_msg=f"problem {i}")
                np.testing.assert_array_equal(e.rollouts("state_costs"), o.rollouts("state_costs"))
        # the problems differ (distinct seeds and endpoints)
        assert not np.array_equal(engines[0].theta(), engines[1].theta())
        for e in engines:
            e.close()
    finally:
        buf.free()
