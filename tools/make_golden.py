#!/usr/bin/env python3
"""Generates the golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no golden vectors and cannot be built or imported here
(SURVEY.md §8c), so these fixtures are outputs of this repo's own CPU oracle
(oracle/stomp_oracle.c) on the synthetic workloads of SURVEY.md §8d: they pin
the oracle against regressions and give the GPU tests fixed expected values.
Parity against the reference itself stays UNPINNED.

Usage: python tools/make_golden.py   (rewrites tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle as po  # noqa: E402
from stomp_motion_planner_icra2011_amd import problem as pb  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
SEED = 0x53544F4D50000000


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"{path}: {os.path.getsize(path)} B")


def math_kats():
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-700, 700, 200), rng.uniform(-30, 30, 200), rng.uniform(0, 1, 100),
                        [0.0, -0.0, 1.0, 0.5, 2.0 ** -30, 1e-300, np.pi, 2 * np.pi, 1e6, -1e6]])
    e = np.array([po.dexp(v) for v in x])
    lg = np.array([po.dlog(v) if v > 0 else 0.0 for v in x])
    sc = np.array([po.dsincos(v) for v in x])
    ctrs = np.array([[0, 0, 0, 0], [0xFFFFFFFF] * 4, [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                     [1, 2, 3, 4]], dtype=np.uint32)
    keys = np.array([[0, 0], [0xFFFFFFFF] * 2, [0xA4093822, 0x299F31D0], [5, 6]], dtype=np.uint32)
    ph = np.array([po.philox(list(map(int, c)), list(map(int, k))) for c, k in zip(ctrs, keys)], dtype=np.uint32)
    cases = [(1, 0, 0, 99), (7, 3, 511, 99), (500, 6, 4095, 199), (2, 13, 17, 1)]
    z = np.concatenate([po.normals(SEED, *c) for c in cases])
    save("math_kats", x=x, exp=e, log=lg, sin=sc[:, 0], cos=sc[:, 1], philox_ctr=ctrs, philox_key=keys,
         philox_out=ph, normal_cases=np.array(cases), normals=z)


def setup_fixture():
    p = pb.make_problem(grid_n=64, num_rollouts=10, num_reused_rollouts=0)
    o = po.Oracle(p)
    save("setup_pr2like7", Rinv=o.matrix("Rinv"), L=o.matrix("L"), M=o.matrix("M"), Qinv0=o.matrix("Qinv", 0),
         Qinv3=o.matrix("Qinv", 3), theta0=o.theta(), pad_positions=o.pad_positions())


def execute_fixture():
    out = {}
    for dof in (7, 14):
        p = pb.make_problem(dof=dof, grid_n=64, num_rollouts=10, num_reused_rollouts=0)
        o = po.Oracle(p)
        rng = np.random.default_rng(dof)
        th = o.theta()
        params = np.stack([th + s * rng.standard_normal(th.shape) for s in (0.0, 0.05, 0.3, 1.5)])
        costs, cfs, trajs = [], [], []
        for prm in params:
            c, cf, tr = o.execute(prm, 1)
            costs.append(c)
            cfs.append(cf)
            trajs.append(tr)
        out[f"params_{dof}"] = params
        out[f"costs_{dof}"] = np.stack(costs)
        out[f"cf_{dof}"] = np.array(cfs)
        out[f"traj_{dof}"] = np.stack(trajs)
    save("execute_cases", **out)


def iterate_fixture():
    # cfg1 shape with the params.yaml ratio: 10 rollouts, 5 reused, 128^3 grid
    p = pb.make_problem(grid_n=128, num_rollouts=10, num_reused_rollouts=5)
    o = po.Oracle(p)
    costs, cfs, thetas = [], [], []
    for it in range(1, 11):
        c, cf = o.iterate(it)
        costs.append(c)
        cfs.append(cf)
        thetas.append(o.theta())
    save("cfg1_iterate_10_5", costs=np.array(costs), cf=np.array(cfs), theta=np.stack(thetas),
         state_costs=o.rollouts("state_costs"), probabilities=o.rollouts("probabilities"))


def optimize_fixture():
    # cfg1: K = 20, K_r = 10, 128^3 grid, 100 iterations of StompOptimizer::optimize
    p = pb.make_problem(grid_n=128, num_rollouts=20, num_reused_rollouts=10, max_iterations=100)
    o = po.Oracle(p)
    st, costs = o.optimize()
    save("cfg1_optimize_20_10", costs=costs, best=o.best_trajectory(), last=o.last_trajectory(),
         stats=np.array([st.iterations, st.success, st.success_iteration, st.collision_success_iteration,
                         st.last_improvement_iteration]), best_cost=np.array([st.best_cost]))


def terms_fixture():
    # torque term (launch/stomp_motion_planner_torques.launch:12 weight) + the upright path
    # constraint of test/test_omp.cpp:76-91, params.yaml 10 / 5 rollouts
    p = pb.make_problem(grid_n=64, num_rollouts=10, num_reused_rollouts=5, torque_cost_weight=0.001,
                        orientation_constraints=[pb.upright_constraint()])
    o = po.Oracle(p)
    rng = np.random.default_rng(21)
    th = o.theta()
    params = np.stack([th + s * rng.standard_normal(th.shape) for s in (0.0, 0.05, 0.3)] + [th.copy()])
    params[3, 4] += np.pi
    costs, cfs, css = [], [], []
    for prm in params:
        c, cf, _ = o.execute(prm, 1)
        costs.append(c)
        cfs.append(cf)
        css.append(o.last_constraints_satisfied)
    it_costs, it_cs, thetas = [], [], []
    for it in range(1, 6):
        c, _ = o.iterate(it)
        it_costs.append(c)
        it_cs.append(o.last_constraints_satisfied)
        thetas.append(o.theta())
    save("terms_cases", params=params, costs=np.stack(costs), cf=np.array(cfs), cs=np.array(css),
         it_costs=np.array(it_costs), it_cs=np.array(it_cs), theta=np.stack(thetas))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    math_kats()
    setup_fixture()
    execute_fixture()
    iterate_fixture()
    optimize_fixture()
    terms_fixture()
