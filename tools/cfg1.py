"""cfg1 (BASELINE.json configs[0], the ICRA CPU case): 7-DOF, 100 wp, K = 20 rollouts with 10
reused, 128^3 SDF.  Times the CPU oracle (1 thread in reference structure, and
banded over all granted cores) and the HIP engine on the same problem, and prints one JSON line.

Usage on a GPU box: python3 tools/cfg1.py [--iterations 500]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from stomp_motion_planner_icra2011_amd import engine as eng   # noqa: E402
from stomp_motion_planner_icra2011_amd import problem as pb   # noqa: E402
from oracle import pyoracle as po                             # noqa: E402  (checker / CPU baseline only)


def time_iterations(obj, n):
    t0 = time.perf_counter()
    for it in range(1, n + 1):
        obj.iterate(it)
    return n / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=500)
    args = ap.parse_args()
    n = args.iterations
    p = pb.make_problem(dof=7, waypoints=100, grid_n=128, num_rollouts=20, num_reused_rollouts=10)
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    cpu1 = time_iterations(po.Oracle(p, dense=True, threads=1), n)
    cpun = time_iterations(po.Oracle(p, dense=False, threads=threads), n)

    e = eng.Engine(p)
    e.run(1, 20)
    e.synchronize()
    e2 = eng.Engine(p)
    t0 = time.perf_counter()
    e2.run(1, n)
    e2.synchronize()
    gpu_run = n / (time.perf_counter() - t0)
    e3 = eng.Engine(p)
    gpu_iter = time_iterations(e3, n)   # one host read-back per iteration, as runSingleIteration
    # the final trajectories agree bit for bit (the same contract the parity tests assert)
    o = po.Oracle(p, threads=threads)
    for it in range(1, n + 1):
        o.iterate(it)
    same = bool((o.theta() == e2.theta()).all() and (o.theta() == e3.theta()).all())
    print(json.dumps({
        "config": "cfg1: 7-DOF, 100 wp (N=99), K=20 (K_r=10), 128^3 SDF",
        "iterations": n,
        "cpu_1thread_reference_structure_its": round(cpu1, 2),
        "cpu_banded_its": round(cpun, 2), "cpu_threads": threads,
        "gpu_run_its": round(gpu_run, 1),
        "gpu_iterate_its": round(gpu_iter, 1),
        "theta_bitwise_equal_to_oracle": same,
    }))
    for x in (e, e2, e3):
        x.close()


if __name__ == "__main__":
    main()
