#!/usr/bin/env python3
"""STOMP iterations/sec on MI355X (BASELINE.json metric), one JSON line on rank 0.

Workload (BASELINE.json configs[1], "cfg2"): 7-DOF PR2-like arm, 100 waypoints
(N = 99 free), K = 512 noisy rollouts per GPU, no reuse, 256^3 fp32 distance
field of the shelf + pole scene, built on the device.  A step is one
PolicyImprovementLoop::runSingleIteration equivalent (noise, projection, control
costs, K rollout executions, probability weighting, update, noiseless rollout),
enqueued by stomp_engine_run with inputs already resident in HBM.  With --gpus N
the K dimension is sharded (K = 512 N, weak scaling) and the per-iteration
reductions run over RCCL inside the engine.

Also reported:
  roofline      dominant stage (rollout_cost = fused k_rollout: noise generation + Task::execute):
                algorithmic bytes per launch K_loc N (4 S + 24 J + 8) + N (4 S + 8 J + 8) over its
                HIP-event duration, from a second pass of the same K steps with events (the value
                pass has none)
  cpu_baseline  the CPU oracle (oracle/, reference-structure dense products, 1 thread)
                timed on this host on a bounded sample of the same workload
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "STOMP iterations/sec (7-DOF, 100 wp, K=512, 256³ SDF) at 1/2/4/8 GPUs"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rollouts-per-gpu", type=int, default=512)
    ap.add_argument("--waypoints", type=int, default=100)
    ap.add_argument("--dof", type=int, default=7)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event pass (no roofline)")
    ap.add_argument("--problems", type=int, default=1,
                    help="independent planning problems per GPU, one engine and stream each (cfg5 mode)")
    ap.add_argument("--optimize-steps", type=int, default=200,
                    help="also time StompOptimizer::optimize (device-resident loop) for this many iterations (0 = skip)")
    return ap.parse_args()


def latest_traffic():
    """HBM bytes per rollout_cost launch from the newest committed rocprofv3 PMC summary, if any."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*rollout_cost_traffic*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline_all_cores(problem, budget_s: float):
    """SURVEY.md 8(d)'s stronger CPU baseline: the oracle with banded stencils and Task::execute
    spread over the host cores this process may use (OpenMP over rollouts)."""
    from oracle import pyoracle as po
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    o = po.Oracle(problem, dense=False, threads=threads)
    t0 = time.perf_counter()
    n = 0
    while True:
        o.iterate(n + 1)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 400:
            break
    return {"value": n / el, "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": f"first {n} iterations of the same workload on the CPU oracle with banded stencils and "
                      f"OpenMP over the rollouts' Task::execute, {threads} threads, {el:.1f} s"}


def cfg_name(args, world: int) -> str:
    """The BASELINE.json config a run's shape matches, or "custom"."""
    shape = (args.dof, args.waypoints, args.rollouts_per_gpu * world, args.grid, args.problems)
    if shape == (7, 100, 512, 256, 1):
        return "cfg2"
    if (args.dof, args.waypoints, args.grid, args.problems) == (7, 200, 256, 1):
        return "cfg3" if args.rollouts_per_gpu * world == 4096 else "cfg3-shape"
    if (args.dof, args.waypoints, args.rollouts_per_gpu * world, args.grid, args.problems) == (14, 100, 1024, 512, 1):
        return "cfg4"
    if (args.dof, args.waypoints, args.rollouts_per_gpu, args.grid) == (7, 100, 128, 256) and args.problems > 1:
        return "cfg5"
    return "custom"


def cpu_baseline(problem, budget_s: float):
    from oracle import pyoracle as po
    o = po.Oracle(problem, dense=True, threads=1)
    t0 = time.perf_counter()
    n = 0
    while True:
        o.iterate(n + 1)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 200:
            break
    return {"value": n / el, "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": f"first {n} iterations of the same workload (K={problem.params.num_rollouts}, N={problem.N}, "
                      f"J={problem.J}, {problem.grid.n}^3 SDF) on the CPU oracle in reference structure "
                      f"(dense N x N products, sequential Task::execute), 1 thread, {el:.1f} s"}


def bench_problems(args, world, rank, local_rank, dist):
    """cfg5: independent planning problems per GPU (distinct start / goal / seed, one shared
    device-built SDF), one engine and one stream each, no communication (replicas); each
    engine's steps are enqueued as one run and the streams run concurrently.  value =
    problem-iterations per second over all ranks."""
    from stomp_motion_planner_icra2011_amd import engine as eng
    from stomp_motion_planner_icra2011_amd import problem as pb
    P = args.problems
    rng = np.random.default_rng(1234 + rank)
    base = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=args.rollouts_per_gpu,
                           num_reused_rollouts=0, build_grid=False)
    sdf = eng.DeviceBuffer(4 * args.grid ** 3, device=local_rank)
    eng.sdf_build_device(base, sdf.ptr)
    engines = []
    for i in range(P):
        d = rng.uniform(-0.15, 0.15, (2, base.J))
        p = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid,
                            num_rollouts=args.rollouts_per_gpu, num_reused_rollouts=0, build_grid=False,
                            seed=base.seed + 1 + rank * P + i, start=list(base.start + d[0]), goal=list(base.goal + d[1]),
                            max_iterations=args.warmup + args.steps + 1)
        engines.append(eng.Engine(p, device=local_rank, sdf_device_ptr=sdf.ptr))

    def sweep(first, count):
        # each problem's iterations as one stomp_engine_run (its noiseless rollouts ride in the
        # next rollout launch; a run of one iteration would flush each as its own launch); the
        # problems' streams overlap on the device while the host enqueues the next problem
        for e in engines:
            e.run(first, count)
        for e in engines:
            e.synchronize()

    sweep(1, args.warmup)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    sweep(args.warmup + 1, args.steps)
    elapsed = time.perf_counter() - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = P * world * args.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "STOMP problem-iterations/sec (64-problem batch, cfg5)", "value": round(value, 3),
            "unit": "problem-iterations/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (PR2-like arm, shelf+pole scene, device-built SDF; Philox noise)",
            "config": {"workload": f"{cfg_name(args, world)}: {P} problems/GPU x {world} GPU, {args.dof}-DOF, {args.waypoints} wp, "
                                   f"K={args.rollouts_per_gpu} each, {args.grid}^3 SDF shared",
                       "problems_per_gpu": P, "parallelism": f"replicas x{world}, one stream per problem",
                       "rollouts_per_s": round(value * args.rollouts_per_gpu, 1)}}))
    for e in engines:
        e.close()
    sdf.free()


def main():
    args = parse()
    if args.problems > 1:
        # one stream per problem: give HIP as many hardware queues as it needs to run them side by
        # side (its default, 4, puts several problems' launches in one in-order queue; measured
        # 24.9k -> 36.4k problem-iterations/s at 8 problems).  Set before the runtime initialises.
        want = min(32, max(4, 2 * args.problems))
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < want:
            os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist  # CPU rendezvous only: the data path is RCCL inside the engine
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from stomp_motion_planner_icra2011_amd import engine as eng
    from stomp_motion_planner_icra2011_amd import problem as pb

    if args.problems > 1:
        bench_problems(args, world, rank, local_rank, dist)
        if dist:
            dist.destroy_process_group()
        return

    K = args.rollouts_per_gpu * world
    p = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=K,
                        num_reused_rollouts=0, build_grid=False, max_iterations=args.warmup + 2 * args.steps + 1)
    sdf = eng.DeviceBuffer(4 * args.grid ** 3, device=local_rank)
    eng.sdf_build_device(p, sdf.ptr)
    comm_id = None
    if world > 1:
        obj = [eng.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    e = eng.Engine(p, device=local_rank, sdf_device_ptr=sdf.ptr, rank=rank, world_size=world, comm_id=comm_id)

    # warmup
    e.run(1, args.warmup)
    e.synchronize()
    if dist:
        dist.barrier()
    e.synchronize()
    t0 = time.perf_counter()
    e.run(args.warmup + 1, args.steps)
    e.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    global_its = args.steps / elapsed
    # The metric's unit is a K = 512 iteration (BASELINE.json).  With K = 512 per GPU the N-GPU
    # run does one K = 512 N iteration per step, i.e. N units of the metric's work, so the
    # whole-job aggregate is N x the global iteration rate (at N = 1 the two are the same).
    value = global_its * world

    # Kernel durations: the same K steps again with HIP events recorded around every stage
    # on the engine stream.  The events themselves cost ~10 us of dispatch gap per stage,
    # which is why `value` comes from the event-free pass above.
    timing = {}
    if not args.no_timing:
        e.set_timing(True)
        e.run(args.warmup + args.steps + 1, args.steps)
        e.synchronize()
        for name in ("noise", "pregen", "rollout_cost", "weights", "update", "noiseless", "all"):
            tot, n = e.timing(name)
            timing[name] = {"total_ms": tot, "launches": n, "avg_us": 1000.0 * tot / max(n, 1)}
        e.set_timing(False)

    S = len(p.spheres)
    K_loc = e.K_loc
    # each launch generates and evaluates K_loc noisy rollouts (noise, params and control rows
    # written: 24 J N bytes; SDF gathers 4 S N; state costs 8 N) and evaluates the deferred
    # noiseless rollout of theta (reads 8 J N)
    bytes_per_launch = K_loc * p.N * (4 * S + 24 * p.J + 8) + p.N * (4 * S + 8 * p.J + 8)
    roofline = None
    if timing.get("rollout_cost", {}).get("launches"):
        avg_s = timing["rollout_cost"]["avg_us"] * 1e-6
        achieved = bytes_per_launch / avg_s / 1e9
        roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4),
                    # the committed PMC summary is of the default workload (cfg2, one GPU)
                    "traffic": latest_traffic() if cfg_name(args, world) == "cfg2" else None,
                    "kernel": "rollout_cost (k_rollout)", "bytes_per_launch": bytes_per_launch,
                    "avg_launch_us": round(timing["rollout_cost"]["avg_us"], 3)}
    if roofline is not None:
        # whole iteration, B_iter = E * N * (4 S + 16 J + 8), E = K + 1, all ranks
        b_iter = (K + 1) * p.N * (4 * S + 16 * p.J + 8)
        roofline["iteration_bytes"] = b_iter
        roofline["iteration_frac"] = round(b_iter * global_its / (HBM_PEAK_GBS * 1e9 * world), 5)   # vs N x peak

    # StompOptimizer::optimize (stomp_optimizer.cpp:249-401) through the device-resident loop:
    # the same iterations with the optimizer's bookkeeping, no early stop
    optimize = None
    if args.optimize_steps > 0:
        po_ = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=K,
                              num_reused_rollouts=0, build_grid=False, max_iterations=args.optimize_steps,
                              max_iterations_after_collision_free=args.optimize_steps + 1)
        eo = eng.Engine(po_, device=local_rank, sdf_device_ptr=sdf.ptr, rank=rank, world_size=world, comm_id=comm_id) \
            if world == 1 else None
        if eo is not None:
            eo.optimize()   # warm
            t0 = time.perf_counter()
            st, _ = eo.optimize()
            dt = time.perf_counter() - t0
            optimize = {"iterations": st.iterations, "iterations_per_s": round(st.iterations / dt, 3)}
            eo.close()

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        pc = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=K,
                             num_reused_rollouts=0)
        cpu = cpu_baseline(pc, args.cpu_seconds)
        cpu_mt = cpu_baseline_all_cores(pc, min(args.cpu_seconds, 8.0))

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "iterations/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (PR2-like arm, shelf+pole scene, device-built SDF; Philox noise)",
            "config": {"workload": f"{cfg_name(args, world)}: {args.dof}-DOF, {args.waypoints} wp (N={p.N}), K={args.rollouts_per_gpu}/GPU "
                                   f"(K={K} total), K_r=0, {args.grid}^3 SDF, S={S} spheres",
                       "rollouts_per_gpu": args.rollouts_per_gpu, "global_rollouts": K,
                       "parallelism": f"rollout shard x{world}" + (" (RCCL)" if world > 1 else ""),
                       "global_iterations_per_s": round(global_its, 3),
                       "value_unit": f"iterations of K={args.rollouts_per_gpu} per second, summed over GPUs "
                                     f"(= global K={K} iterations/s x {world})",
                       "rollouts_per_s": round(global_its * K, 1)},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_mt,
            "kernel_timing_us": {k: round(v["avg_us"], 3) for k, v in timing.items()},
            "optimize_loop": optimize,
        }
        print(json.dumps(out))
    e.close()
    sdf.free()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
