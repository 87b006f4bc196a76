#!/usr/bin/env python3
"""STOMP iterations/sec on MI355X (BASELINE.json metric), one JSON line on rank 0.

Workloads (BASELINE.json configs; --workload, default cfg2 = configs[1], the metric's own):
  cfg2  7-DOF PR2-like arm, 100 waypoints (N = 99 free), K = 512 rollouts, no reuse, 256^3
        fp32 distance field of the shelf + pole scene built on the device
  cfg3  7-DOF, 200 waypoints (N = 199), K = 4096, 256^3
  cfg4  14-DOF two-arm tree, 100 waypoints, K = 1024, 512^3 (the HBM-bound field)
  cfg5  64 independent problems (7-DOF, 100 wp, K = 128 each, distinct start / goal / seed),
        64 / N problems per GPU, no communication; a GPU's problems form one engine group
        (stomp_group_run: one rollout, weights and update launch per iteration for all of them;
        --group 0 = one engine and stream per problem)
A step is one PolicyImprovementLoop::runSingleIteration equivalent (noise, projection, control
costs, K rollout executions, probability weighting, update, noiseless rollout), enqueued by
stomp_engine_run with inputs already resident in HBM.  With --gpus N the K rollouts of the
workload are sharded over the N ranks (K / N per GPU, STRONG scaling: the global iteration is the
unit of the metric at every N) and the per-iteration exchanges run over RCCL inside the engine;
value = global iterations per second.  cfg5 runs replicas (problems split over the ranks).

Also reported:
  roofline      the dominant kernel k_rollout (noise phase + Task::execute of the K_loc noisy
                rollouts and the deferred noiseless one): achieved = SURVEY.md 8(d) algorithmic
                bytes per unit (4 S + 16 J + 8) x (K_loc + 1) N units / its HIP-event average
                duration (second pass of the same K steps with events; the value pass has none);
                traffic = HBM bytes per launch from the committed rocprofv3 PMC summary of
                this very build (matched by the engine's source hash; null otherwise);
  valu          the same kernel's VALU issue fraction: SQ_INSTS_VALU (that PMC summary) x 4
                cycles / 1024 SIMDs / (the event-measured duration x 2.4 GHz)
  cpu_baseline  the CPU oracle (oracle/, reference-structure dense products, 1 thread) timed on
                this host on a bounded sample of the same workload; cpu_baseline_all_cores the
                banded oracle over the CPU share this job is granted (the cgroup quota when one is
                set, else OMP_NUM_THREADS, else the affinity mask), all three counts reported
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
VALU_CLOCK_HZ = 2.4e9  # MI355X peak engine clock; 256 CUs x 4 SIMDs, a wave64 VALU op issues in 4 cycles
METRIC = "STOMP iterations/sec (7-DOF, 100 wp, K=512, 256³ SDF) at 1/2/4/8 GPUs"

# BASELINE.json configs[0..4] (configs[0], cfg1, is the reference's own CPU case: K = 20 with
# 10 reused rollouts)
WORKLOADS = {
    "cfg1": dict(dof=7, waypoints=100, rollouts=20, grid=128, problems=1, reused=10),
    "cfg2": dict(dof=7, waypoints=100, rollouts=512, grid=256, problems=1, reused=0),
    "cfg3": dict(dof=7, waypoints=200, rollouts=4096, grid=256, problems=1, reused=0),
    "cfg4": dict(dof=14, waypoints=100, rollouts=1024, grid=512, problems=1, reused=0),
    "cfg5": dict(dof=7, waypoints=100, rollouts=128, grid=256, problems=64, reused=0),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg2")
    ap.add_argument("--rollouts", type=int, default=None, help="K of the whole job (default: the workload's)")
    ap.add_argument("--waypoints", type=int, default=None)
    ap.add_argument("--dof", type=int, default=None)
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--problems", type=int, default=None, help="cfg5: problems of the whole job")
    ap.add_argument("--reused", type=int, default=None, help="K_r, reused rollouts (cfg1: 10)")
    ap.add_argument("--enqueue-threads", type=int, default=1, help="cfg5: host threads enqueueing the problems")
    ap.add_argument("--group", type=int, default=-1,
                    help="cfg5: problems per engine group (shared launches; -1 = all of a GPU's problems, "
                         "0 = one stream per problem)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event pass (no roofline)")
    ap.add_argument("--optimize-steps", type=int, default=200,
                    help="also time StompOptimizer::optimize (device-resident loop) for this many iterations (0 = skip)")
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    for k, v in w.items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.custom = any(getattr(a, k) != v for k, v in w.items())
    return a


def workload_name(args) -> str:
    return args.workload + (" (modified)" if args.custom else "")


def loaded_hash() -> str:
    """the source hash compiled into the engine library this process loaded (stomp_engine_source_hash):
    the build that was timed, which a PMC summary must match"""
    from stomp_motion_planner_icra2011_amd import engine as eng
    return eng.load_library().stomp_engine_source_hash().decode()


def pmc_summary(workload: str = "cfg2"):
    """The newest committed rocprofv3 PMC summary (tools/pmc_traffic.py) of this workload on one
    GPU and whether it was taken of this build (the engine's source hash).  Returns (summary or
    None, provenance dict)."""
    here = loaded_hash()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*rollout_cost_traffic*.json"), recursive=True),
                   key=os.path.getmtime)
    newest = None
    for path in reversed(files):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("workload", "cfg2") != workload:
            continue
        rel = os.path.relpath(path, os.path.join(ROOT, "profiles"))
        if newest is None:
            newest = (rel, d.get("source_hash"))
        if d.get("source_hash") == here:
            return d, {"file": rel, "workload": workload, "source_hash": here, "loaded_library_hash": here,
                       "matches_build": True}
    return None, {"file": newest[0] if newest else None, "workload": workload,
                  "source_hash": newest[1] if newest else None, "loaded_library_hash": here, "matches_build": False,
                  "note": "no PMC pass of this build and workload is committed: traffic and VALU counts are null"}


def pmc_fields(pmc, prov, avg_s):
    """traffic (HBM bytes per launch of the dominant kernel) and its VALU issue, from a PMC summary"""
    insts = pmc.get("valu_insts_per_launch") if pmc else None
    stage = ((pmc.get("kernels") or {}).get(pmc.get("stage")) or {}) if pmc else {}
    return {"traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
            # the same kernel's average duration in the rocprofv3 kernel trace of this build
            "rocprof_avg_ns": stage.get("avg_ns"),
            "traffic_uncorrected": pmc.get("hbm_bytes_per_launch_uncorrected") if pmc else None,
            "traffic_source": prov,
            "valu": {"insts_per_launch": insts,
                     "issue_cycles_per_simd": round(insts * 4.0 / 1024, 1) if insts else None,
                     "frac_valu_issue": round(insts * 4.0 / 1024 / (avg_s * VALU_CLOCK_HZ), 4) if insts else None,
                     "clock_ghz": VALU_CLOCK_HZ / 1e9, "simds": 1024, "source": prov}}


def roofline_bound(traffic, avg_s, valu):
    """The bound that binds, from the evidence of this build (the PMC summary): "latency" when
    neither the VALU issue fraction nor the measured HBM bandwidth is near its peak (the launch
    waits on dependent chains), "hbm" when the measured bytes approach the HBM peak, "valu" when
    the issue fraction does; "hbm" (the roofline it is priced against) without a summary."""
    frac_valu = (valu or {}).get("frac_valu_issue")
    if traffic is None or frac_valu is None:
        return "hbm", None
    hbm = traffic / avg_s / 1e9 / HBM_PEAK_GBS
    if hbm >= 0.6:
        return "hbm", hbm
    if frac_valu >= 0.6:
        return "valu", hbm
    return "latency", hbm


def rocprof_fields(pf, bytes_per_launch):
    """frac from the rocprofv3 kernel-trace average of the same build beside the event-based one"""
    ns = pf.get("rocprof_avg_ns")
    if not ns:
        return {"rocprof_avg_launch_us": None, "frac_rocprof": None}
    return {"rocprof_avg_launch_us": round(ns / 1000.0, 3),
            "frac_rocprof": round(bytes_per_launch / (ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 5)}


def cpu_share():
    """CPUs this job may use: the cgroup quota (v2 cpu.max or v1 cfs quota) when one is set."""
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    return quota


def host_info():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"nproc": os.cpu_count(), "sched_affinity": avail, "cgroup_cpu_quota": cpu_share(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "model": model}


def cpu_baseline(problem, budget_s: float):
    """SURVEY.md 8(d) CPU baseline: the oracle in reference structure (dense N x N products,
    sequential per-rollout Task::execute), 1 thread, bounded sample of the same workload."""
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
    return {"value": n / el, "unit": "iterations/s", "cores": 1, "kind": "port", "host": host_info(),
            "sample": f"first {n} iterations of the same workload (K={problem.params.num_rollouts}, N={problem.N}, "
                      f"J={problem.J}, {problem.grid.n}^3 SDF) on the CPU oracle in reference structure "
                      f"(dense N x N products, sequential Task::execute), 1 thread, {el:.1f} s"}


def cpu_baseline_all_cores(problem, budget_s: float):
    """SURVEY.md 8(d)'s stronger CPU baseline: the oracle with banded stencils and Task::execute
    spread over the host cores this job is granted (OpenMP over rollouts).  The GPU box's
    affinity mask shows the whole machine, but a one-GPU job's CPU share is a fraction of it
    (the harness sets OMP_NUM_THREADS to it); threads past the share only time-slice."""
    from oracle import pyoracle as po
    h = host_info()
    quota = h["cgroup_cpu_quota"]
    if quota:
        threads, basis = max(1, int(quota)), "cgroup CPU quota"
    elif os.environ.get("OMP_NUM_THREADS"):
        threads, basis = int(os.environ["OMP_NUM_THREADS"]), "OMP_NUM_THREADS (the job's CPU share)"
    else:
        threads, basis = int(h["sched_affinity"] or 1), "affinity mask"
    threads = min(threads, int(h["sched_affinity"] or threads))

    def timed(nthreads):
        o = po.Oracle(problem, dense=False, threads=nthreads)
        t0 = time.perf_counter()
        n = 0
        while True:
            o.iterate(n + 1)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget_s or n >= 400:
                return n, el

    n, el = timed(threads)
    # also at every CPU of the affinity mask (SURVEY 8(d) says all host cores): reported beside
    # the quota run, and the baseline when it is faster
    aff = int(h["sched_affinity"] or threads)
    at_aff = None
    if aff > threads:
        na, ela = timed(aff)
        at_aff = {"threads": aff, "value": na / ela, "iterations": na, "seconds": round(ela, 2)}
        if na / ela > n / el:
            n, el, threads, basis = na, ela, aff, "affinity mask (faster than the cgroup quota's threads)"
    return {"value": n / el, "unit": "iterations/s", "cores": threads, "cores_basis": basis,
            "affinity_cores": h["sched_affinity"], "at_affinity_count": at_aff, "kind": "port", "host": h,
            "sample": f"first {n} iterations of the same workload on the CPU oracle with banded stencils and "
                      f"OpenMP over the rollouts' Task::execute, {threads} threads ({basis}; affinity mask "
                      f"{h['sched_affinity']} CPUs), {el:.1f} s"}


def shard_why(e) -> str:
    """why the engine chose its K-sharded decomposition (measured at creation, maxima over ranks)"""
    i = e.shard_info
    if not i:
        if os.environ.get("STOMP_SHARD_MODE"):
            return ": requested by STOMP_SHARD_MODE"
        return ": the only decomposition this shape allows (not measured)"
    g = i["t_gather"] + i["l_allgather_state"]
    p = i["t_partials"] + i["l_allreduce"] + 2 * i["l_allgather_partials"]
    return (f": measured gather {i['t_gather']:.1f} + all-gather {i['l_allgather_state']:.1f} = {g:.1f} us vs "
            f"partials {i['t_partials']:.1f} + 3 collectives {p - i['t_partials']:.1f} = {p:.1f} us")


def max_over_ranks(dist, x: float) -> float:
    if not dist:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_problems(args, world, rank, local_rank, dist):
    """cfg5: the batch of independent planning problems split over the ranks (replicas, no
    communication), distinct start / goal / seed, one shared device-built SDF per GPU, one engine
    and one stream each; each engine's steps are enqueued as one run and the streams run
    concurrently.  value = problem-iterations per second over all ranks."""
    from stomp_motion_planner_icra2011_amd import engine as eng
    from stomp_motion_planner_icra2011_amd import problem as pb
    P_all = args.problems
    per = [P_all // world + (1 if r < P_all % world else 0) for r in range(world)]
    P, first_id = per[rank], sum(per[:rank])
    rng = np.random.default_rng(1234)
    base = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=args.rollouts,
                           num_reused_rollouts=0, build_grid=False)
    sdf = eng.DeviceBuffer(2 * args.grid ** 3, device=local_rank)   # uint16 d2 per voxel
    eng.sdf_build_device(base, sdf.ptr)
    gsize = P if args.group < 0 else args.group
    streams = [eng.Stream(local_rank) for _ in range((P + gsize - 1) // gsize)] if gsize else []
    engines = []
    offsets = rng.uniform(-0.15, 0.15, (P_all, 2, base.J))
    for i in range(first_id, first_id + P):
        d = offsets[i]
        p = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid,
                            num_rollouts=args.rollouts, num_reused_rollouts=0, build_grid=False,
                            seed=base.seed + 1 + i, start=list(base.start + d[0]), goal=list(base.goal + d[1]),
                            max_iterations=args.warmup + 2 * args.steps + 1)
        k = i - first_id
        engines.append(eng.Engine(p, device=local_rank, sdf_device_ptr=sdf.ptr,
                                  stream=streams[k // gsize].ptr if gsize else None))
    # --group G: the problems in groups of G engines on one stream each, every group advanced by
    # shared launches (stomp_group_run: three dispatches per iteration for the whole group)
    groups = [eng.EngineGroup(engines[k:k + gsize]) for k in range(0, P, gsize)] if gsize else []

    threads = max(1, min(args.enqueue_threads, len(engines)))
    pool = None
    if threads > 1:
        import concurrent.futures as cf
        pool = cf.ThreadPoolExecutor(threads)

    def sweep(first, count):
        # each problem's iterations as one stomp_engine_run (its noiseless rollouts ride in the
        # next rollout launch; a run of one iteration would flush each as its own launch); the
        # problems' streams overlap on the device while the host enqueues the next problem.
        # Enqueueing is the limit at several problems per GPU (three launches per problem-
        # iteration), so host threads share it: distinct engines may be driven concurrently
        # (stomp_engine.h), and the ctypes calls release the GIL
        if groups:
            for g in groups:
                g.run(first, count)
            for g in groups:
                g.synchronize()
            return
        if pool is None:
            for e in engines:
                e.run(first, count)
        else:
            def part(k):
                for e in engines[k::threads]:
                    e.run(first, count)
            list(pool.map(part, range(threads)))
        for e in engines:
            e.synchronize()

    sweep(1, args.warmup)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    sweep(args.warmup + 1, args.steps)
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, elapsed)
    value = P_all * args.steps / elapsed

    # the roofline of the dominant kernel, the grouped rollout launch (every engine of a group:
    # k_rollout_group), timed with HIP events on the group's stream in a second pass of the same
    # steps (stomp_group_run records its launches on its first engine's timers)
    roofline = None
    timing = {}
    if groups and not args.no_timing:
        e0 = groups[0].engines[0]
        e0.set_timing(True)
        sweep(args.warmup + args.steps + 1, args.steps)
        for name in ("rollout_cost", "weights", "update"):
            tot, n = e0.timing(name)
            timing[name] = 1000.0 * tot / max(n, 1)
        e0.set_timing(False)
        S = len(base.spheres)
        unit_bytes = 4 * S + 16 * base.J + 8
        per_launch = len(groups[0].engines) * (args.rollouts + 1) * base.N   # (rollout, waypoint) units
        avg_s = timing["rollout_cost"] * 1e-6
        achieved = per_launch * unit_bytes / avg_s / 1e9
        pmc, prov = pmc_summary("cfg5") if (world == 1 and not args.custom) else \
            (None, {"note": "PMC summaries are of the BASELINE workloads on one GPU"})
        pf = pmc_fields(pmc, prov, avg_s)
        bound, hbm_meas = roofline_bound(pf["traffic"], avg_s, pf["valu"])
        roofline = {"bound": bound, "priced_against": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pf["traffic"],
                    "traffic_uncorrected": pf["traffic_uncorrected"], "traffic_source": prov,
                    "hbm_frac_measured": round(hbm_meas, 5) if hbm_meas is not None else None,
                    **rocprof_fields(pf, per_launch * unit_bytes),
                    "kernel": "k_rollout_group", "unit_bytes": unit_bytes, "units_per_launch": per_launch,
                    "bytes_per_launch": per_launch * unit_bytes, "avg_launch_us": round(timing["rollout_cost"], 3),
                    "sdf_only_gbs": round(per_launch * 4 * S / avg_s / 1e9, 2),
                    "unit_bytes_actual": 2 * S + 16 * base.J + 8,
                    "iteration_bytes": P_all * (args.rollouts + 1) * base.N * unit_bytes,
                    "iteration_frac": round(P_all * (args.rollouts + 1) * base.N * unit_bytes * value / P_all /
                                            (HBM_PEAK_GBS * 1e9 * world), 5),
                    "valu": pf["valu"]}
    if rank == 0:
        print(json.dumps({
            "metric": "STOMP problem-iterations/sec (64-problem batch, cfg5)", "value": round(value, 3),
            "unit": "problem-iterations/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 5), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (PR2-like arm, shelf+pole scene, device-built SDF; Philox noise)",
            "config": {"workload": f"{workload_name(args)}: {P_all} problems over {world} GPU ({max(per)} per GPU), "
                                   f"{args.dof}-DOF, {args.waypoints} wp, K={args.rollouts} each, "
                                   f"{args.grid}^3 SDF shared per GPU",
                       "problems": P_all, "parallelism": f"replicas x{world}, " + (f"groups of {gsize} problems (shared launches)" if gsize else "one stream per problem"),
                       "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "enqueue_threads": threads, "group": gsize,
                       "rollouts_per_s": round(value * args.rollouts, 1)},
            "roofline": roofline,
            "kernel_timing_us": {k: round(v, 3) for k, v in timing.items()}}))
    for g in groups:
        g.close()
    for e in engines:
        e.close()
    for st in streams:
        st.close()
    sdf.free()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # STOMP_BENCH_DEVICE: every rank on this device (a multi-rank rehearsal on a one-GPU box)
    local_rank = int(os.environ.get("STOMP_BENCH_DEVICE", local_rank))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    if args.workload == "cfg5":
        # one stream per problem: give HIP as many hardware queues as it can use to run them
        # side by side (its default, 4, puts several problems' launches in one in-order queue;
        # measured 24.9k -> 36.4k problem-iterations/s at 8 problems).  Set before the runtime
        # initialises.
        per_gpu = (args.problems + world - 1) // world
        want = min(32, max(4, 2 * per_gpu))
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < want:
            os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    dist = None
    if world > 1:
        # a stuck or mismatched collective fails the run within a minute (the engine's bounded wait
        # aborts the communicator and names the collective) instead of hanging it
        os.environ.setdefault("STOMP_COMM_TIMEOUT_S", "60")
        import torch.distributed as dist  # CPU rendezvous only: the data path is RCCL inside the engine
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from stomp_motion_planner_icra2011_amd import engine as eng
    from stomp_motion_planner_icra2011_amd import problem as pb

    if args.workload == "cfg5":
        bench_problems(args, world, rank, local_rank, dist)
        if dist:
            dist.destroy_process_group()
        return

    K = args.rollouts
    if world > 1 and K % (64 * world) != 0:
        raise SystemExit(f"K={K} must split into whole 64-rollout blocks over {world} GPUs")
    p = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=K,
                        num_reused_rollouts=args.reused, build_grid=False,
                        max_iterations=args.warmup + 2 * args.steps + 1)
    sdf = eng.DeviceBuffer(2 * args.grid ** 3, device=local_rank)   # uint16 d2 per voxel
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
    elapsed = max_over_ranks(dist, t1 - t0)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = args.steps / elapsed   # global iterations (of the whole K) per second

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
    # per (rollout, waypoint) unit, one fp32 SDF voxel per sphere (4 S; SURVEY's
    # figure, kept for comparison across rounds: this field's voxel is 2 bytes), the
    # write + read of the fp64 noise per joint (16 J) and the fp64 state cost (8); one k_rollout
    # launch executes the K_loc noisy rollouts of this rank and the deferred noiseless one
    unit_bytes = 4 * S + 16 * p.J + 8
    # with K_r reused rollouts the launch evaluates only the generated ones (and the noiseless)
    rows_launch = (K_loc - args.reused if world == 1 else K_loc) + 1
    bytes_per_launch = rows_launch * p.N * unit_bytes
    # the same launch counting every row it writes (noise, params, control: 24 J) and the
    # noiseless rollout's params read (8 J) instead of 16 J
    bytes_written_rows = (rows_launch - 1) * p.N * (4 * S + 24 * p.J + 8) + p.N * (4 * S + 8 * p.J + 8)
    roofline = None
    if timing.get("rollout_cost", {}).get("launches"):
        avg_s = timing["rollout_cost"]["avg_us"] * 1e-6
        achieved = bytes_per_launch / avg_s / 1e9
        headline = args.workload == "cfg2" and not args.custom and world == 1
        one_gpu = not args.custom and world == 1
        pmc, prov = pmc_summary(args.workload) if one_gpu else \
            (None, {"note": "PMC summaries are of the BASELINE workloads on one GPU"})
        pf = pmc_fields(pmc, prov, avg_s)
        # bound: what the evidence says binds (PMC VALU issue and measured HBM bytes of this
        # build); the roofline fraction is priced against HBM either way
        bound, hbm_meas = roofline_bound(pf["traffic"], avg_s, pf["valu"])
        roofline = {"bound": bound, "priced_against": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                    "traffic": pf["traffic"], "traffic_uncorrected": pf["traffic_uncorrected"],
                    "traffic_source": prov,
                    "hbm_frac_measured": round(hbm_meas, 5) if hbm_meas is not None else None,
                    **rocprof_fields(pf, bytes_per_launch),
                    "kernel": "k_rollout", "unit_bytes": unit_bytes, "units_per_launch": rows_launch * p.N,
                    "bytes_per_launch": bytes_per_launch, "avg_launch_us": round(timing["rollout_cost"]["avg_us"], 3),
                    "frac_vs_measured_6290": round(achieved / 6290.0, 5),
                    "sdf_only_gbs": round(rows_launch * p.N * 4 * S / avg_s / 1e9, 2),
                    # this field's voxel is the 2-byte squared cell distance, not SURVEY's fp32
                    "unit_bytes_actual": 2 * S + 16 * p.J + 8,
                    "frac_actual_bytes": round(rows_launch * p.N * (2 * S + 16 * p.J + 8) / avg_s / 1e9 /
                                               HBM_PEAK_GBS, 5),
                    "frac_rows_written_24J": round(bytes_written_rows / avg_s / 1e9 / HBM_PEAK_GBS, 5),
                    "iteration_bytes": (K - args.reused + 1) * p.N * unit_bytes,
                    "iteration_frac": round((K - args.reused + 1) * p.N * unit_bytes * value /
                                            (HBM_PEAK_GBS * 1e9 * world), 5)}
        # the bound that actually binds: fp64 VALU issue (SQ_INSTS_VALU of the same build's PMC pass)
        roofline["valu"] = pf["valu"]

    # StompOptimizer::optimize (stomp_optimizer.cpp:249-401) through the device-resident loop:
    # the same iterations with the optimizer's bookkeeping, no early stop
    optimize = None
    if args.optimize_steps > 0 and world == 1:
        po_ = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=K,
                              num_reused_rollouts=args.reused, build_grid=False, max_iterations=args.optimize_steps,
                              max_iterations_after_collision_free=args.optimize_steps + 1)
        eo = eng.Engine(po_, device=local_rank, sdf_device_ptr=sdf.ptr)
        eo.optimize()   # warm
        t0 = time.perf_counter()
        st, _ = eo.optimize()
        dt = time.perf_counter() - t0
        optimize = {"iterations": st.iterations, "iterations_per_s": round(st.iterations / dt, 3)}
        eo.close()

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        pc = pb.make_problem(dof=args.dof, waypoints=args.waypoints, grid_n=args.grid, num_rollouts=K,
                             num_reused_rollouts=args.reused)
        cpu = cpu_baseline(pc, args.cpu_seconds)
        cpu_mt = cpu_baseline_all_cores(pc, min(args.cpu_seconds, 8.0))

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "iterations/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (PR2-like arm, shelf+pole scene, device-built SDF; Philox noise)",
            "config": {"workload": f"{workload_name(args)}: {args.dof}-DOF, {args.waypoints} wp (N={p.N}), K={K} "
                                   f"({K_loc}/GPU), K_r={args.reused}, {args.grid}^3 SDF, S={S} spheres",
                       "global_rollouts": K, "rollouts_per_gpu": K_loc,
                       "parallelism": f"rollout shard x{world}" + (f" (RCCL, {e.shard_mode}{shard_why(e)})"
                                                                     if world > 1 else ""),
                       "shard_choice": e.shard_info,
                       "rollouts_per_s": round(value * K, 1)},
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
    try:
        main()
    except RuntimeError as ex:
        # an engine failure (e.g. STOMP_E_COMM from the bounded collective wait): the message, a
        # non-zero exit, no retry
        print(f"bench.py rank {os.environ.get('RANK', '0')}: {ex}", file=sys.stderr)
        sys.exit(3)
