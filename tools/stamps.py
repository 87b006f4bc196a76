"""Diagnostic: per-phase cycle breakdown of the STOMP kernels from in-kernel s_memtime stamps.

Needs the stamps library (python -m stomp_motion_planner_icra2011_amd._build --stamps); never
used for timing claims (the stamps serialise the kernels they instrument).
Usage: STOMP_ENGINE_LIB=.../libstomp_engine_stamps.so python tools/stamps.py [K] [grid] [dof] [K_r] [waypoints]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stomp_motion_planner_icra2011_amd import engine as eng  # noqa: E402
from stomp_motion_planner_icra2011_amd import problem as pb  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 512
G = int(sys.argv[2]) if len(sys.argv) > 2 else 256
DOF = int(sys.argv[3]) if len(sys.argv) > 3 else 7
KR = int(sys.argv[4]) if len(sys.argv) > 4 else 0
WP = int(sys.argv[5]) if len(sys.argv) > 5 else 100
lib = eng.load_library()
p = pb.make_problem(dof=DOF, waypoints=WP, grid_n=G, num_rollouts=K, num_reused_rollouts=KR, build_grid=False)
sdf = eng.DeviceBuffer(4 * G ** 3)
eng.sdf_build_device(p, sdf.ptr)
e = eng.Engine(p, sdf_device_ptr=sdf.ptr)
e.run(1, 5)
e.synchronize()
buf = (C.c_ulonglong * 256)()


def show(name, block, labels):
    fn = getattr(lib, "stomp_debug_stamps_" + name)
    fn.argtypes = [C.c_int, C.c_void_p, C.c_int]
    fn(block, None, 1)
    e.run(6, 1)
    e.synchronize()
    fn(block, buf, 0)
    v = np.array(buf[:], dtype=np.int64)
    idx = [i for i in range(256) if v[i] != 0]
    if not idx:
        print(name, "no stamps")
        return
    idx = sorted(idx, key=lambda i: v[i])   # time order
    t0 = v[idx[0]]
    print(f"--- {name} block {block}: total {(v[idx[-1]] - t0)} cycles")
    prev = t0
    for i in idx:
        print(f"  {labels(i):28s} +{v[i] - prev:8d}  @{v[i] - t0:8d}")
        prev = v[i]


SPLIT_LABELS = {200: "start", 201: "row loads + tables", 202: "row (noise / from pregen)", 203: "joint limits",
                204: "traj out + sin/cos", 205: "FK (+ control rows)", 206: "pairs", 207: "velocities",
                208: "fold + stores", 209: "count / last piece"}


def cost_label(i):
    if i in SPLIT_LABELS:
        return "split: " + SPLIT_LABELS[i]
    if i in (61, 62, 63):
        return {61: "control terms (thread 0)", 62: "control terms barrier", 63: "control costs stored (t0)"}[i]
    if 100 <= i < 140:
        return f"FK op {i - 100}"
    if 140 <= i < 160:
        return f"JL pass {i - 140}: argmax, loads issued"
    if 160 <= i < 180:
        return f"JL pass {i - 160}: finished joints published"
    if i == 180:
        return "JL group end"
    if 40 <= i < 100:
        return f"slot {i - 40}: gathers issued (last round)"
    if 10 <= i < 40:
        g, ph = (i - 10) // 4, (i - 10) % 4
        return f"slot {g}: " + ["FK + publish", "positions+gathers+pots", "velocity", "fold (lanes t<N)"][ph]
    return {0: "start", 6: "normals / traj + tables", 7: "normals barrier | first FK advance", 8: "L z", 9: "M eps", 1: "control", 2: "joint limits", 3: "traj out",
            4: "FK/pairs done", 5: "end"}.get(i, str(i))


show("cost", 1, cost_label)   # a noisy rollout of the last iteration launch (odd: FK on waves 2-3)
show("cost", 2, cost_label)   # an even one (FK on waves 0-1, thread 0 stamps inside the FK lanes)
show("cost", 0, cost_label)   # the last launch: the flushed noiseless rollout
for b in [int(x) for x in os.environ.get("STAMP_COST_BLOCKS", "").split(",") if x]:
    show("cost", b, cost_label)   # chosen blocks (a split launch: rollout e's piece p is e P + p)
if os.environ.get("STAMP_SPAN"):
    # start / end of every workgroup of the last launch that ran it (block records), relative
    # to the earliest start: which pieces finish last
    fn = lib.stomp_debug_blocks_cost
    fn.argtypes = [C.c_void_p]
    bb = np.zeros((8192, 6), np.uint64)
    e.run(6, 1)
    e.synchronize()
    fn(bb.ctypes.data)
    n = int(os.environ["STAMP_SPAN"])
    rec = bb[:n].astype(np.int64)
    lo = rec[:, 2][rec[:, 2] > 0].min()
    for i in range(n):
        if rec[i, 2] > 0:
            print(f"    block {i:4d} start {int(rec[i, 2] - lo):8d} end {int(rec[i, 3] - lo):8d}")
NOISE_LABELS = {0: "start", 6: "reuse: loads in, staged", 10: "reuse: K-ranked", 11: "reuse: row loads issued", 12: "reuse: t-chains (wave 0)", 7: "reuse: barrier", 1: "rows loaded / normals", 2: "M eps (rows) / L z", 3: "M eps", 4: "control", 5: "end",
                9: "control: padding", 61: "control terms (thread 0)", 62: "control terms barrier",
                63: "control costs stored (t0)"}
show("noise", 0, lambda i: NOISE_LABELS.get(i, str(i)))
if KR > 0:
    show("misc", 0, lambda i: {0: "k_reuse: start", 1: "rows staged", 2: "t-chains", 3: "total counted",
                               10: "last: start", 11: "last: totals loaded", 12: "last: ranked",
                               13: "last: rows copied"}.get(i, str(i)))
WEIGHT_LABELS = {0: "start", 1: "min/max", 2: "exp", 3: "psum", 4: "u partials", 5: "end", 6: "tile loaded",
                 10: "pick: start", 11: "pick: loads issued", 12: "pick: staged (barrier)", 13: "pick: ranked",
                 14: "pick: extra total / choice", 15: "pick: rows written", 16: "pick: weights done"}
show("weights", 0, lambda i: WEIGHT_LABELS.get(i, str(i)))


def residency():
    """Workgroups of one rollout-cost launch per CU, and their overlap in time."""
    fn = lib.stomp_debug_blocks_cost
    fn.argtypes = [C.c_void_p]
    buf = np.zeros((8192, 6), np.uint64)
    e.run(7, 1)
    e.synchronize()
    fn(buf.ctypes.data)
    b = buf[: int(os.environ.get("STAMP_BLOCKS", K + 1))].astype(np.int64)
    cu = ((b[:, 1] & 0xF) << 8) | ((b[:, 0] >> 8) & 0xFF)
    t0, t1 = b[:, 2], b[:, 3]
    import collections
    per = collections.defaultdict(list)
    for i in range(len(b)):
        per[int(cu[i])].append((int(t0[i]), int(t1[i])))
    conc = []
    for v in per.values():
        ev = sorted([(a, 1) for a, _ in v] + [(c, -1) for _, c in v])
        cur = mx = 0
        for _, d in ev:
            cur += d
            mx = max(mx, cur)
        conc.append(mx)
    # durations by how many rollout WGs their CU ran concurrently (at their start)
    by_conc = collections.defaultdict(list)
    for i in range(len(b)):
        c = int(cu[i])
        n_at = sum(1 for (a0, a1) in per[c] if a0 <= t0[i] < a1)
        by_conc[n_at].append(int(t1[i] - t0[i]))
    for k in sorted(by_conc):
        v = np.array(by_conc[k])
        print(f"    CU running {k} rollout WGs at start: {len(v)} WGs, duration mean {int(v.mean())} max {int(v.max())}")
    ctl, jl = b[:, 4] - t0, b[:, 5] - b[:, 4]
    rest = t1 - b[:, 5]
    dur = t1 - t0
    for name, v in (("start..control", ctl), ("joint limits", jl), ("FK/pairs/fold/end", rest)):
        print(f"    {name:18s} min/median/max {int(v.min())}/{int(np.median(v))}/{int(v.max())}  "
              f"corr with duration {np.corrcoef(v, dur)[0, 1]:.2f}")
    slow = np.argsort(-(t1 - t0))[:8]
    print("    slowest blocks:", [(int(i), int(t1[i] - t0[i]), len(per[int(cu[i])])) for i in slow])
    span = int(t1.max() - t0.min())
    print(f"--- residency: {len(per)} CUs used by {len(b)} workgroups; per CU: "
          f"{collections.Counter(len(v) for v in per.values())}; max concurrent per CU: {collections.Counter(conc)}")
    print(f"    launch span {span} cycles; workgroup duration min/median/max "
          f"{int((t1 - t0).min())}/{int(np.median(t1 - t0))}/{int((t1 - t0).max())}")



def slowest_detail(it=9, count=3):
    """Phase stamps of the slowest rollout workgroups of one launch (and the fastest): the
    residency record of iteration it picks them, then theta is restored and the same iteration is
    run again with the stamps on each picked block (the noise is counter-based, so block b is the
    same rollout both times)."""
    fn = lib.stomp_debug_blocks_cost
    fn.argtypes = [C.c_void_p]
    th = e.theta()
    e.run(it, 1)
    e.synchronize()
    buf = np.zeros((8192, 6), np.uint64)
    fn(buf.ctypes.data)
    b = buf[:K].astype(np.int64)
    dur = b[:, 3] - b[:, 2]
    order = np.argsort(-dur)
    print(f"--- iteration {it}: rollout WG duration min/median/max {int(dur.min())}/{int(np.median(dur))}/{int(dur.max())}")
    picks = [int(i) for i in order[:count]] + [int(order[-1])]
    for blk in picks:
        e.set_theta(th)
        show_one(blk, it, int(dur[blk]))


def show_one(block, it, dur):
    fn = lib.stomp_debug_stamps_cost
    fn.argtypes = [C.c_int, C.c_void_p, C.c_int]
    fn(block, None, 1)
    e.run(it, 1)
    e.synchronize()
    fn(block, buf, 0)
    v = np.array(buf[:], dtype=np.int64)
    idx = sorted([i for i in range(256) if v[i] != 0], key=lambda i: v[i])
    if not idx:
        print("no stamps")
        return
    t0 = v[idx[0]]
    print(f"--- block {block} (residency-pass duration {dur}): total {v[idx[-1]] - t0} cycles")
    prev = t0
    for i in idx:
        print(f"  {cost_label(i):28s} +{v[i] - prev:8d}  @{v[i] - t0:8d}")
        prev = v[i]


residency()
if os.environ.get("STAMP_SLOW"):
    slowest_detail()
