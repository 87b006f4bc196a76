"""Host enqueue time vs device time of stomp_engine_run (is a run launch-bound on the host?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stomp_motion_planner_icra2011_amd import engine as eng  # noqa: E402
from stomp_motion_planner_icra2011_amd import problem as pb  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 512
P = int(sys.argv[2]) if len(sys.argv) > 2 else 1
base = pb.make_problem(num_rollouts=K, num_reused_rollouts=0, build_grid=False, max_iterations=400)
sdf = eng.DeviceBuffer(4 * 256 ** 3)
eng.sdf_build_device(base, sdf.ptr)
es = [eng.Engine(pb.make_problem(num_rollouts=K, num_reused_rollouts=0, build_grid=False, seed=base.seed + i,
                                 max_iterations=400), sdf_device_ptr=sdf.ptr) for i in range(P)]
for e in es:
    e.run(1, 10)
for e in es:
    e.synchronize()
n = 100
t0 = time.perf_counter()
for k in range(n):
    for e in es:
        e.run(11 + k, 1)
t1 = time.perf_counter()
for e in es:
    e.synchronize()
t2 = time.perf_counter()
print(f"K={K} P={P}: enqueue {1e6 * (t1 - t0) / n:.1f} us per round, total {1e6 * (t2 - t0) / n:.1f} us per round")
