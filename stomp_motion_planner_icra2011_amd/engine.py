"""ctypes binding of the C ABI in include/stomp_engine.h (libstomp_engine.so, built in-tree).

There is no CPU fallback: if the HIP library is missing or cannot be loaded the
constructor raises.  The CPU oracle lives under oracle/ and is test-only.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import _build

_LIB_PATH = _build.LIB
ABI_VERSION = 4


class stomp_segment(C.Structure):
    _fields_ = [("parent", C.c_int32), ("q_index", C.c_int32), ("rot", C.c_double * 9),
                ("trans", C.c_double * 3), ("axis", C.c_double * 3)]


class stomp_sphere(C.Structure):
    _fields_ = [("segment", C.c_int32), ("radius", C.c_double), ("clearance", C.c_double), ("pos", C.c_double * 3)]


class stomp_shape(C.Structure):
    _fields_ = [("type", C.c_int32), ("position", C.c_double * 3), ("orientation", C.c_double * 4),
                ("dims", C.c_double * 3), ("vertices", C.POINTER(C.c_double)), ("num_vertices", C.c_int32)]


class stomp_joint(C.Structure):
    _fields_ = [("has_limits", C.c_int32), ("min", C.c_double), ("max", C.c_double), ("joint_cost", C.c_double)]


class stomp_grid(C.Structure):
    _fields_ = [("nx", C.c_int32), ("ny", C.c_int32), ("nz", C.c_int32), ("origin", C.c_double * 3),
                ("resolution", C.c_double), ("data", C.c_void_p), ("data_on_device", C.c_int32)]


class stomp_inertia(C.Structure):
    _fields_ = [("mass", C.c_double), ("com", C.c_double * 3), ("inertia", C.c_double * 6)]


class stomp_orientation_constraint(C.Structure):
    _fields_ = [("segment", C.c_int32), ("orientation", C.c_double * 4), ("body_fixed", C.c_int32),
                ("absolute_roll_tolerance", C.c_double), ("absolute_pitch_tolerance", C.c_double),
                ("absolute_yaw_tolerance", C.c_double), ("weight", C.c_double)]


class stomp_engine_desc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("num_joints", C.c_int32), ("num_time_steps", C.c_int32),
                ("num_rollouts", C.c_int32), ("num_reused_rollouts", C.c_int32), ("num_segments", C.c_int32),
                ("segments", C.POINTER(stomp_segment)), ("num_spheres", C.c_int32),
                ("spheres", C.POINTER(stomp_sphere)), ("joints", C.POINTER(stomp_joint)), ("grid", stomp_grid),
                ("discretization", C.c_double), ("smoothness_costs", C.c_double * 3), ("ridge_factor", C.c_double),
                ("smoothness_cost_weight", C.c_double), ("obstacle_cost_weight", C.c_double),
                ("constraint_cost_weight", C.c_double), ("torque_cost_weight", C.c_double),
                ("noise_stddev", C.POINTER(C.c_double)), ("noise_decay", C.POINTER(C.c_double)),
                ("use_cumulative_costs", C.c_int32), ("start", C.POINTER(C.c_double)),
                ("goal", C.POINTER(C.c_double)), ("seed", C.c_uint64), ("max_iterations", C.c_int32),
                ("max_iterations_after_collision_free", C.c_int32), ("device", C.c_int32), ("stream", C.c_void_p),
                ("rank", C.c_int32), ("world_size", C.c_int32), ("comm_id", C.c_void_p),
                ("inertias", C.POINTER(stomp_inertia)), ("torque_root", C.c_int32), ("torque_tip", C.c_int32),
                ("gravity", C.c_double * 3), ("num_orientation_constraints", C.c_int32),
                ("orientation_constraints", C.POINTER(stomp_orientation_constraint))]


class stomp_iter_out(C.Structure):
    _fields_ = [("cost", C.c_double), ("collision_free", C.c_int32), ("constraints_satisfied", C.c_int32)]


class stomp_stats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("success", C.c_int32), ("success_iteration", C.c_int32),
                ("collision_success_iteration", C.c_int32), ("last_improvement_iteration", C.c_int32),
                ("best_cost", C.c_double), ("success_duration", C.c_double),
                ("collision_success_duration", C.c_double)]


# every symbol include/stomp_engine.h declares (checked by tests/test_abi.py)
EXPORTED = ["stomp_engine_create", "stomp_engine_destroy", "stomp_engine_last_error", "stomp_last_error",
            "stomp_engine_get_theta", "stomp_engine_set_theta", "stomp_engine_iterate", "stomp_engine_run",
            "stomp_engine_synchronize", "stomp_engine_eval", "stomp_engine_optimize",
            "stomp_engine_get_best_trajectory", "stomp_engine_get_last_trajectory", "stomp_engine_get_rollouts",
            "stomp_engine_get_matrix", "stomp_engine_get_pad_positions", "stomp_engine_set_timing",
            "stomp_engine_get_timing", "stomp_engine_local_rollouts", "stomp_sdf_build", "stomp_comm_unique_id",
            "stomp_device_selftest", "stomp_device_normals", "stomp_device_alloc", "stomp_device_free",
            "stomp_device_copy_to_host", "stomp_device_count", "stomp_diff_rules", "stomp_comm_local_id",
            "stomp_engine_get_best_torques", "stomp_pi_get_rollouts", "stomp_pi_set_rollout_costs",
            "stomp_pi_improve_policy", "stomp_pi_add_extra_rollouts", "stomp_pi_reset", "stomp_sdf_build_objects",
            "stomp_stream_create", "stomp_stream_destroy", "stomp_group_create", "stomp_group_run",
            "stomp_group_synchronize", "stomp_group_last_error", "stomp_group_destroy", "stomp_engine_shard_mode",
            "stomp_engine_shard_info", "stomp_shard_decide", "stomp_engine_source_hash",
            "stomp_engine_refresh_field"]

_lib = None


def load_library(path: Optional[str] = None):
    """Loads libstomp_engine.so (building it first if absent and hipcc is available)."""
    global _lib
    if _lib is not None:
        return _lib
    explicit = path or os.environ.get("STOMP_ENGINE_LIB")
    path = explicit or _LIB_PATH
    if not os.path.exists(path):
        if os.path.exists(_build.HIPCC):
            _build.build()
        else:
            raise RuntimeError(f"STOMP HIP engine library missing: {path} (run __graft_entry__.build())")
    if not explicit:
        # the product library must be built from this checkout's sources (a variant named by
        # STOMP_ENGINE_LIB is an experiment's build with its own defines)
        built, want = _build.embedded_hash(path), _build.source_hash()
        if built != want:
            raise RuntimeError(f"stale STOMP engine library {path}: built from sources {built}, the checkout's "
                               f"are {want} (run __graft_entry__.build())")
    l = C.CDLL(path)
    l.stomp_engine_source_hash.restype = C.c_char_p
    l.stomp_engine_source_hash.argtypes = []
    P, dp = C.c_void_p, C.POINTER(C.c_double)
    l.stomp_engine_create.argtypes = [C.POINTER(stomp_engine_desc), C.POINTER(C.c_void_p)]
    l.stomp_engine_destroy.argtypes = [P]
    l.stomp_engine_last_error.restype = C.c_char_p
    l.stomp_engine_last_error.argtypes = [P]
    l.stomp_last_error.restype = C.c_char_p
    l.stomp_engine_get_theta.argtypes = [P, dp]
    l.stomp_engine_refresh_field.argtypes = [P]
    l.stomp_engine_set_theta.argtypes = [P, dp]
    l.stomp_engine_iterate.argtypes = [P, C.c_int32, C.POINTER(stomp_iter_out)]
    l.stomp_engine_run.argtypes = [P, C.c_int32, C.c_int32]
    l.stomp_engine_synchronize.argtypes = [P]
    l.stomp_engine_eval.argtypes = [P, dp, C.c_int32, dp, C.POINTER(C.c_uint8), dp, C.c_int32, C.POINTER(C.c_uint8)]
    l.stomp_engine_optimize.argtypes = [P, C.POINTER(stomp_stats), dp]
    l.stomp_engine_get_best_trajectory.argtypes = [P, dp]
    l.stomp_engine_get_best_torques.argtypes = [P, dp]
    l.stomp_pi_get_rollouts.argtypes = [P, C.c_int32, dp, dp, C.POINTER(C.c_int32)]
    l.stomp_pi_set_rollout_costs.argtypes = [P, dp, C.c_double, dp]
    l.stomp_pi_improve_policy.argtypes = [P, dp]
    l.stomp_pi_add_extra_rollouts.argtypes = [P, C.c_int32, dp, dp]
    l.stomp_pi_reset.argtypes = [P]
    l.stomp_engine_get_last_trajectory.argtypes = [P, dp]
    l.stomp_engine_get_rollouts.argtypes = [P, C.c_char_p, dp]
    l.stomp_engine_get_matrix.argtypes = [P, C.c_char_p, C.c_int32, dp]
    l.stomp_engine_get_pad_positions.argtypes = [P, dp]
    l.stomp_engine_set_timing.argtypes = [P, C.c_int32]
    l.stomp_engine_get_timing.argtypes = [P, C.c_char_p, dp, C.POINTER(C.c_int32)]
    l.stomp_engine_local_rollouts.argtypes = [P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    l.stomp_engine_shard_mode.argtypes = [P, C.POINTER(C.c_int32)]
    l.stomp_engine_shard_info.argtypes = [P, dp]
    l.stomp_shard_decide.argtypes = [dp, C.POINTER(C.c_int32)]
    l.stomp_sdf_build.argtypes = [C.c_int32, C.c_int32, C.c_int32, dp, C.c_double, C.c_double, dp, C.c_int32, dp,
                                  C.c_int32, C.c_void_p, C.c_void_p]
    l.stomp_sdf_build_objects.argtypes = [C.c_int32, C.c_int32, C.c_int32, dp, C.c_double, C.c_double,
                                          C.POINTER(stomp_shape), C.c_int32, dp, C.c_int64, C.c_void_p,
                                          C.POINTER(C.c_int64), C.c_void_p]
    l.stomp_stream_create.argtypes = [C.c_int32, C.POINTER(C.c_void_p)]
    l.stomp_stream_destroy.argtypes = [C.c_void_p]
    l.stomp_group_create.argtypes = [C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_void_p)]
    l.stomp_group_run.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    l.stomp_group_synchronize.argtypes = [C.c_void_p]
    l.stomp_group_last_error.restype = C.c_char_p
    l.stomp_group_last_error.argtypes = [C.c_void_p]
    l.stomp_group_destroy.argtypes = [C.c_void_p]
    l.stomp_comm_unique_id.argtypes = [C.c_void_p]
    l.stomp_comm_local_id.argtypes = [C.c_int32, C.c_void_p]
    l.stomp_device_alloc.argtypes = [C.c_int32, C.c_uint64, C.POINTER(C.c_void_p)]
    l.stomp_device_free.argtypes = [C.c_void_p]
    l.stomp_device_copy_to_host.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    l.stomp_device_count.argtypes = [C.POINTER(C.c_int32)]
    l.stomp_diff_rules.argtypes = [dp]
    l.stomp_device_selftest.argtypes = [dp, C.c_int32, dp, dp, dp, dp, dp]
    l.stomp_device_normals.argtypes = [C.c_uint64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, dp]
    _lib = l
    return l


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _check(rc: int, handle=None):
    if rc != 0:
        l = load_library()
        msg = (l.stomp_engine_last_error(handle) if handle else l.stomp_last_error()).decode()
        raise RuntimeError(f"stomp engine error {rc}: {msg}")


def sdf_build_device(problem, device_tensor_ptr: int, stream: int = 0):
    """Builds problem.grid's distance field directly into a device buffer of n^3 uint16 squared cell
    distances (stomp_grid's representation; problem.build_sdf is the host twin)."""
    l = load_library()
    g = problem.grid
    boxes = np.array([list(b.center) + list(b.dims) for b in problem.boxes], np.float64).reshape(-1)
    cyl = np.array([list(c.center) + [c.radius, c.length] for c in problem.cylinders], np.float64).reshape(-1)
    origin = np.array(g.origin, np.float64)
    boxes = boxes if boxes.size else np.zeros(1)
    cyl = cyl if cyl.size else np.zeros(1)
    _check(l.stomp_sdf_build(g.n, g.n, g.n, _dp(origin), g.resolution, g.max_expansion, _dp(boxes),
                             len(problem.boxes), _dp(cyl), len(problem.cylinders), C.c_void_p(device_tensor_ptr),
                             C.c_void_p(stream)))


def shape_array(objects):
    """problem.SceneObject list -> stomp_shape[] (ctypes array; length >= 1; it keeps the mesh
    vertex arrays alive as ._keep)."""
    arr = (stomp_shape * max(len(objects), 1))()
    arr._keep = []
    for i, o in enumerate(objects):
        arr[i].type = int(o.type)
        arr[i].position[:] = [float(v) for v in o.position]
        arr[i].orientation[:] = [float(v) for v in o.orientation]
        d = list(o.dims) + [0.0] * (3 - len(o.dims))
        arr[i].dims[:] = [float(v) for v in d[:3]]
        if getattr(o, "vertices", None) is not None:
            v = np.ascontiguousarray(o.vertices, np.float64).reshape(-1, 3)
            arr._keep.append(v)
            arr[i].vertices = _dp(v)
            arr[i].num_vertices = len(v)
    return arr


def sdf_build_objects_device(grid, objects, device_ptr: int, points=None, stream: int = 0) -> int:
    """The reference's distance-field fill (stomp_sdf_build_objects) of problem.Grid `grid` from
    collision objects (problem.SceneObject) and collision-map points (P x 3) into a device buffer
    of n^3 uint16 squared cell distances.  Returns the number of points that landed in the grid."""
    l = load_library()
    origin = np.array(grid.origin, np.float64)
    pts = np.ascontiguousarray(points if points is not None else np.zeros((0, 3)), np.float64).reshape(-1, 3)
    marked = C.c_int64(0)
    _check(l.stomp_sdf_build_objects(grid.n, grid.n, grid.n, _dp(origin), grid.resolution, grid.max_expansion,
                                     shape_array(objects), len(objects), _dp(pts if pts.size else np.zeros(3)),
                                     len(pts), C.c_void_p(device_ptr), C.byref(marked), C.c_void_p(stream)))
    return marked.value


class Engine:
    """One planning problem on one device: the StompOptimizer / PolicyImprovementLoop pair."""

    def __init__(self, problem, device: int = 0, sdf_device_ptr: Optional[int] = None, stream: Optional[int] = None,
                 rank: int = 0, world_size: int = 1, comm_id: Optional[bytes] = None):
        l = load_library()
        p = problem
        self.problem = p
        self.J, self.N, self.K = p.J, p.N, p.params.num_rollouts
        self.S = len(p.spheres)
        self._segs = (stomp_segment * len(p.robot.segments))(*[
            stomp_segment(s.parent, s.q_index, (C.c_double * 9)(*s.rot), (C.c_double * 3)(*s.trans),
                          (C.c_double * 3)(*s.axis)) for s in p.robot.segments])
        self._sph = (stomp_sphere * max(self.S, 1))(*[
            stomp_sphere(s.segment, s.radius, s.clearance, (C.c_double * 3)(*s.pos)) for s in p.spheres])
        self._joints = (stomp_joint * self.J)(*[
            stomp_joint(int(j.has_limits), j.min, j.max, j.joint_cost) for j in p.robot.joints])
        pr = p.params
        self._sig = pr.per_joint("noise_stddev", self.J)
        self._dec = pr.per_joint("noise_decay", self.J)
        self._start = np.ascontiguousarray(p.start, np.float64)
        self._goal = np.ascontiguousarray(p.goal, np.float64)
        g = p.grid
        d = stomp_engine_desc()
        d.abi_version = ABI_VERSION
        d.num_joints, d.num_time_steps, d.num_rollouts = self.J, self.N, self.K
        d.num_reused_rollouts = pr.num_reused_rollouts
        d.num_segments = len(p.robot.segments)
        d.segments = self._segs
        d.num_spheres = self.S
        d.spheres = self._sph
        d.joints = self._joints
        if sdf_device_ptr is not None:
            grid_ptr, on_dev = sdf_device_ptr, 1
        else:
            # ABI v4: the field is the integer squared cell distance (PropagationDistanceField's
            # distance_square_), not metres; a float field would truncate to "in collision" silently
            sdf = np.asarray(p.sdf)
            if not np.issubdtype(sdf.dtype, np.integer):
                raise TypeError(f"problem.sdf must hold integer squared cell distances (uint16), got {sdf.dtype}")
            if sdf.size and (int(sdf.min()) < 0 or int(sdf.max()) > 65535):
                raise ValueError("problem.sdf squared cell distances must lie in [0, 65535]")
            self._sdf = np.ascontiguousarray(sdf, np.uint16)
            grid_ptr, on_dev = self._sdf.ctypes.data, 0
        d.grid = stomp_grid(g.n, g.n, g.n, (C.c_double * 3)(*g.origin), g.resolution, C.c_void_p(grid_ptr), on_dev)
        d.discretization = pr.trajectory_discretization
        d.smoothness_costs = (C.c_double * 3)(pr.smoothness_cost_velocity, pr.smoothness_cost_acceleration,
                                              pr.smoothness_cost_jerk)
        d.ridge_factor = pr.ridge_factor
        d.smoothness_cost_weight = pr.smoothness_cost_weight
        d.obstacle_cost_weight = pr.obstacle_cost_weight
        d.constraint_cost_weight = pr.constraint_cost_weight
        d.torque_cost_weight = pr.torque_cost_weight
        d.noise_stddev = _dp(self._sig)
        d.noise_decay = _dp(self._dec)
        d.use_cumulative_costs = int(pr.use_cumulative_costs)
        d.start = _dp(self._start)
        d.goal = _dp(self._goal)
        d.seed = p.seed
        d.max_iterations = pr.max_iterations
        d.max_iterations_after_collision_free = pr.max_iterations_after_collision_free
        d.device = device
        d.stream = C.c_void_p(stream) if stream else None
        d.rank = rank
        d.world_size = world_size
        self._comm = C.create_string_buffer(comm_id, 128) if comm_id else None
        d.comm_id = C.cast(self._comm, C.c_void_p) if comm_id else None
        nseg = len(p.robot.segments)
        self._inertia = (stomp_inertia * nseg)(*[
            stomp_inertia(s.inertia.mass, (C.c_double * 3)(*s.inertia.com), (C.c_double * 6)(*s.inertia.inertia))
            if s.inertia else stomp_inertia() for s in p.robot.segments])
        d.inertias = self._inertia
        d.torque_root = p.robot.index(p.torque_root)
        d.torque_tip = p.robot.index(p.torque_tip)
        d.gravity = (C.c_double * 3)(*p.gravity)
        oc = p.orientation_constraints
        self._oc = (stomp_orientation_constraint * max(len(oc), 1))(*[
            stomp_orientation_constraint(p.robot.index(c.link_name), (C.c_double * 4)(*c.orientation),
                                         0 if c.header_frame else 1, c.absolute_roll_tolerance,
                                         c.absolute_pitch_tolerance, c.absolute_yaw_tolerance, c.weight)
            for c in oc])
        d.num_orientation_constraints = len(oc)
        d.orientation_constraints = self._oc
        self._desc = d
        h = C.c_void_p()
        _check(l.stomp_engine_create(C.byref(d), C.byref(h)))
        self.h = h
        first, count = C.c_int32(), C.c_int32()
        l.stomp_engine_local_rollouts(self.h, C.byref(first), C.byref(count))
        self.first, self.K_loc = first.value, count.value
        mode = C.c_int32()
        _check(l.stomp_engine_shard_mode(self.h, C.byref(mode)))
        self.shard_mode = {0: "none", 1: "partials", 2: "gather"}[mode.value]
        info = np.zeros(6)
        _check(l.stomp_engine_shard_info(self.h, _dp(info)))
        # measured at creation when both decompositions were possible (stomp_engine_shard_info), us
        self.shard_info = None if info[1] == 0.0 else dict(
            t_gather=info[1], t_partials=info[2], l_allreduce=info[3], l_allgather_state=info[4],
            l_allgather_partials=info[5])

    def close(self):
        h = getattr(self, "h", None)
        if h:
            load_library().stomp_engine_destroy(h)
            self.h = None

    def __del__(self):
        self.close()

    # ---------------------------------------------------------------- API
    def theta(self) -> np.ndarray:
        out = np.zeros((self.J, self.N))
        _check(load_library().stomp_engine_get_theta(self.h, _dp(out)), self.h)
        return out

    def set_theta(self, theta):
        t = np.ascontiguousarray(theta, np.float64)
        _check(load_library().stomp_engine_set_theta(self.h, _dp(t)), self.h)

    def iterate(self, iteration_number: int):
        o = stomp_iter_out()
        _check(load_library().stomp_engine_iterate(self.h, iteration_number, C.byref(o)), self.h)
        self.last_constraints_satisfied = bool(o.constraints_satisfied)
        return o.cost, bool(o.collision_free)

    def run(self, first_iteration: int, count: int):
        _check(load_library().stomp_engine_run(self.h, first_iteration, count), self.h)

    def synchronize(self):
        _check(load_library().stomp_engine_synchronize(self.h), self.h)

    def refresh_field(self):
        """stomp_engine_refresh_field: the caller rebuilt its device field in place."""
        _check(load_library().stomp_engine_refresh_field(self.h), self.h)

    def execute(self, params, iteration_member: int = 1):
        prm = np.ascontiguousarray(params, np.float64)
        single = prm.ndim == 2
        prm = prm.reshape(-1, self.J, self.N)
        n = prm.shape[0]
        costs = np.zeros((n, self.N))
        cf = np.zeros(n, np.uint8)
        traj = np.zeros((n, self.J, self.N))
        cs = np.zeros(n, np.uint8)
        u8 = C.POINTER(C.c_uint8)
        _check(load_library().stomp_engine_eval(self.h, _dp(prm), n, _dp(costs), cf.ctypes.data_as(u8), _dp(traj),
                                                iteration_member, cs.ctypes.data_as(u8)), self.h)
        self.last_constraints_satisfied = cs.astype(bool)
        if single:
            return costs[0], bool(cf[0]), traj[0]
        return costs, cf.astype(bool), traj

    def optimize(self):
        st = stomp_stats()
        costs = np.zeros(max(self.problem.params.max_iterations, 1))
        _check(load_library().stomp_engine_optimize(self.h, C.byref(st), _dp(costs)), self.h)
        return st, costs[: st.iterations]

    def best_trajectory(self) -> np.ndarray:
        out = np.zeros((self.J, self.N))
        _check(load_library().stomp_engine_get_best_trajectory(self.h, _dp(out)), self.h)
        return out

    def last_trajectory(self) -> np.ndarray:
        out = np.zeros((self.J, self.N))
        _check(load_library().stomp_engine_get_last_trajectory(self.h, _dp(out)), self.h)
        return out

    def best_torques(self) -> np.ndarray:
        out = np.zeros(self.N)
        _check(load_library().stomp_engine_get_best_torques(self.h, _dp(out)), self.h)
        return out

    # ---------------------------------------------------- PolicyImprovement API (stomp_pi_*)
    def pi_get_rollouts(self, iteration: int, noise_stddev) -> np.ndarray:
        sig = np.ascontiguousarray(noise_stddev, np.float64)
        out = np.zeros((self.K, self.J, self.N))
        n = C.c_int32()
        _check(load_library().stomp_pi_get_rollouts(self.h, iteration, _dp(sig), _dp(out), C.byref(n)), self.h)
        return out[: n.value]

    def pi_set_rollout_costs(self, costs, control_cost_weight: float) -> np.ndarray:
        c = np.zeros((self.K, self.N))
        cc = np.asarray(costs, np.float64)
        c[: cc.shape[0]] = cc
        totals = np.zeros(self.K)
        _check(load_library().stomp_pi_set_rollout_costs(self.h, _dp(c), control_cost_weight, _dp(totals)), self.h)
        return totals

    def pi_improve_policy(self) -> np.ndarray:
        out = np.zeros((self.J, self.N))
        _check(load_library().stomp_pi_improve_policy(self.h, _dp(out)), self.h)
        return out

    def pi_add_extra_rollout(self, params, costs):
        p = np.ascontiguousarray(params, np.float64)
        c = np.ascontiguousarray(costs, np.float64)
        _check(load_library().stomp_pi_add_extra_rollouts(self.h, 1, _dp(p), _dp(c)), self.h)

    def rollouts(self, which: str) -> np.ndarray:
        if which.startswith("x_"):
            shape = (self.N,) if which == "x_state_costs" else (self.J, self.N)
        else:
            shape = (self.K_loc, self.N) if which == "state_costs" else (self.K_loc, self.J, self.N)
        out = np.zeros(shape)
        _check(load_library().stomp_engine_get_rollouts(self.h, which.encode(), _dp(out)), self.h)
        return out

    def matrix(self, which: str, joint: int = 0) -> np.ndarray:
        n = self.N + 12 if which in ("D0", "D1", "D2") else self.N
        out = np.zeros((n, n))
        _check(load_library().stomp_engine_get_matrix(self.h, which.encode(), joint, _dp(out)), self.h)
        return out

    def pad_positions(self) -> np.ndarray:
        out = np.zeros((12, self.S, 3))
        _check(load_library().stomp_engine_get_pad_positions(self.h, _dp(out)), self.h)
        return out

    def set_timing(self, enable: bool):
        _check(load_library().stomp_engine_set_timing(self.h, int(enable)), self.h)

    def timing(self, name: str):
        t, n = C.c_double(), C.c_int32()
        _check(load_library().stomp_engine_get_timing(self.h, name.encode(), C.byref(t), C.byref(n)), self.h)
        return t.value, n.value


class Stream:
    """A HIP stream of the engine runtime (engines of one group share one)."""

    def __init__(self, device: int = 0):
        self.ptr = None
        p = C.c_void_p()
        _check(load_library().stomp_stream_create(device, C.byref(p)))
        self.ptr = p.value

    def close(self):
        if self.ptr:
            load_library().stomp_stream_destroy(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        self.close()


class EngineGroup:
    """Engines of one shape on one shared stream, advanced in lockstep by shared launches
    (stomp_group_run: three dispatches per iteration for the whole group)."""

    def __init__(self, engines):
        self._h = None   # set before the call that may raise, so __del__ has nothing to free
        l = load_library()
        self.engines = list(engines)
        arr = (C.c_void_p * len(self.engines))(*[e.h.value for e in self.engines])
        h = C.c_void_p()
        rc = l.stomp_group_create(arr, len(self.engines), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"stomp group error {rc}: {l.stomp_last_error().decode()}")
        self._h = h

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f"stomp group error {rc}: {load_library().stomp_group_last_error(self._h).decode()}")

    def run(self, first: int, count: int):
        self._check(load_library().stomp_group_run(self._h, first, count))

    def synchronize(self):
        self._check(load_library().stomp_group_synchronize(self._h))

    def close(self):
        if self._h is not None and self._h.value:
            load_library().stomp_group_destroy(self._h)
        self._h = None

    def __del__(self):
        self.close()


class DeviceBuffer:
    """Engine-runtime device allocation (keeps torch's bundled HIP runtime out of the process)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.ptr = None   # set before the call that may raise, so __del__ has nothing to free
        p = C.c_void_p()
        _check(load_library().stomp_device_alloc(device, nbytes, C.byref(p)))
        self.ptr, self.nbytes = p.value, nbytes

    def to_numpy(self, dtype, shape):
        out = np.empty(shape, dtype)
        assert out.nbytes <= self.nbytes
        _check(load_library().stomp_device_copy_to_host(out.ctypes.data, C.c_void_p(self.ptr), out.nbytes))
        return out

    def free(self):
        if self.ptr:
            load_library().stomp_device_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        self.free()


def diff_rules() -> np.ndarray:
    """DIFF_RULES as compiled into the engine (host only)."""
    out = np.zeros((3, 7))
    _check(load_library().stomp_diff_rules(_dp(out)))
    return out


def device_count() -> int:
    n = C.c_int32()
    load_library().stomp_device_count(C.byref(n))
    return n.value


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    _check(load_library().stomp_comm_unique_id(buf))
    return buf.raw


def shard_decide(t_gather, t_partials, l_allreduce, l_allgather_state, l_allgather_partials) -> str:
    """The engine's decomposition rule on measured times (us), host only (stomp_shard_decide)."""
    m = np.array([t_gather, t_partials, l_allreduce, l_allgather_state, l_allgather_partials], np.float64)
    mode = C.c_int32()
    _check(load_library().stomp_shard_decide(_dp(m), C.byref(mode)))
    return {1: "partials", 2: "gather"}[mode.value]


def comm_local_id(world_size: int) -> bytes:
    """Id of an in-process exchange group (ranks = engines of this process, one host thread each)."""
    buf = C.create_string_buffer(128)
    _check(load_library().stomp_comm_local_id(world_size, buf))
    return buf.raw


def device_math(x: np.ndarray):
    x = np.ascontiguousarray(x, np.float64)
    n = len(x)
    outs = [np.zeros(n) for _ in range(5)]
    _check(load_library().stomp_device_selftest(_dp(x), n, *[_dp(o) for o in outs]))
    return outs


def device_normals(seed: int, iteration: int, joint: int, rollout: int, n: int) -> np.ndarray:
    z = np.zeros(n)
    _check(load_library().stomp_device_normals(seed, iteration, joint, rollout, n, _dp(z)))
    return z
