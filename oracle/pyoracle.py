"""TEST INFRASTRUCTURE: ctypes binding of the CPU oracle (oracle/libstomp_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
PARITY UNPINNED against the reference itself (see oracle/stomp_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_DIR, "libstomp_oracle.so")


class so_segment(C.Structure):
    _fields_ = [("parent", C.c_int), ("q_index", C.c_int), ("rot", C.c_double * 9),
                ("trans", C.c_double * 3), ("axis", C.c_double * 3)]


class so_sphere(C.Structure):
    _fields_ = [("segment", C.c_int), ("radius", C.c_double), ("clearance", C.c_double), ("pos", C.c_double * 3)]


class so_joint(C.Structure):
    _fields_ = [("has_limits", C.c_int), ("min", C.c_double), ("max", C.c_double), ("joint_cost", C.c_double)]


class so_sdf(C.Structure):
    _fields_ = [("nx", C.c_int), ("ny", C.c_int), ("nz", C.c_int), ("origin", C.c_double * 3),
                ("resolution", C.c_double), ("data", C.POINTER(C.c_uint16))]


class so_inertia(C.Structure):
    _fields_ = [("mass", C.c_double), ("com", C.c_double * 3), ("inertia", C.c_double * 6)]


class so_orientation_constraint(C.Structure):
    _fields_ = [("segment", C.c_int), ("orientation", C.c_double * 4), ("body_fixed", C.c_int),
                ("absolute_roll_tolerance", C.c_double), ("absolute_pitch_tolerance", C.c_double),
                ("absolute_yaw_tolerance", C.c_double), ("weight", C.c_double)]


class so_config(C.Structure):
    _fields_ = [("num_joints", C.c_int), ("num_time_steps", C.c_int), ("num_rollouts", C.c_int),
                ("num_reused_rollouts", C.c_int), ("num_segments", C.c_int),
                ("segments", C.POINTER(so_segment)), ("num_spheres", C.c_int),
                ("spheres", C.POINTER(so_sphere)), ("joints", C.POINTER(so_joint)), ("sdf", so_sdf),
                ("discretization", C.c_double), ("smoothness_costs", C.c_double * 3),
                ("ridge_factor", C.c_double), ("smoothness_cost_weight", C.c_double),
                ("obstacle_cost_weight", C.c_double), ("constraint_cost_weight", C.c_double),
                ("torque_cost_weight", C.c_double), ("noise_stddev", C.POINTER(C.c_double)),
                ("noise_decay", C.POINTER(C.c_double)), ("use_cumulative_costs", C.c_int),
                ("start", C.POINTER(C.c_double)), ("goal", C.POINTER(C.c_double)), ("seed", C.c_uint64),
                ("max_iterations", C.c_int), ("max_iterations_after_collision_free", C.c_int),
                ("sum_block", C.c_int), ("dense", C.c_int), ("threads", C.c_int),
                ("inertias", C.POINTER(so_inertia)), ("torque_root", C.c_int), ("torque_tip", C.c_int),
                ("gravity", C.c_double * 3), ("num_orientation_constraints", C.c_int),
                ("orientation_constraints", C.POINTER(so_orientation_constraint)), ("ref_arith", C.c_int)]


class so_iter_out(C.Structure):
    _fields_ = [("cost", C.c_double), ("collision_free", C.c_int), ("constraints_satisfied", C.c_int)]


class so_stats(C.Structure):
    _fields_ = [("iterations", C.c_int), ("success", C.c_int), ("success_iteration", C.c_int),
                ("collision_success_iteration", C.c_int), ("last_improvement_iteration", C.c_int),
                ("best_cost", C.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.check_call(["make", "-s", "-C", _DIR])
        l = C.CDLL(_LIB)
        P = C.c_void_p
        dp = C.POINTER(C.c_double)
        l.so_create.restype = P
        l.so_create.argtypes = [C.POINTER(so_config)]
        l.so_destroy.argtypes = [P]
        l.so_last_error.restype = C.c_char_p
        l.so_get_matrix.argtypes = [P, C.c_char_p, C.c_int, dp]
        l.so_get_theta.argtypes = [P, dp]
        l.so_set_theta.argtypes = [P, dp]
        l.so_get_pad_positions.argtypes = [P, dp]
        l.so_execute.argtypes = [P, dp, dp, C.POINTER(C.c_int), dp, C.c_int, C.POINTER(C.c_int)]
        l.so_iterate.argtypes = [P, C.c_int, C.POINTER(so_iter_out)]
        l.so_optimize.argtypes = [P, C.POINTER(so_stats), dp]
        l.so_get_best_trajectory.argtypes = [P, dp]
        l.so_get_best_torques.argtypes = [P, dp]
        l.so_get_last_trajectory.argtypes = [P, dp]
        l.so_get_rollouts.argtypes = [P, C.c_char_p, dp]
        l.so_reuse_log.argtypes = [P, C.POINTER(C.c_int), C.c_int]
        l.so_philox4x32.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        l.so_normals.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, dp]
        l.so_diff_rules.argtypes = [dp]
        l.so_exp.restype = C.c_double
        l.so_exp.argtypes = [C.c_double]
        l.so_log.restype = C.c_double
        l.so_log.argtypes = [C.c_double]
        l.so_sincos.argtypes = [C.c_double, dp, dp]
        l.so_sphere_positions.argtypes = [P, dp, dp]
        l.so_sdf_distance.restype = C.c_double
        l.so_sdf_distance.argtypes = [P, C.c_double, C.c_double, C.c_double]
        l.so_potential.argtypes = [P, C.c_int, dp, dp]
        l.so_inverse_dynamics.argtypes = [P, dp, dp, dp, dp]
        l.so_atan2.restype = C.c_double
        l.so_atan2.argtypes = [C.c_double, C.c_double]
        l.so_asin.restype = C.c_double
        l.so_asin.argtypes = [C.c_double]
        l.so_sdf_build_objects.restype = C.c_longlong
        l.so_sdf_build_objects.argtypes = [C.c_int, C.c_int, C.c_int, dp, C.c_double, C.c_double,
                                           C.POINTER(so_shape), C.c_int, dp, C.c_longlong,
                                           C.POINTER(C.c_ubyte), C.POINTER(C.c_uint16)]
        l.so_sdf_from_occupancy.restype = C.c_int
        l.so_hull_planes.restype = C.c_int
        l.so_hull_planes.argtypes = [dp, C.c_int, dp, C.c_int]
        l.so_sdf_from_occupancy.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double,
                                            C.POINTER(C.c_ubyte), C.POINTER(C.c_uint16)]
        _lib = l
    return _lib


class so_shape(C.Structure):
    _fields_ = [("type", C.c_int), ("position", C.c_double * 3), ("orientation", C.c_double * 4),
                ("dims", C.c_double * 3), ("vertices", C.POINTER(C.c_double)), ("num_vertices", C.c_int)]


def sdf_build_objects(grid, objects, points=None, with_field: bool = True):
    """so_sdf_build_objects (oracle/sdf_oracle.c) for problem.Grid `grid`: (field n^3 uint16 squared cell distances or None,
    marks n^3 uint8, number of points marked)."""
    n = grid.n
    arr = (so_shape * max(len(objects), 1))()
    keep = []
    for i, o in enumerate(objects):
        arr[i].type = int(o.type)
        arr[i].position[:] = [float(v) for v in o.position]
        arr[i].orientation[:] = [float(v) for v in o.orientation]
        d = list(o.dims) + [0.0] * (3 - len(o.dims))
        arr[i].dims[:] = [float(v) for v in d[:3]]
        if getattr(o, "vertices", None) is not None:
            v = np.ascontiguousarray(o.vertices, np.float64).reshape(-1, 3)
            keep.append(v)
            arr[i].vertices = _dp(v)
            arr[i].num_vertices = len(v)
    pts = np.ascontiguousarray(points if points is not None else np.zeros((0, 3)), np.float64).reshape(-1, 3)
    occ = np.zeros((n, n, n), np.uint8)
    field = np.zeros((n, n, n), np.uint16) if with_field else None
    origin = np.array(grid.origin, np.float64)
    marked = lib().so_sdf_build_objects(
        n, n, n, _dp(origin), grid.resolution, grid.max_expansion, arr, len(objects),
        _dp(pts if pts.size else np.zeros(3)), len(pts), occ.ctypes.data_as(C.POINTER(C.c_ubyte)),
        field.ctypes.data_as(C.POINTER(C.c_uint16)) if field is not None else None)
    if marked < 0:
        raise ValueError("so_sdf_build_objects: invalid input")
    return field, occ, int(marked)


def hull_planes(vertices) -> np.ndarray:
    """so_hull_planes: the supporting planes (nx, ny, nz, d) of the vertices' convex hull."""
    v = np.ascontiguousarray(vertices, np.float64).reshape(-1, 3)
    cap = 2 * len(v) * len(v) + 8
    out = np.zeros((cap, 4), np.float64)
    n = lib().so_hull_planes(_dp(v), len(v), _dp(out), cap)
    if n < 0:
        raise ValueError("so_hull_planes: the vertices span no volume")
    return out[:n].copy()


def sdf_from_occupancy(occ: np.ndarray, resolution: float, max_expansion: float) -> np.ndarray:
    occ = np.ascontiguousarray(occ, np.uint8)
    out = np.zeros(occ.shape, np.uint16)
    if lib().so_sdf_from_occupancy(*occ.shape, resolution, max_expansion, occ.ctypes.data_as(C.POINTER(C.c_ubyte)),
                                   out.ctypes.data_as(C.POINTER(C.c_uint16))) != 0:
        raise ValueError("so_sdf_from_occupancy: cap above 255 cells")
    return out


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _arr(vals, T):
    vals = list(vals)
    return (T * max(len(vals), 1))(*vals)


class Oracle:
    """One planning problem on the CPU oracle (keeps every buffer it points at alive)."""

    def __init__(self, problem, dense: bool = False, threads: int = 1, sum_block: int = 64, ref_arith: int = 0):
        """dense: the reference's dense N x N products (CPU baseline structure); ref_arith 1: the
        reference's written arithmetic order (non-fused L z / M eps, sequential rollout sums)
        instead of the engine's contract; 2: also Eigen 2's two-lane packet VectorXd::sum(); 3: also
        the C library's exp / sin / cos / atan2 / asin where the reference calls them."""
        L = lib()
        p = problem
        self.problem = p
        self.J, self.N, self.K = p.J, p.N, p.params.num_rollouts
        self.S = len(p.spheres)
        segs = []
        for s in p.robot.segments:
            segs.append(so_segment(s.parent, s.q_index, (C.c_double * 9)(*s.rot), (C.c_double * 3)(*s.trans),
                                   (C.c_double * 3)(*s.axis)))
        self._segs = _arr(segs, so_segment)
        self._sph = _arr([so_sphere(s.segment, s.radius, s.clearance, (C.c_double * 3)(*s.pos)) for s in p.spheres],
                         so_sphere)
        self._joints = _arr([so_joint(int(j.has_limits), j.min, j.max, j.joint_cost) for j in p.robot.joints], so_joint)
        self._sdf = np.ascontiguousarray(p.sdf, dtype=np.uint16)
        pr = p.params
        self._sig = pr.per_joint("noise_stddev", self.J)
        self._dec = pr.per_joint("noise_decay", self.J)
        self._start = np.ascontiguousarray(p.start, np.float64)
        self._goal = np.ascontiguousarray(p.goal, np.float64)
        g = p.grid
        cfg = so_config()
        cfg.num_joints, cfg.num_time_steps, cfg.num_rollouts = self.J, self.N, self.K
        cfg.num_reused_rollouts = pr.num_reused_rollouts
        cfg.num_segments = len(segs)
        cfg.segments = self._segs
        cfg.num_spheres = self.S
        cfg.spheres = self._sph
        cfg.joints = self._joints
        cfg.sdf = so_sdf(g.n, g.n, g.n, (C.c_double * 3)(*g.origin), g.resolution,
                         self._sdf.ctypes.data_as(C.POINTER(C.c_uint16)))
        cfg.discretization = pr.trajectory_discretization
        cfg.smoothness_costs = (C.c_double * 3)(pr.smoothness_cost_velocity, pr.smoothness_cost_acceleration,
                                                pr.smoothness_cost_jerk)
        cfg.ridge_factor = pr.ridge_factor
        cfg.smoothness_cost_weight = pr.smoothness_cost_weight
        cfg.obstacle_cost_weight = pr.obstacle_cost_weight
        cfg.constraint_cost_weight = pr.constraint_cost_weight
        cfg.torque_cost_weight = pr.torque_cost_weight
        cfg.noise_stddev = _dp(self._sig)
        cfg.noise_decay = _dp(self._dec)
        cfg.use_cumulative_costs = int(pr.use_cumulative_costs)
        cfg.start = _dp(self._start)
        cfg.goal = _dp(self._goal)
        cfg.seed = p.seed
        cfg.max_iterations = pr.max_iterations
        cfg.max_iterations_after_collision_free = pr.max_iterations_after_collision_free
        cfg.sum_block = sum_block
        cfg.dense = int(dense)
        cfg.threads = threads
        self._inertia = _arr([so_inertia(s.inertia.mass, (C.c_double * 3)(*s.inertia.com),
                                         (C.c_double * 6)(*s.inertia.inertia)) if s.inertia else so_inertia()
                              for s in p.robot.segments], so_inertia)
        cfg.inertias = self._inertia
        cfg.torque_root = p.robot.index(p.torque_root)
        cfg.torque_tip = p.robot.index(p.torque_tip)
        cfg.gravity = (C.c_double * 3)(*p.gravity)
        self._oc = _arr([so_orientation_constraint(p.robot.index(c.link_name), (C.c_double * 4)(*c.orientation),
                                                   0 if c.header_frame else 1, c.absolute_roll_tolerance,
                                                   c.absolute_pitch_tolerance, c.absolute_yaw_tolerance, c.weight)
                         for c in p.orientation_constraints], so_orientation_constraint)
        cfg.num_orientation_constraints = len(p.orientation_constraints)
        cfg.orientation_constraints = self._oc
        cfg.ref_arith = int(ref_arith)
        self._cfg = cfg
        self.h = L.so_create(C.byref(cfg))
        if not self.h:
            raise RuntimeError("so_create: " + L.so_last_error().decode())

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            lib().so_destroy(h)
            self.h = None

    def matrix(self, which: str, joint: int = 0) -> np.ndarray:
        n = self.N + 12 if which in ("Rall", "D0", "D1", "D2") else self.N
        out = np.zeros((n, n))
        if lib().so_get_matrix(self.h, which.encode(), joint, _dp(out)) != 0:
            raise KeyError(which)
        return out

    def theta(self) -> np.ndarray:
        out = np.zeros((self.J, self.N))
        lib().so_get_theta(self.h, _dp(out))
        return out

    def set_theta(self, theta: np.ndarray):
        t = np.ascontiguousarray(theta, np.float64)
        lib().so_set_theta(self.h, _dp(t))

    def pad_positions(self) -> np.ndarray:
        out = np.zeros((12, self.S, 3))
        lib().so_get_pad_positions(self.h, _dp(out))
        return out

    def execute(self, params: np.ndarray, iteration_member: int = 1):
        prm = np.ascontiguousarray(params, np.float64)
        costs = np.zeros(self.N)
        traj = np.zeros((self.J, self.N))
        cf, cs = C.c_int(), C.c_int()
        lib().so_execute(self.h, _dp(prm), _dp(costs), C.byref(cf), _dp(traj), iteration_member, C.byref(cs))
        self.last_constraints_satisfied = bool(cs.value)
        return costs, bool(cf.value), traj

    def iterate(self, iteration_number: int):
        o = so_iter_out()
        lib().so_iterate(self.h, iteration_number, C.byref(o))
        self.last_constraints_satisfied = bool(o.constraints_satisfied)
        return o.cost, bool(o.collision_free)

    def optimize(self):
        st = so_stats()
        costs = np.zeros(max(self.problem.params.max_iterations, 1))
        lib().so_optimize(self.h, C.byref(st), _dp(costs))
        return st, costs[: st.iterations]

    def best_trajectory(self) -> np.ndarray:
        out = np.zeros((self.J, self.N))
        lib().so_get_best_trajectory(self.h, _dp(out))
        return out

    def best_torques(self) -> np.ndarray:
        out = np.zeros(self.N)
        if lib().so_get_best_torques(self.h, _dp(out)) != 0:
            raise RuntimeError(lib().so_last_error().decode())
        return out

    def last_trajectory(self) -> np.ndarray:
        out = np.zeros((self.J, self.N))
        lib().so_get_last_trajectory(self.h, _dp(out))
        return out

    def rollouts(self, which: str) -> np.ndarray:
        if which.startswith("x_"):
            shape = (self.N,) if which == "x_state_costs" else (self.J, self.N)
        else:
            shape = (self.K, self.N) if which == "state_costs" else (self.K, self.J, self.N)
        out = np.zeros(shape)
        if lib().so_get_rollouts(self.h, which.encode(), _dp(out)) != 0:
            raise KeyError(which)
        return out

    def reuse_log(self) -> np.ndarray:
        """[rankings][num_reused_rollouts] candidate indices kept by every reuse ranking so far
        (-1 = the extra rollout), in generateRollouts' order (policy_improvement.cpp:198-224)."""
        kr = max(int(self.problem.params.num_reused_rollouts), 1)
        n = lib().so_reuse_log(self.h, None, 0)
        out = np.zeros(max(n, 1), np.int32)
        lib().so_reuse_log(self.h, out.ctypes.data_as(C.POINTER(C.c_int)), n)
        return out[:n].reshape(-1, kr)

    def sphere_positions(self, q) -> np.ndarray:
        qq = np.ascontiguousarray(q, np.float64)
        out = np.zeros((self.S, 3))
        lib().so_sphere_positions(self.h, _dp(qq), _dp(out))
        return out

    def inverse_dynamics(self, q, qd, qdd) -> np.ndarray:
        a = [np.ascontiguousarray(v, np.float64) for v in (q, qd, qdd)]
        tau = np.zeros(self.J)
        if lib().so_inverse_dynamics(self.h, _dp(a[0]), _dp(a[1]), _dp(a[2]), _dp(tau)) != 0:
            raise RuntimeError("torque term off")
        return tau

    def sdf_distance(self, x, y, z) -> float:
        return lib().so_sdf_distance(self.h, x, y, z)

    def potential(self, sphere: int, pos):
        p = np.ascontiguousarray(pos, np.float64)
        v = np.zeros(1)
        col = lib().so_potential(self.h, sphere, _dp(p), _dp(v))
        return float(v[0]), bool(col)


def normals(seed: int, iteration: int, joint: int, rollout: int, n: int) -> np.ndarray:
    z = np.zeros(n)
    lib().so_normals(seed, iteration, joint, rollout, n, _dp(z))
    return z


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().so_philox4x32(c, k, o)
    return list(o)


def diff_rules() -> np.ndarray:
    out = np.zeros((3, 7))
    lib().so_diff_rules(_dp(out))
    return out


def dexp(x: float) -> float:
    return lib().so_exp(x)


def dlog(x: float) -> float:
    return lib().so_log(x)


def datan2(y: float, x: float) -> float:
    return lib().so_atan2(y, x)


def dasin(x: float) -> float:
    return lib().so_asin(x)


def dsincos(x: float):
    s, c = C.c_double(), C.c_double()
    lib().so_sincos(x, C.byref(s), C.byref(c))
    return s.value, c.value
