"""Synthetic planning problems for the STOMP engine (host-side setup data).

The reference builds its robot model from the PR2 URDF through kdl_parser
(stomp_robot_model.cpp:81-86), its collision spheres by the link-radius rule
(stomp_robot_model.cpp:265-306) and its distance field from the shelf / pole
scenes (config/environment_shelf.yaml:4-64, environment_pole.yaml:4-10) through
arm_navigation's PropagationDistanceField (stomp_collision_space.cpp:60-197).
None of that is available here (no URDF, ROS or KDL), so this module provides:

* ``pr2like7`` / ``pr2like14``: PR2-like kinematic trees (7-DOF right arm, and a
  14-DOF two-arm tree on a shared torso) with PR2 link offsets and joint limits,
  as a flat segment table in DFS order (the layout the engine consumes);
* ``make_spheres``: the reference's sphere rule, radii/extension/clearance from
  config/pr2_both_arms_stomp_config.yaml:1-39;
* ``build_sdf``: the capped, quantised distance field
  ``sqrt(min(d2, ceil(max_expansion/res)^2)) * res`` where d2 is the integer
  squared voxel distance to the nearest obstacle voxel (exact EDT), fp32;
* ``StompParameters``: the reference's parameter names and params.yaml values.
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Optional, Sequence

import numpy as np

PAD = 6  # DIFF_RULE_LENGTH - 1 (stomp_utils.h:47)


@dataclasses.dataclass
class Segment:
    name: str
    parent: int
    q_index: int  # -1 for a fixed segment
    trans: Sequence[float]
    axis: Sequence[float] = (0.0, 0.0, 1.0)
    rot: Sequence[float] = (1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0)
    inertia: Optional["Inertia"] = None   # None: massless


@dataclasses.dataclass
class Joint:
    name: str
    has_limits: bool
    min: float = 0.0
    max: float = 0.0
    joint_cost: float = 1.0


@dataclasses.dataclass
class Sphere:
    segment: int
    radius: float
    clearance: float
    pos: Sequence[float]
    link: str = ""


@dataclasses.dataclass
class Inertia:
    """KDL::RigidBodyInertia(m, cog, Ic) of a segment, in the segment frame; Ic about the
    centre of mass as (Ixx, Iyy, Izz, Ixy, Ixz, Iyz)."""
    mass: float
    com: Sequence[float] = (0.0, 0.0, 0.0)
    inertia: Sequence[float] = (0.0, 0.0, 0.0, 0.0, 0.0, 0.0)


@dataclasses.dataclass
class OrientationConstraint:
    """motion_planning_msgs::OrientationConstraint as consumed by
    OrientationConstraintEvaluator (constraint_evaluator.cpp:50-73)."""
    link_name: str
    orientation: Sequence[float]  # quaternion (x, y, z, w)
    header_frame: bool = False    # type == HEADER_FRAME (else body-fixed)
    absolute_roll_tolerance: float = math.pi
    absolute_pitch_tolerance: float = math.pi
    absolute_yaw_tolerance: float = math.pi
    weight: float = 1.0


@dataclasses.dataclass
class Robot:
    segments: List[Segment]
    joints: List[Joint]
    sphere_links: List[tuple]  # (link name, radius, extension) in GroupLinkUnion order

    def children(self, s: int) -> List[int]:
        return [i for i, g in enumerate(self.segments) if g.parent == s]

    def index(self, name: str) -> int:
        for i, g in enumerate(self.segments):
            if g.name == name:
                return i
        raise KeyError(name)


# collision_links of config/pr2_both_arms_stomp_config.yaml:3-31 (right arm part)
_LINK_RADII = [
    ("upper_arm_link", 0.10, 0.0),
    ("forearm_link", 0.065, 0.0),
    ("gripper_palm_link", 0.06, 0.0),
    ("gripper_l_finger_link", 0.03, 0.01),
    ("gripper_l_finger_tip_link", 0.03, 0.01),
    ("gripper_r_finger_link", 0.03, 0.01),
    ("gripper_r_finger_tip_link", 0.03, 0.01),
]
COLLISION_CLEARANCE = 0.07  # pr2_both_arms_stomp_config.yaml:1


# Synthetic PR2-like link inertias (mass kg, centre of mass m, inertia about it kg m^2).  The
# PR2 URDF is not in the container; the masses follow the published PR2 arm figures and the
# centres / inertias are rod-like estimates, so the torque term is exercised on a realistic
# scale.  Links not listed (finger links, tool frame) are massless.
_LINK_INERTIA = {
    "shoulder_pan_link": Inertia(25.8, (-0.032, 0.0, -0.27), (0.866, 0.874, 0.273, -0.006, 0.121, -0.059)),
    "shoulder_lift_link": Inertia(2.75, (0.0, 0.0, 0.0), (0.021, 0.021, 0.020, 0.0, 0.0, 0.0)),
    "upper_arm_roll_link": Inertia(0.1, (0.0, 0.0, 0.0), (0.01, 0.01, 0.01, 0.0, 0.0, 0.0)),
    "upper_arm_link": Inertia(6.01, (0.216, 0.0, -0.0003), (0.015, 0.0747, 0.0761, -0.0012, 0.0087, -0.0001)),
    "elbow_flex_link": Inertia(1.9, (0.01, 0.0, -0.012), (0.0035, 0.0044, 0.0031, 0.0, 0.0001, 0.0)),
    "forearm_roll_link": Inertia(0.1, (0.0, 0.0, 0.0), (0.01, 0.01, 0.01, 0.0, 0.0, 0.0)),
    "forearm_link": Inertia(2.57, (0.181, 0.0, 0.0), (0.0037, 0.0150, 0.0166, 0.0001, 0.0, 0.0)),
    "wrist_flex_link": Inertia(0.61, (-0.0016, 0.0, 0.0), (0.0007, 0.0007, 0.0006, 0.0, 0.0, 0.0)),
    "wrist_roll_link": Inertia(0.1, (0.0, 0.0, 0.0), (0.01, 0.01, 0.01, 0.0, 0.0, 0.0)),
    "gripper_palm_link": Inertia(0.58, (0.06, 0.0, 0.0), (0.0004, 0.0011, 0.0010, 0.0, 0.0, 0.0)),
}


def _set_inertia(segs, name: str, sign: float, inertia: Inertia):
    for s in segs:
        if s.name == name:
            c = (inertia.com[0], sign * inertia.com[1], inertia.com[2])
            i = inertia.inertia
            s.inertia = Inertia(inertia.mass, c, (i[0], i[1], i[2], sign * i[3], i[4], sign * i[5]))
            return
    raise KeyError(name)


def _arm(prefix: str, sign: float, parent: int, q0: int, segs: List[Segment], joints: List[Joint]):
    """PR2 arm chain below the torso (PR2 URDF offsets)."""
    def add(name, q, trans, axis=(0.0, 0.0, 1.0), par=None):
        segs.append(Segment(prefix + name, len(segs) - 1 if par is None else par, q, trans, axis))
        return len(segs) - 1

    add("shoulder_pan_link", q0 + 0, (0.0, sign * -0.188, 0.0), (0.0, 0.0, 1.0), par=parent)
    add("shoulder_lift_link", q0 + 1, (0.1, 0.0, 0.0), (0.0, 1.0, 0.0))
    add("upper_arm_roll_link", q0 + 2, (0.0, 0.0, 0.0), (1.0, 0.0, 0.0))
    add("upper_arm_link", -1, (0.0, 0.0, 0.0))
    add("elbow_flex_link", q0 + 3, (0.4, 0.0, 0.0), (0.0, 1.0, 0.0))
    add("forearm_roll_link", q0 + 4, (0.0, 0.0, 0.0), (1.0, 0.0, 0.0))
    add("forearm_link", -1, (0.0, 0.0, 0.0))
    add("wrist_flex_link", q0 + 5, (0.321, 0.0, 0.0), (0.0, 1.0, 0.0))
    add("wrist_roll_link", q0 + 6, (0.0, 0.0, 0.0), (1.0, 0.0, 0.0))
    palm = add("gripper_palm_link", -1, (0.0, 0.0, 0.0))
    lf = add("gripper_l_finger_link", -1, (0.07691, 0.01, 0.0), par=palm)
    add("gripper_l_finger_tip_link", -1, (0.09137, 0.00495, 0.0), par=lf)
    rf = add("gripper_r_finger_link", -1, (0.07691, -0.01, 0.0), par=palm)
    add("gripper_r_finger_tip_link", -1, (0.09137, -0.00495, 0.0), par=rf)
    add("gripper_tool_frame", -1, (0.18, 0.0, 0.0), par=palm)
    for name, inertia in _LINK_INERTIA.items():
        _set_inertia(segs, prefix + name, sign, inertia)
    if sign > 0:  # right arm limits (PR2 URDF)
        lim = [(-2.2853981634, 0.714601836603), (-0.5236, 1.3963), (-3.9, 0.8), (-2.3213, 0.0),
               None, (-2.18, 0.0), None]
    else:  # left arm: pan and upper-arm roll mirrored
        lim = [(-0.714601836603, 2.2853981634), (-0.5236, 1.3963), (-0.8, 3.9), (-2.3213, 0.0),
               None, (-2.18, 0.0), None]
    names = ["shoulder_pan_joint", "shoulder_lift_joint", "upper_arm_roll_joint", "elbow_flex_joint",
             "forearm_roll_joint", "wrist_flex_joint", "wrist_roll_joint"]
    for n, l in zip(names, lim):
        if l is None:  # continuous joints wrap around (stomp_robot_model.cpp:160-161)
            joints.append(Joint(prefix + n, False))
        else:
            joints.append(Joint(prefix + n, True, l[0], l[1]))


def pr2like7(torso_z: float = 0.9) -> Robot:
    """PR2-like right arm: base_footprint -> torso_lift_link -> 7 revolute joints -> gripper."""
    segs = [Segment("base_footprint", -1, -1, (0.0, 0.0, 0.0)),
            Segment("torso_lift_link", 0, -1, (-0.05, 0.0, torso_z))]
    joints: List[Joint] = []
    _arm("r_", 1.0, 1, 0, segs, joints)
    return Robot(segs, joints, [("r_" + n, r, e) for n, r, e in _LINK_RADII])


def pr2like14(torso_z: float = 0.9) -> Robot:
    """Two PR2-like arms on a shared torso (right arm joints 0..6, left arm 7..13)."""
    segs = [Segment("base_footprint", -1, -1, (0.0, 0.0, 0.0)),
            Segment("torso_lift_link", 0, -1, (-0.05, 0.0, torso_z))]
    joints: List[Joint] = []
    _arm("r_", 1.0, 1, 0, segs, joints)
    _arm("l_", -1.0, 1, 7, segs, joints)
    links = [("r_" + n, r, e) for n, r, e in _LINK_RADII] + [("l_" + n, r, e) for n, r, e in _LINK_RADII]
    return Robot(segs, joints, links)


def make_spheres(robot: Robot, clearance: float = COLLISION_CLEARANCE) -> List[Sphere]:
    """StompRobotModel::addCollisionPointsFromLinkRadius (stomp_robot_model.cpp:265-306).

    For each child of the link: spacing = r/2, distance = |child joint origin| +
    extension, n = ceil(distance/spacing) + 1, points at origin * i/(n-1) (the
    extension only changes n), the origin point only for the first child.
    """
    out: List[Sphere] = []
    for link, radius, ext in robot.sphere_links:
        s = robot.index(link)
        first_child = True
        for c in robot.children(s):
            o = np.array(robot.segments[c].trans, dtype=np.float64)
            spacing = radius / 2.0
            distance = math.sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]) + ext
            n = int(math.ceil(distance / spacing)) + 1
            for i in range(n):
                if not first_child and i == 0:
                    continue
                f = float(i / (n - 1.0))
                out.append(Sphere(s, radius, clearance, (o[0] * f, o[1] * f, o[2] * f), link))
            first_child = False
    return out


# ----------------------------------------------------------------- scene + SDF

@dataclasses.dataclass
class Box:  # axis-aligned, centre + full dimensions (environment_shelf.yaml)
    center: Sequence[float]
    dims: Sequence[float]


@dataclasses.dataclass
class Cylinder:  # z-aligned, centre + (radius, length) (environment_pole.yaml)
    center: Sequence[float]
    radius: float
    length: float


def shelf_scene(with_pole: bool = True):
    """config/environment_shelf.yaml:4-64 (10 boxes, /base_footprint) and the pole of
    environment_pole.yaml:4-10 (in /base_link, 0.051 m above /base_footprint)."""
    boxes = [Box((0.8, -0.1, z), (0.4, 1.2, 0.03)) for z in (0.015, 0.329, 0.643, 0.957, 1.271, 1.585)]
    boxes += [Box((0.8, y, 0.8), (0.4, 0.03, 1.6)) for y in (-0.685, -0.295, 0.095, 0.485)]
    cyls = [Cylinder((0.62, -0.62, 0.6 + 0.051), 0.1, 1.2)] if with_pole else []
    return boxes, cyls


# collision-space objects as the reference's voxeliser takes them (stomp_engine.h STOMP_SHAPE_* /
# STOMP_BODY_*; stomp_collision_space.cpp:199-297, 592-650)
SHAPE_BOX, SHAPE_CYLINDER, BODY_SPHERE, BODY_BOX, BODY_CYLINDER, BODY_MESH = 0, 1, 2, 3, 4, 5


@dataclasses.dataclass
class SceneObject:
    type: int
    position: Sequence[float]
    orientation: Sequence[float] = (0.0, 0.0, 0.0, 1.0)   # quaternion x, y, z, w
    dims: Sequence[float] = (0.0, 0.0, 0.0)
    vertices: Optional[np.ndarray] = None   # BODY_MESH: V x 3 in the body frame, scaled; dims[0] = padding


def quaternion_from_rpy(roll: float, pitch: float, yaw: float):
    """btQuaternion::setRPY, as test_collision_world.cpp:180-185 turns a scene file's
    orientation [roll, pitch, yaw] into the object's pose quaternion (x, y, z, w)."""
    hy, hp, hr = yaw * 0.5, pitch * 0.5, roll * 0.5
    cy, sy, cp, sp, cr, sr = math.cos(hy), math.sin(hy), math.cos(hp), math.sin(hp), math.cos(hr), math.sin(hr)
    return (sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
            cr * cp * cy + sr * sp * sy)


def shelf_objects(with_pole: bool = True) -> List[SceneObject]:
    """The shelf + pole scene (shelf_scene) as collision objects with the scene files' poses
    (environment_shelf.yaml:4-64, environment_pole.yaml:4-10; orientation [0, 0, 0])."""
    boxes, cyls = shelf_scene(with_pole)
    q = quaternion_from_rpy(0.0, 0.0, 0.0)
    out = [SceneObject(SHAPE_BOX, tuple(b.center), q, tuple(b.dims)) for b in boxes]
    out += [SceneObject(SHAPE_CYLINDER, tuple(c.center), q, (c.radius, c.length, 0.0)) for c in cyls]
    return out


def mesh_object(vertices, triangles=None, position=(0.0, 0.0, 0.0), rpy=(0.0, 0.0, 0.0), scale=(1.0, 1.0, 1.0),
                padding: float = 0.0) -> SceneObject:
    """A MESH collision object as the reference's scene files give one (environment_mesh.yaml:
    position, orientation [roll, pitch, yaw], scale): bodies::ConvexMesh of the scaled vertices
    (the triangles do not enter the convex hull)."""
    v = np.asarray(vertices, np.float64).reshape(-1, 3) * np.asarray(scale, np.float64)[None, :]
    return SceneObject(BODY_MESH, tuple(float(x) for x in position), quaternion_from_rpy(*rpy), (padding, 0.0, 0.0),
                       np.ascontiguousarray(v))


@dataclasses.dataclass
class Grid:
    n: int                    # cells per axis (cube)
    origin: Sequence[float]
    resolution: float
    max_expansion: float

    @property
    def max_dist_int(self) -> int:
        return int(math.ceil(self.max_expansion / self.resolution))


def default_grid(n: int, max_expansion: float = 0.17, edge: float = 2.0, origin=(-0.5, -1.0, -0.3)) -> Grid:
    return Grid(n, tuple(origin), edge / n, max_expansion)


def _box_range(lo: float, hi: float, o: float, res: float, n: int):
    i0 = max(int(math.ceil((lo - o) / res)), 0)
    i1 = min(int(math.floor((hi - o) / res)), n - 1)
    return i0, i1


def _axis_d2(i0: int, i1: int, n: int) -> np.ndarray:
    i = np.arange(n, dtype=np.int64)
    d = np.maximum(np.maximum(i0 - i, 0), i - i1)
    return d * d


def cylinder_disc_d2(c: Cylinder, grid: Grid) -> np.ndarray:
    """Integer squared distance (in the xy plane) from every cell column to the
    nearest cell column whose centre lies inside the disc; -1 rows if empty."""
    n, res = grid.n, grid.resolution
    ox, oy = grid.origin[0], grid.origin[1]
    xs = ox + np.arange(n, dtype=np.float64) * res - c.center[0]
    ys = oy + np.arange(n, dtype=np.float64) * res - c.center[1]
    inside = (xs[:, None] * xs[:, None] + ys[None, :] * ys[None, :]) <= c.radius * c.radius
    pi, pj = np.nonzero(inside)
    big = np.int64(1) << 40
    out = np.full((n, n), big, dtype=np.int64)
    if len(pi) == 0:
        return out
    ii = np.arange(n, dtype=np.int64)
    for a, b in zip(pi, pj):
        dx = (ii - a) ** 2
        dy = (ii - b) ** 2
        np.minimum(out, dx[:, None] + dy[None, :], out=out)
    return out


def build_sdf(grid: Grid, boxes, cylinders) -> np.ndarray:
    """Capped distance field as squared cell distances: uint16 d2 = min(d2, cap^2), shape (n, n, n),
    index [x, y, z] (z fastest).  The distance of a cell is sqrt(d2) * res (sdf_metres): the
    integer distance_square_ and sqrt_table_ of PropagationDistanceField."""
    n, res = grid.n, grid.resolution
    cap = grid.max_dist_int
    cap2 = cap * cap
    d2 = np.full((n, n, n), cap2, dtype=np.int64)
    o = grid.origin
    for b in boxes:
        rngs = []
        for a in range(3):
            lo = b.center[a] - b.dims[a] / 2.0
            hi = b.center[a] + b.dims[a] / 2.0
            rngs.append(_box_range(lo, hi, o[a], res, n))
        if any(r[0] > r[1] for r in rngs):
            continue
        dx, dy, dz = (_axis_d2(r[0], r[1], n) for r in rngs)
        np.minimum(d2, dx[:, None, None] + dy[None, :, None] + dz[None, None, :], out=d2)
    for c in cylinders:
        z0, z1 = _box_range(c.center[2] - c.length / 2.0, c.center[2] + c.length / 2.0, o[2], res, n)
        if z0 > z1:
            continue
        dxy = cylinder_disc_d2(c, grid)
        if dxy.min() >= (np.int64(1) << 40):
            continue
        dz = _axis_d2(z0, z1, n)
        np.minimum(d2, np.minimum(dxy[:, :, None] + dz[None, None, :], cap2), out=d2)
    if cap2 > 65535:
        raise ValueError("max_expansion / resolution above 255 cells: d2 does not fit 16 bits")
    return np.minimum(d2, cap2).astype(np.uint16)


def sdf_metres(grid: Grid, d2: np.ndarray) -> np.ndarray:
    """Distance in metres of squared cell distances: sqrt(double(d2)) * resolution, PropagationDistanceField's
    sqrt_table_ (third party; call site stomp_collision_space.h:187-191)."""
    return np.sqrt(np.asarray(d2, np.float64)) * grid.resolution


# ----------------------------------------------------------------- parameters

@dataclasses.dataclass
class StompParameters:
    """config/params.yaml + StompParameters defaults (stomp_parameters.cpp:50-76)."""
    trajectory_duration: float = 5.0
    trajectory_discretization: float = 0.05
    max_iterations: int = 500
    max_iterations_after_collision_free: int = 500
    smoothness_cost_velocity: float = 0.0
    smoothness_cost_acceleration: float = 1.0
    smoothness_cost_jerk: float = 0.0
    smoothness_cost_weight: float = 0.000001
    obstacle_cost_weight: float = 1.0
    constraint_cost_weight: float = 0.2
    torque_cost_weight: float = 0.0
    ridge_factor: float = 0.0
    use_cumulative_costs: bool = False
    num_rollouts: int = 10
    num_reused_rollouts: int = 5
    noise_stddev: object = 2.0     # one value for every joint, or a per-joint list (params.yaml:19-26)
    noise_decay: object = 0.999

    def per_joint(self, name: str, J: int) -> np.ndarray:
        """noise_stddev / noise_decay as the J-vector PolicyImprovementLoop reads
        (policy_improvement_loop.cpp:99-100); a list must have one entry per joint."""
        v = np.asarray(getattr(self, name), np.float64)
        if v.ndim == 0:
            return np.full(J, float(v))
        if v.shape != (J,):
            raise ValueError(f"{name} has {v.size} entries for {J} joints")
        return v.copy()

    @property
    def num_time_steps(self) -> int:
        # full trajectory has duration/discretization + 1 points (stomp_trajectory.cpp:48),
        # of which all but the first and last are free (:52-53)
        return int(self.trajectory_duration / self.trajectory_discretization + 1) - 2


# start/goal for the shelf scene: hand inside the cell at z=0.486 (start) and the
# cell at z=0.8 (goal), same column; the min-acceleration interpolant passes
# through the plank at z=0.643.  Found by tools/find_start_goal.py (seeded search).
SHELF_START_7 = [0.6348, 1.2798, 0.8, -1.2668, -1.1205, -0.1563, -3.1085]
SHELF_GOAL_7 = [-0.3308, -0.2633, -2.2194, -1.8965, -3.1416, -1.4767, -0.3451]


@dataclasses.dataclass
class Problem:
    robot: Robot
    spheres: List[Sphere]
    grid: Grid
    boxes: list
    cylinders: list
    params: StompParameters
    start: np.ndarray
    goal: np.ndarray
    seed: int = 0x53544F4D50000000
    sdf: Optional[np.ndarray] = None
    # inverse-dynamics chain of the torque term: KDL getChain("torso_lift_link",
    # "r_gripper_tool_frame") with gravity (0, 0, -9.8) (stomp_robot_model.cpp:185-189)
    torque_root: str = "torso_lift_link"
    torque_tip: str = "r_gripper_tool_frame"
    gravity: Sequence[float] = (0.0, 0.0, -9.8)
    orientation_constraints: List[OrientationConstraint] = dataclasses.field(default_factory=list)

    def torque_chain(self) -> List[int]:
        """Segment indices of the chain root (exclusive) -> tip (inclusive), root side first."""
        r, s = self.robot.index(self.torque_root), self.robot.index(self.torque_tip)
        out = []
        while s != r:
            if s < 0:
                raise ValueError("torque tip is not below the torque root")
            out.append(s)
            s = self.robot.segments[s].parent
        return out[::-1]

    @property
    def J(self) -> int:
        return len(self.robot.joints)

    @property
    def N(self) -> int:
        return self.params.num_time_steps


def make_problem(dof: int = 7, waypoints: int = 100, grid_n: int = 64, num_rollouts: int = 10,
                 num_reused_rollouts: int = 5, build_grid: bool = True, seed: Optional[int] = None,
                 with_pole: bool = True, start=None, goal=None, orientation_constraints=None,
                 **param_overrides) -> Problem:
    robot = pr2like7() if dof == 7 else pr2like14()
    spheres = make_spheres(robot)
    max_exp = max(s.radius + s.clearance for s in spheres)
    grid = default_grid(grid_n, max_exp)
    boxes, cyls = shelf_scene(with_pole)
    duration = 5.0 if waypoints == 100 else (waypoints * 0.05)
    params = StompParameters(trajectory_duration=duration, num_rollouts=num_rollouts,
                             num_reused_rollouts=num_reused_rollouts, **param_overrides)
    if start is None:
        start = SHELF_START_7 if dof == 7 else SHELF_START_7 + _mirror(SHELF_START_7)
    if goal is None:
        goal = SHELF_GOAL_7 if dof == 7 else SHELF_GOAL_7 + _mirror(SHELF_GOAL_7)
    p = Problem(robot, spheres, grid, boxes, cyls, params, np.array(start, np.float64), np.array(goal, np.float64))
    if seed is not None:
        p.seed = seed
    if orientation_constraints:
        p.orientation_constraints = list(orientation_constraints)
    if build_grid:
        p.sdf = build_sdf(grid, boxes, cyls)
    return p


def upright_constraint(link: str = "r_gripper_tool_frame") -> OrientationConstraint:
    """The reference's upright path constraint (test/test_omp.cpp:76-91): HEADER_FRAME, identity
    nominal orientation, roll / pitch within 0.2 rad, yaw free (tolerance 10 >= pi), weight 1."""
    return OrientationConstraint(link, (0.0, 0.0, 0.0, 1.0), header_frame=True, absolute_roll_tolerance=0.2,
                                 absolute_pitch_tolerance=0.2, absolute_yaw_tolerance=10.0, weight=1.0)


def _mirror(q):
    # left arm mirrored through the xz plane: pan and the roll joints change sign
    return [-q[0], q[1], -q[2], q[3], -q[4], q[5], -q[6]]


# ----------------------------------------------------------------- numpy FK (host reference)

def rot2(axis, angle):
    """KDL Rotation::Rot2 (orocos KDL frames.cpp), libm sin/cos."""
    a = axis
    ct, st = math.cos(angle), math.sin(angle)
    vt = 1.0 - ct
    m0, m1, m2 = vt * a[0], vt * a[1], vt * a[2]
    s0, s1, s2 = a[0] * st, a[1] * st, a[2] * st
    m01, m02, m12 = m0 * a[1], m0 * a[2], m1 * a[2]
    return np.array([[ct + m0 * a[0], -s2 + m01, s1 + m02],
                     [s2 + m01, ct + m1 * a[1], -s0 + m12],
                     [-s1 + m02, s0 + m12, ct + m2 * a[2]]])


def fk_frames(robot: Robot, q) -> list:
    frames = []
    for s in robot.segments:
        R = np.array(s.rot, dtype=np.float64).reshape(3, 3)
        if s.q_index >= 0:
            R = R @ rot2(s.axis, q[s.q_index])
        p = np.array(s.trans, dtype=np.float64)
        if s.parent >= 0:
            PR, Pp = frames[s.parent]
            R, p = PR @ R, PR @ p + Pp
        frames.append((R, p))
    return frames


def sphere_positions(robot: Robot, spheres: List[Sphere], q) -> np.ndarray:
    fr = fk_frames(robot, q)
    return np.array([fr[s.segment][0] @ np.array(s.pos) + fr[s.segment][1] for s in spheres])


def c_round(x):
    """C round(): halves away from zero (numpy's round is half-to-even)."""
    t = np.trunc(x)
    return np.where(np.abs(x - t) >= 0.5, t + np.sign(x), t)


def sdf_lookup(p: Problem, pos: np.ndarray) -> np.ndarray:
    g = p.grid
    f = c_round((pos - np.array(g.origin)) * (1.0 / g.resolution))
    ok = np.all((f >= 1) & (f < g.n - 1), axis=-1)
    idx = np.where(ok[..., None], f, 0).astype(np.int64)
    d = sdf_metres(g, p.sdf[idx[..., 0], idx[..., 1], idx[..., 2]])
    return np.where(ok, d, 0.0)
