"""Synthetic random-obstacle worlds for the Kinova Gen3.

A world is (q0, qd0, qdd0, q_des, obstacles[O,12]) exactly as the reference's planner input
(KPR/README.md:99-112, KPR/armour_main.cu:54-77): an obstacle row is the zonotope
[center(3), g1(3), g2(3), g3(3)], i.e. MATLAB's Z = [c, G] reshaped column-major
(KSI/uarmtd_planner.m:189).

Generator (seeded, numpy PCG64):
  * q0 uniform inside the joint limits (continuous joints in [-pi, pi], revolute joints with a
    0.2 rad margin), qd0 ~ U(-0.25, 0.25) * speed_limit, qdd0 ~ U(-0.5, 0.5) rad/s^2 (half the
    SURVEY §8(d) ranges: at the full ranges ~1/3 of the worlds violate the torque limits already
    at k = 0, i.e. are infeasible before any obstacle is placed),
    q_des = q0 + U(-1, 1) * pi/48 * 0.8 (KSI/kinova_world_static.m:134-138, 246-248);
  * box obstacles with side lengths ~ U(0.01, 0.5) per axis (kinova_world_static.m:7, 297-298),
    centres ~ U over [-1,1] x [-1,1] x [0,2] shrunk by half the largest side
    (SCR/kinova_run_100_worlds.m:157, kinova_world_static.m:289-294), generators diag(side/2)
    (SIM/worlds/obstacles/box_obstacle_zonotope.m:21-26);
  * obstacles that intersect the arm's start configuration are rejected (bounding-sphere test
    against the FK of the link boxes at q0), so worlds are not trivially infeasible.
"""
from __future__ import annotations

import numpy as np

from .robots import KINOVA, Robot


def _rpy(r, p, y):
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    return np.array([
        [cp * cy, -cp * sy, sp],
        [cr * sy + cy * sp * sr, cr * cy - sp * sr * sy, -cp * sr],
        [sr * sy - cr * cy * sp, cy * sr + cr * sp * sy, cp * cr],
    ])


def _rot(axis, q):
    c, s = np.cos(q), np.sin(q)
    if axis == 1:
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == 2:
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    if axis == 3:
        return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
    return np.eye(3)


def link_spheres(robot: Robot, q: np.ndarray):
    """Point forward kinematics of the link boxes (the PZ FK of KPR/Dynamics.cu:69-81 at k fixed,
    no error terms): returns (centres[NJ,3], radii[NJ]) of bounding spheres."""
    R = np.eye(3)
    p = np.zeros(3)
    cs, rs = [], []
    for i in range(robot.num_joints):
        p = p + R @ robot.trans[i]
        R = R @ _rpy(*robot.rots[i])
        if robot.axes[i] != 0 and i < len(q):
            R = R @ _rot(abs(robot.axes[i]), q[i])
        cs.append(p + R @ robot.link_c[i])
        rs.append(float(np.linalg.norm(robot.link_g[i])))
    return np.array(cs), np.array(rs)


PROFILES = ("default", "survey")


def make_world(seed: int, num_obstacles: int, robot: Robot = KINOVA, profile: str = "default"):
    """profile "default": the generator above (half ranges, 5 cm clearance at the start);
    "survey": SURVEY §8(d) exactly — qd0 ~ U(-0.5, 0.5) * speed_limit, qdd0 ~ U(-1, 1), obstacles
    rejected only when they intersect the start configuration (no clearance margin). About a third
    of the "survey" worlds are over the torque limits at k = 0."""
    if profile not in PROFILES:
        raise ValueError(f"unknown world profile {profile!r}")
    rng = np.random.default_rng(seed)
    n = 7
    lb = np.where(robot.state_lb < -100, -np.pi, robot.state_lb + 0.2)
    ub = np.where(robot.state_ub > 100, np.pi, robot.state_ub - 0.2)
    q0 = rng.uniform(lb, ub)
    f = 1.0 if profile == "survey" else 0.5
    margin = 0.0 if profile == "survey" else 0.05
    qd0 = rng.uniform(-0.5 * f, 0.5 * f, n) * robot.speed_limits
    qdd0 = rng.uniform(-f, f, n)
    q_des = q0 + rng.uniform(-1.0, 1.0, n) * (np.pi / 48) * 0.8
    centres, radii = link_spheres(robot, q0)
    obs = []
    tries = 0
    while len(obs) < num_obstacles:
        tries += 1
        side = rng.uniform(0.01, 0.5, 3)
        half = side.max() / 2
        lo = np.array([-1.0, -1.0, 0.0]) + half
        hi = np.array([1.0, 1.0, 2.0]) - half
        c = rng.uniform(lo, hi)
        if tries < 100000:
            r_obs = float(np.linalg.norm(side / 2))
            if np.any(np.linalg.norm(centres - c, axis=1) < radii + r_obs + margin):
                continue
        g = np.diag(side / 2)
        obs.append(np.concatenate([c, g[:, 0], g[:, 1], g[:, 2]]))
    obstacles = np.array(obs, dtype=np.float64).reshape(num_obstacles, 12)
    return q0, qd0, qdd0, q_des, obstacles


# The commented example input of KPR/armour_main.cu:19-34 (10 box obstacles)
EXAMPLE_Q0 = np.array([0.6543, -0.0876, -0.4837, -1.2278, -1.5735, -1.0720, 0.0])
EXAMPLE_QDES = np.array([0.6831, 0.009488, -0.2471, -0.9777, -1.414, -0.9958, 0.0])
_EX_ROWS = [
    [-0.28239, -0.33281, 0.88069, 0.069825, 0, 0, 0, 0.09508, 0, 0, 0, 0.016624],
    [-0.19033, 0.035391, 1.3032, 0.11024, 0, 0, 0, 0.025188, 0, 0, 0, 0.014342],
    [0.67593, -0.085841, 0.43572, 0.17408, 0, 0, 0, 0.07951, 0, 0, 0, 0.18012],
    [0.75382, 0.51895, 0.4731, 0.030969, 0, 0, 0, 0.22312, 0, 0, 0, 0.22981],
    [0.75382, 0.51895, 0.4731, 0.030969, 0, 0, 0, 0.22312, 0, 0, 0, 0.22981],
]
EXAMPLE_OBSTACLES = np.array(_EX_ROWS + _EX_ROWS, dtype=np.float64)


def example_world():
    z = np.zeros(7)
    return EXAMPLE_Q0.copy(), z.copy(), z.copy(), EXAMPLE_QDES.copy(), EXAMPLE_OBSTACLES.copy()


def straight_line_waypoint(q_cur, q_goal, lookahead=0.1, robot: Robot = KINOVA):
    """q_des of the straight-line high-level planner (simulator/planners/high_level_planners/
    robot_arm_straight_line_HLP.m:45-57; lookahead 0.1 as kinova_src/scripts/
    kinova_run_100_worlds.m:57): a step of `lookahead` toward the goal, angle-wrapped on the
    continuous joints."""
    q_cur = np.asarray(q_cur, dtype=np.float64)
    d = np.asarray(q_goal, dtype=np.float64) - q_cur
    cont = robot.state_lb <= -1000.0
    d[cont] = (d[cont] + np.pi) % (2 * np.pi) - np.pi
    return q_cur + lookahead * d / np.linalg.norm(d)


def csv_world(rows, robot: Robot = KINOVA):
    """Planning problem of a saved world (kinova_src/saved_worlds/random/*.csv, read as
    kinova_simulator_interfaces/kinova_scenarios/load_saved_world.m: row 1 start, row 2 goal,
    rows 4.. box obstacles [centre(3), side lengths(3)]): the first replan from rest with the
    straight-line waypoint as q_des. Obstacles become zonotopes with generators diag(side / 2)
    (simulator/worlds/obstacles/box_obstacle_zonotope.m)."""
    rows = np.asarray(rows, dtype=np.float64)
    start, goal = rows[0, :7], rows[1, :7]
    obs = []
    for r in rows[3:]:
        c, side = r[:3], r[3:6]
        obs.append(np.concatenate([c, np.diag(side / 2).T.reshape(-1)]))
    z = np.zeros(7)
    return start.copy(), z.copy(), z.copy(), straight_line_waypoint(start, goal, robot=robot), np.array(obs)
