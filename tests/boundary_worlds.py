"""Decision-boundary worlds — TEST INFRASTRUCTURE (uses the oracle as the tuning instrument).

The random worlds of armour_amd.worlds keep every obstacle clear of the arm, so every collision
row sits centimetres from the reference's violation threshold (1e-4, KPR/Parameters.h:38,
KPR/NLPclass.cu:472-484) and every plan is feasible. These worlds are built to sit ON the
decisions the reference makes:

  * "graze":  obstacles tuned with the oracle so that each one's largest collision value at the
              start point x0 lies in 1e-4 + U(-2e-3, 2e-3): the solver starts against (or just
              inside) active collision constraints, and near-threshold rows are plentiful
              (KPR/CollisionChecking.cu:230-299 values; NLPclass.cu:472-484 decision).
              From rest (qd0 = qdd0 = 0, as the saved-world replans, load_saved_world.m) the
              arm's k = 0 trajectory is still, so a tuned obstacle puts ~T rows near the threshold.
  * "graze_moving": the same with SURVEY §8(d)'s full start-state ranges
              (qd0 ~ U(-0.5, 0.5) * speed_limit, qdd0 ~ U(-1, 1)).
  * "start":  one obstacle enclosing a link box at the start configuration: every k collides
              at t = 0, so finalize_solution must report infeasible and armour_main write -1
              (KPR/armour_main.cu:326-334).
  * "torque": the reference's own debug state (KPR/debug_script.m:29-31: q0 = -+1, qd0 = +-1,
              qdd0 = 2) or full-range start states, typically over the torque limits already at
              k = 0 (NLPclass.cu:455-463).

Tuning: oracle reach once per world (the reach sets do not depend on obstacles), then per
obstacle a bisection of its distance from a chosen link centre along a random direction, with
OraclePlanner.set_obstacles + eval (one obstacle at a time, so each bisection step is cheap).
`tests/golden/make_boundary.py` freezes the resulting worlds (inputs + the oracle's decisions
and plans) into tests/golden/boundary_*.npz.
"""
from __future__ import annotations

import numpy as np

from armour_amd.robots import KINOVA
from armour_amd.worlds import make_world
from oracle import OraclePlanner

COL_THR = 1e-4  # COLLISION_AVOIDANCE_CONSTRAINT_VIOLATION_THRESHOLD (KPR/Parameters.h:38)
DEBUG_Q0 = np.array([-1.0, -1.0, -1.0, -1.0, 1.0, 1.0, 1.0])      # KPR/debug_script.m:29
DEBUG_QD0 = np.array([1.0, 1.0, 1.0, -1.0, -1.0, -1.0, -1.0])     # :30
DEBUG_QDD0 = np.full(7, 2.0)                                       # :31


def collision_slice(T, NJ, O, nt=None):
    """rows of the collision block g[nt + (l*T + t)*O + o] (NLPclass.cu:290-296); nt = 7T torque rows
    before it (ARMTD, ACMP/NLPclass.cu:273: none)"""
    nt = 7 * T if nt is None else nt
    return slice(nt, nt + NJ * T * O)


def start_state(rng, kind, robot=KINOVA):
    n = 7
    lb = np.where(robot.state_lb < -100, -np.pi, robot.state_lb + 0.2)
    ub = np.where(robot.state_ub > 100, np.pi, robot.state_ub - 0.2)
    q0 = rng.uniform(lb, ub)
    if kind in ("graze", "start"):
        qd0, qdd0 = np.zeros(n), np.zeros(n)
    elif kind == "torque" and rng.uniform() < 0.5:
        q0, qd0, qdd0 = DEBUG_Q0.copy(), DEBUG_QD0.copy(), DEBUG_QDD0.copy()
    else:  # SURVEY §8(d) full ranges
        qd0 = rng.uniform(-0.5, 0.5, n) * robot.speed_limits
        qdd0 = rng.uniform(-1.0, 1.0, n)
    q_des = q0 + rng.uniform(-1.0, 1.0, n) * (np.pi / 48) * 0.8
    return q0, qd0, qdd0, q_des


def _box(c, half):
    return np.concatenate([c, np.diag(half).T.reshape(-1)])


def _obstacle_max(R, obs, x0, T, NJ, nt=None):
    R.set_obstacles(obs[None, :])
    g = R.eval(x0, jac=False)
    return g[collision_slice(T, NJ, 1, nt)].max()


def tune_obstacle(R, rng, lc, x0, T, NJ, target, t_lo=0.3, nt=None):
    """box obstacle whose largest collision value at x0 is `target` (to ~1e-7): centre on a ray from
    a link centre lc[t, l] (t in [t_lo, 1) of the plan), distance found by bisection."""
    for _ in range(20):
        t = int(rng.integers(int(t_lo * T), T))
        l = int(rng.integers(1, NJ))
        half = rng.uniform(0.005, 0.15, 3)
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        base = lc[t, l]
        lo, hi = 0.0, 1.5
        if _obstacle_max(R, _box(base + u * hi, half), x0, T, NJ, nt) >= target:
            continue
        if _obstacle_max(R, _box(base + u * lo, half), x0, T, NJ, nt) <= target:
            continue
        for _ in range(48):
            mid = 0.5 * (lo + hi)
            if _obstacle_max(R, _box(base + u * mid, half), x0, T, NJ, nt) > target:
                lo = mid
            else:
                hi = mid
        return _box(base + u * hi, half)
    raise RuntimeError("could not place a tuned obstacle")


def start_obstacle(robot_geo, q0, rng):
    """a box enclosing link l's box at q0 (point FK of armour_amd.worlds.link_spheres)"""
    from armour_amd.worlds import link_spheres

    cs, rs = link_spheres(robot_geo, q0)
    l = int(rng.integers(2, len(cs)))
    half = np.full(3, rs[l] + 0.02)
    return _box(cs[l], half)


ROBOTS = ("kinova", "fetch")


def robot_of(name="kinova"):
    """(geometry for the world generator, armour_robot struct for the oracle or None, tables or
    None) of a fixture's robot: "kinova" = the built-in KPR/KinovaWithoutGripperInfo.h tables,
    "fetch" = tests/golden/robot_fetch.json (the Fetch arm from its URDF, 8 joints)"""
    if name == "kinova":
        return KINOVA, None, None
    import os

    from armour_amd import robot_tables as RT
    tables = RT.load_json(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "robot_fetch.json"))
    return RT.geometry(tables), RT.to_struct(tables), tables


def boundary_world(seed, kind, T, O, threads=8, robot=KINOVA, n_tuned=None, t_lo=0.5, robot_struct=None):
    """one decision-boundary world (q0, qd0, qdd0, q_des, obstacles[O, 12]) plus the x0 it is tuned at.
    n_tuned obstacles are tuned near the threshold (default: half of them for graze kinds, a quarter otherwise);
    the rest come from the ordinary generator. robot: the generator's geometry; robot_struct: the
    oracle's armour_robot tables (None: Kinova)."""
    rng = np.random.default_rng(10_000 + seed)
    q0, qd0, qdd0, q_des = start_state(rng, kind, robot)
    x0 = np.zeros(7)
    filler = make_world(seed, O, robot=robot)[4]
    R = OraclePlanner(q0, qd0, qdd0, q_des, filler, T=T, threads=threads, robot=robot_struct)
    R.reach()
    NJ = R.NJ
    _, _, lc = R.eval(x0, centers=True)
    if n_tuned is None:
        n_tuned = (O + 1) // 2 if kind.startswith("graze") else O // 4
    # most tuned obstacles just clear at x0 (the solver works against active constraints), about
    # one in six just inside the threshold (the solver must move out, or cannot)
    obs = [tune_obstacle(R, rng, lc, x0, T, NJ, COL_THR + rng.uniform(-3e-3, 6e-4), t_lo=t_lo)
           for _ in range(n_tuned)]
    obs += list(filler[:O - n_tuned])
    if kind == "start" and O > 0:
        obs[-1] = start_obstacle(robot, q0, rng)
    obstacles = np.array(obs, dtype=np.float64).reshape(O, 12)
    return (q0, qd0, qdd0, q_des, obstacles), x0


def near_threshold_rows(g, T, NJ, O, band=1e-3, nt=None):
    col = g[collision_slice(T, NJ, O, nt)]
    return int(np.sum(np.abs(col - COL_THR) < band))
