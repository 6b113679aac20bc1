"""The oracle's reachable sets enclose the reference's definitions.

The reference ships no outputs, so the oracle cannot be pinned to reference
values. What can be pinned is what the sets MEAN, checked with the independent point models of
tests/point_model.py (no PZ code) at sampled points:

  * Bezier identities of the desired trajectory (KPR/Trajectory.cu:542-599): q(0) = q0,
    qd(0) = qd0, qdd(0) = qdd0, q(1) = q0 + k, qd(1) = qdd(1) = 0 — and the oracle's position /
    velocity extremum rows (Trajectory.cu:256-540, the last 28 rows of g) bracket a dense sampling
    of that trajectory;
  * link-set containment: the point FK of every link-box corner at a random time inside interval
    s, with k = x * k_range and a joint error within +-qe, lies in the sliced link zonotope
    centre(x) + residual generators (KPR/Dynamics.cu:69-81, PZsparse.cu:370-402), checked as
    zonotope membership over its facet normals;
  * torque containment: the point RNEA torque at sampled (t, k, tracking errors within qe / qde /
    qdae / qddae), with nominal and +-3 % mass / inertia (KPR/KinovaWithoutGripperInfo.h:41,61),
    lies in the sliced torque centre +- (torque radius - alpha (M_max - M_min) eps)
    (KPR/armour_main.cu:173-211, the check of KPR/debug_script.m:98-123).

The same checks run on the HIP path's outputs in tests/test_gpu_containment.py.
"""
import os

import numpy as np
import pytest

import armour_amd as A
import point_model as PM
from armour_amd import robot_tables as RT
from oracle import OraclePlanner

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
K_RANGE = np.pi / 48   # KPR/Parameters.h:21
SLACK = 1e-9           # rounding of the sets' own arithmetic (metres / N m)


def kinova():
    """the tables of KPR/KinovaWithoutGripperInfo.h (the oracle's robot 0; pinned to the header by
    tests/test_robot_tables.py). The URDF-derived tables differ in the link boxes by the header's
    6-decimal rounding (5e-7 m), more than the containment slack."""
    return RT.builtin(0)


def fetch():
    return RT.load_json(os.path.join(GOLD, "robot_fetch.json"))


def containment(robot, world, T, x, centers, gens, tq_center, tq_radius, rng, n_t=2, n_par=2):
    """(worst link excess [m], worst torque excess [N m], samples) of the sets of one world at x.
    centers [T, NJ, 3], gens [T, NJ, 3, 6], tq_center [T, 7], tq_radius [T, 7]"""
    q0, qd0, qdd0 = (np.asarray(v, dtype=np.float64) for v in world[:3])
    beta = PM.control_points(q0, qd0, qdd0, np.asarray(x) * K_RANGE)     # [7, 6]
    qe, qde, qdae, qddae = PM.ultimate_bounds(robot)
    NJ = int(robot["num_joints"])
    s = np.repeat(np.arange(T), n_t)
    t = (s + rng.uniform(0, 1, s.size)) / T
    q, qd, qdd = PM.bezier(beta[None, :, :], t[:, None])                # [N, 7]
    N = t.size
    # links: every box corner at q + e, |e| <= qe
    qs = q + rng.uniform(-qe, qe, q.shape)
    pts = PM.link_points(robot, qs)                                      # [NJ, N, 8, 3]
    exc = PM.zonotope_excess(centers[s].transpose(1, 0, 2), gens[s].transpose(1, 0, 2, 3), pts)
    link_worst = float(exc.max())
    # torques: nominal parameters and +-3 % mass / inertia, errors within the ultimate bounds
    tq_worst = -np.inf
    bound = tq_radius[s] - PM.robust_term(robot) - robot["friction"][:7]
    for k in range(n_par):
        e = [rng.uniform(-b, b, q.shape) for b in (qe, qde, qdae, qddae)]
        if k == 0:
            m, I = None, None
        else:
            mu, iu = robot["mass_uncertainty"], robot["inertia_uncertainty"]
            m = robot["mass"] * (1 + rng.uniform(-mu, mu, (N, NJ)))
            I = robot["inertia"] * (1 + rng.uniform(-iu, iu, (N, NJ, 3, 3)))
        u = PM.rnea(robot, q + e[0], qd + e[1], qd + e[2], qdd + e[3], mass=m, inertia=I)
        tq_worst = max(tq_worst, float((np.abs(u - tq_center[s]) - bound).max()))
    return link_worst, tq_worst, N


def oracle_sets(R, x):
    g, lc = R.eval(x, jac=False, centers=True)
    T = R.T
    return lc, R.link_gens(), g[:7 * T].reshape(T, 7), R.torque_radius()


WORLDS = [("survey", s) for s in (0, 1, 2, 5)] + [("debug", 0)]


def _world(kind, seed, O=20, robot_geo=A.KINOVA):
    if kind == "debug":
        import boundary_worlds as B
        return (B.DEBUG_Q0, B.DEBUG_QD0, B.DEBUG_QDD0, B.DEBUG_Q0 + 0.03, A.make_world(seed, O)[4])
    return A.make_world(seed, O, robot=robot_geo, profile="survey")


@pytest.mark.parametrize("kind,seed", WORLDS)
def test_oracle_sets_contain_point_models(kind, seed):
    robot = kinova()
    T = 100
    world = _world(kind, seed)
    R = OraclePlanner(*world, T=T, threads=8)
    R.reach()
    rng = np.random.default_rng(seed + 7)
    n = 0
    for x in (np.zeros(7), rng.uniform(-1, 1, 7), np.sign(rng.uniform(-1, 1, 7))):
        lw, tw, k = containment(robot, world, T, x, *oracle_sets(R, x), rng)
        n += k
        assert lw <= SLACK, f"link point outside its zonotope by {lw:.3e} m at x={x}"
        assert tw <= SLACK, f"torque outside centre +- radius by {tw:.3e} N m at x={x}"
    assert n >= 600


def test_fetch_oracle_sets_contain_point_models():
    """the same on the Fetch arm from its URDF (8 joints, the fixed gripper last)"""
    robot = fetch()
    T = 40
    world = A.make_world(31, 8, robot=RT.geometry(robot), profile="survey")
    R = OraclePlanner(*world, T=T, threads=8, robot=RT.to_struct(robot))
    R.reach()
    rng = np.random.default_rng(3)
    for x in (np.zeros(7), rng.uniform(-1, 1, 7)):
        lw, tw, _ = containment(robot, world, T, x, *oracle_sets(R, x), rng)
        assert lw <= SLACK and tw <= SLACK, (lw, tw)


def test_bezier_identities():
    """KPR/Trajectory.cu:542-599 at the curve's ends (DURATION = 1)"""
    rng = np.random.default_rng(0)
    q0, qd0, qdd0, k = (rng.uniform(-1, 1, 7) for _ in range(4))
    beta = PM.control_points(q0, qd0, qdd0, k)
    q, qd, qdd = PM.bezier(beta, np.zeros(7))
    np.testing.assert_allclose(q, q0, atol=1e-14)
    np.testing.assert_allclose(qd, qd0, atol=1e-14)
    np.testing.assert_allclose(qdd, qdd0, atol=1e-13)
    q, qd, qdd = PM.bezier(beta, np.ones(7))
    np.testing.assert_allclose(q, q0 + k, atol=1e-14)
    np.testing.assert_allclose(qd, 0, atol=1e-13)
    np.testing.assert_allclose(qdd, 0, atol=1e-12)
    # the reference's closed form q_des_func (Trajectory.cu:542-557) is this curve
    t = 0.37
    B = [-(t - 1) ** 5, 5 * t * (t - 1) ** 4, -10 * t ** 2 * (t - 1) ** 3, 10 * t ** 3 * (t - 1) ** 2,
         -5 * t ** 4 * (t - 1), t ** 5]
    ref = sum(b * beta[:, i] for i, b in enumerate(B))
    np.testing.assert_allclose(PM.bezier(beta, np.full(7, t))[0], ref, atol=1e-14)


@pytest.mark.parametrize("seed", [0, 3, 9])
def test_oracle_extremum_rows_bracket_the_trajectory(seed):
    """rows [min q, max q, min qd, max qd] of g (NLPclass.cu:305-318 via Trajectory.cu:256-540) are
    the exact extrema over t in [0, 1]: they bracket a dense sampling of the point model's curve
    and are attained within the sampling's resolution"""
    T, O = 20, 2
    world = A.make_world(seed, O, profile="survey")
    R = OraclePlanner(*world, T=T, threads=4)
    R.reach()
    rng = np.random.default_rng(seed)
    ts = np.linspace(0, 1, 20001)
    for x in (np.zeros(7), rng.uniform(-1, 1, 7)):
        g = R.eval(x, jac=False)
        ext = g[-28:].reshape(4, 7)
        beta = PM.control_points(world[0], world[1], world[2], x * K_RANGE)
        q, qd, _ = PM.bezier(beta[None, :, :], ts[:, None])
        for row, v, fn in ((0, q, np.min), (1, q, np.max), (2, qd, np.min), (3, qd, np.max)):
            sampled = fn(v, axis=0)
            if fn is np.min:
                assert np.all(ext[row] <= sampled + 1e-12), (row, ext[row] - sampled)
            else:
                assert np.all(ext[row] >= sampled - 1e-12), (row, ext[row] - sampled)
            assert np.abs(ext[row] - sampled).max() < 1e-6, (row, np.abs(ext[row] - sampled).max())
