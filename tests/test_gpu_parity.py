"""HIP path (libarmour_hip.so through the C ABI) against the golden fixtures and a fresh oracle.

Tolerances (fp64 throughout; north_star: "constraints within 1e-9, collision decisions
bit-exact"): reach-set outputs and constraints/Jacobian 1e-9 absolute (observed ~1e-14); the
solver's k_opt 1e-8 with identical iteration counts and feasibility; every collision decision
(g > 1e-4, NLPclass.cu:472-484) and the feasibility re-check exactly equal.
"""
import numpy as np
import pytest

import os

import armour_amd as A
from armour_amd import robot_tables as RT
from conftest import engine, golden_names, load_golden, world_of
from oracle import OraclePlanner

pytestmark = pytest.mark.gpu
TOL = 1e-9
COL_THR = 1e-4  # COLLISION_AVOIDANCE_CONSTRAINT_VIOLATION_THRESHOLD (Parameters.h:38)
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def collision_rows(T, O, NJ):
    """g[7T + (l*T + t)*O + o] for every link l < NJ (NLPclass.cu:290-296; Fetch has NJ = 8)"""
    return slice(7 * T, 7 * T + NJ * T * O)


ENGINES = ["lane", "job", "narrow"]  # both reach engines, the per-job one at both widths (conftest.engine)


@pytest.mark.parametrize("eng", ENGINES)
@pytest.mark.parametrize("name", golden_names())
def test_fixture(name, eng):
    fx = load_golden(name)
    T, O = int(fx["T"]), fx["obstacles"].shape[0]
    with engine(eng):
        P = A.Planner(T=T, max_obstacles=max(O, 1), max_worlds=1)
    world = world_of(fx)
    P.reach([world])
    np.testing.assert_allclose(P.torque_radius(0), fx["torque_radius"], rtol=0, atol=TOL)
    np.testing.assert_allclose(P.link_generators(0), fx["link_gens"], rtol=0, atol=TOL)
    chk = OraclePlanner(*world, T=T, threads=2)  # feasibility decision of the GPU's g
    chk.reach()
    if "x" in fx:
        for x, g0, J0, f0 in zip(fx["x"], fx["g"], fx["J"], fx["feasible_at_x"]):
            g, J = P.eval_constraints(0, x)
            np.testing.assert_allclose(g, g0, rtol=0, atol=TOL)
            np.testing.assert_allclose(J, J0, rtol=0, atol=TOL)
            cr = collision_rows(T, O, P.NJ)
            np.testing.assert_array_equal(g[cr] > COL_THR, g0[cr] > COL_THR)
            assert chk.feasible(g) == bool(f0)
    res, tm = P.plan([world])
    r = res[0]
    assert r["feasible"] == bool(fx["feasible"])
    assert r["iterations"] == int(fx["iterations"]) and r["status"] == int(fx["status"])
    np.testing.assert_allclose(r["k_opt"], fx["k_opt"], rtol=0, atol=1e-8)
    np.testing.assert_allclose(r["cost"], fx["cost"], rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(P.constraints(0), fx["g_opt"], rtol=0, atol=1e-7)
    assert tm["reach_kernel_ms"] > 0 and tm["reach_bytes"] > 0


def _compare_batch(T, O, seeds, xs, robot=None, eng=None):
    geo = RT.geometry(robot) if robot is not None else A.KINOVA
    worlds = [A.make_world(s, O, robot=geo) for s in seeds]
    with engine(eng):
        P = A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds), robot=robot)
    P.reach(worlds)
    refs = []
    for w, world in enumerate(worlds):
        R = OraclePlanner(*world, T=T, threads=8, robot=RT.to_struct(robot) if robot is not None else None)
        R.reach()
        refs.append(R)
        np.testing.assert_allclose(P.torque_radius(w), R.torque_radius(), rtol=0, atol=TOL)
        np.testing.assert_allclose(P.link_generators(w), R.link_gens(), rtol=0, atol=TOL)
        for x in xs:
            g, J = P.eval_constraints(w, x)
            go, Jo = R.eval(x)
            np.testing.assert_allclose(g, go, rtol=0, atol=TOL)
            np.testing.assert_allclose(J, Jo, rtol=0, atol=TOL)
            cr = collision_rows(T, O, P.NJ)
            np.testing.assert_array_equal(g[cr] > COL_THR, go[cr] > COL_THR)
            assert R.feasible(g) == R.feasible(go)
    res, _ = P.plan(worlds)
    for r, R in zip(res, refs):
        ro = R.plan()
        assert r["feasible"] == ro["feasible"] and r["iterations"] == ro["iterations"]
        np.testing.assert_allclose(r["k_opt"], ro["k_opt"], rtol=0, atol=1e-8)


@pytest.mark.parametrize("eng", ENGINES)
def test_config2_batch(eng):
    """BASELINE configs[1]: Kinova, T=100, O=20"""
    _compare_batch(100, 20, [11, 12, 13, 14], [np.zeros(7), np.array([0.5, 0.6, 0.7, 0.0, -0.5, -0.6, -0.7])],
                   eng=eng)


def test_config2_bench_batch_sweep():
    """BASELINE configs[1] at batch scale: 64 worlds (100 bundles of the reach engine, so bundle
    boundaries fall inside worlds), every plan against the oracle"""
    rng = np.random.default_rng(5)
    _compare_batch(100, 20, list(range(500, 564)), [rng.uniform(-1, 1, 7)])


def test_config5_fetch_batch():
    """BASELINE configs[4]: the Fetch arm from its URDF (tests/golden/robot_fetch.json: 7 actuated
    joints + the fixed gripper), here at fp64 and reduced sizes (T=40, O=8); the full-size run is
    `bench.py --robot fetch`. Fetch's reach program does not fit the per-job engine's LDS pool, so
    every batch size runs on the bundle engine (planner.hip job_fits)"""
    fetch = RT.load_json(os.path.join(GOLD, "robot_fetch.json"))
    _compare_batch(40, 8, [31, 32, 33], [np.zeros(7), np.linspace(-0.6, 0.6, 7)], robot=fetch)


def test_config5_fetch_full_size():
    """BASELINE configs[4] at its full size (T=100, O=20), fp64"""
    fetch = RT.load_json(os.path.join(GOLD, "robot_fetch.json"))
    _compare_batch(100, 20, list(range(600, 616)), [np.full(7, 0.3)], robot=fetch)


@pytest.mark.parametrize("eng", ENGINES)
def test_config3_batch(eng):
    """BASELINE configs[2]: T=200, O=40 (MAX_OBSTACLE_NUM)"""
    _compare_batch(200, 40, [21, 22], [np.full(7, -0.4)], eng=eng)


def test_rerun_bitwise_and_batch_position_stable():
    """Rerunning a batch is bitwise reproducible. A world's place in the batch changes only the
    summation order of its pruned amounts: the bundle engine (lane_engine.h) sums them per wave
    over the bundle's union groups, and which union groups exist depends on the bundle's other
    jobs. So across positions the values agree to rounding and every decision is identical."""
    T, O = 20, 6
    worlds = [A.make_world(s, O) for s in range(5)]
    P = A.Planner(T=T, max_obstacles=O, max_worlds=5)
    res_a, _ = P.plan(worlds)
    g_a = [P.constraints(w) for w in range(5)]
    res_b, _ = P.plan(worlds[::-1])
    g_b = [P.constraints(4 - w) for w in range(5)]
    res_c, _ = P.plan(worlds)
    for w in range(5):
        assert np.array_equal(res_a[w]["k_opt"], res_c[w]["k_opt"])
        assert np.array_equal(g_a[w], P.constraints(w))
        assert np.abs(res_a[w]["k_opt"] - res_b[4 - w]["k_opt"]).max() < 1e-8
        assert res_a[w]["feasible"] == res_b[4 - w]["feasible"]
        assert res_a[w]["iterations"] == res_b[4 - w]["iterations"]
        assert np.abs(g_a[w] - g_b[w]).max() < TOL
        rows = collision_rows(T, O, P.NJ)
        assert np.array_equal(g_a[w][rows] > COL_THR, g_b[w][rows] > COL_THR)
