"""The oracle (CPU restatement) against the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py), and the fixture inputs against the reference's own input data."""
import numpy as np
import pytest

from conftest import golden_names, load_golden, world_of
from oracle import OraclePlanner

NAMES = golden_names()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_fixture(name):
    fx = load_golden(name)
    T = int(fx["T"])
    P = OraclePlanner(*world_of(fx), T=T, threads=4)
    P.reach()
    np.testing.assert_allclose(P.torque_radius(), fx["torque_radius"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(P.link_gens(), fx["link_gens"], rtol=0, atol=1e-14)
    if "x" in fx:
        for x, g0, J0, f0 in zip(fx["x"], fx["g"], fx["J"], fx["feasible_at_x"]):
            g, J = P.eval(x)
            np.testing.assert_allclose(g, g0, rtol=0, atol=1e-12)
            np.testing.assert_allclose(J, J0, rtol=0, atol=1e-12)
            assert P.feasible(g) == bool(f0)
    r = P.plan()
    assert r["feasible"] == bool(fx["feasible"])
    assert r["iterations"] == int(fx["iterations"]) and r["status"] == int(fx["status"])
    np.testing.assert_allclose(r["k_opt"], fx["k_opt"], rtol=0, atol=1e-10)


def test_example_world_is_reference_example():
    """armour_main.cu:19-34: the commented example input (10 obstacles, rows repeated)."""
    from armour_amd.worlds import example_world

    q0, qd0, qdd0, qdes, obs = example_world()
    np.testing.assert_array_equal(q0, [0.6543, -0.0876, -0.4837, -1.2278, -1.5735, -1.0720, 0])
    np.testing.assert_array_equal(qdes, [0.6831, 0.009488, -0.2471, -0.9777, -1.414, -0.9958, 0])
    assert obs.shape == (10, 12) and np.array_equal(obs[:5], obs[5:])
    np.testing.assert_array_equal(obs[0], [-0.28239, -0.33281, 0.88069, 0.069825, 0, 0, 0, 0.09508, 0, 0, 0, 0.016624])


def test_csv_world_conversion():
    """load_saved_world.m + box_obstacle_zonotope.m + robot_arm_straight_line_HLP.m on a synthetic CSV."""
    from armour_amd.worlds import csv_world

    rows = np.full((5, 7), np.nan)
    rows[0] = [0.1, 0.2, 3.0, 0.4, -3.0, 0.6, 0.7]
    rows[1] = [0.1, 0.2, -3.0, 0.4, 3.0, 0.6, 1.7]
    rows[3, :6] = [1, 2, 3, 0.2, 0.4, 0.6]
    rows[4, :6] = [-1, -2, 0.5, 0.1, 0.1, 0.1]
    q0, qd0, qdd0, qdes, obs = csv_world(rows)
    assert np.all(qd0 == 0) and np.all(qdd0 == 0)
    d = qdes - q0
    np.testing.assert_allclose(np.linalg.norm(d), 0.1)
    # continuous joints 2 and 4 wrap: 3.0 -> -3.0 is +0.283 rad the short way
    assert d[2] > 0 and d[4] < 0 and d[6] > 0 and d[0] == 0
    np.testing.assert_array_equal(obs[0], [1, 2, 3, 0.1, 0, 0, 0, 0.2, 0, 0, 0, 0.3])
    assert obs.shape == (2, 12)


@pytest.mark.parametrize("name", [n for n in NAMES if n.startswith("csv_")])
def test_csv_fixtures_are_reference_worlds(name):
    """CSV fixtures carry start/goal-derived inputs of real reference worlds: q0 within joint
    limits, rest start, step of 0.1 toward the goal, boxes with axis-aligned generators."""
    fx = load_golden(name)
    assert np.all(fx["qd0"] == 0) and np.all(fx["qdd0"] == 0)
    np.testing.assert_allclose(np.linalg.norm(fx["q_des"] - fx["q0"]), 0.1, rtol=1e-12)
    obs = fx["obstacles"].reshape(-1, 4, 3)
    for o in obs:
        G = o[1:]
        assert np.count_nonzero(G) == 3 and np.all(np.diag(G) > 0)
