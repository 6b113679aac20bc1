"""ARMTD comparison planner (ACMP/, oracle/src/armtd.cpp): the oracle against the committed
fixtures (tests/golden/armtd_T100_O10.npz, tests/golden/make_armtd.py) and against the reference's
own definitions; the fixtures' JRS tables against the reference's offline JRS files when present."""
import os

import numpy as np
import pytest

import boundary_worlds as B
from oracle import OracleArmtd

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    return dict(np.load(os.path.join(GOLD, "armtd_T100_O10.npz")))


def world(fx, w):
    return fx["q0"][w], fx["qd0"][w], fx["q_des"][w], fx["tables"][w], fx["k_range"][w], fx["obstacles"][w]


@pytest.mark.parametrize("w", range(8))
def test_oracle_reproduces_fixture(w):
    fx = load()
    T, O = int(fx["T"]), fx["obstacles"].shape[1]
    R = OracleArmtd(*world(fx, w), T=T, threads=4)
    R.reach()
    g0 = R.eval(fx["x0"][w], jac=False)
    np.testing.assert_array_equal(np.packbits(g0[:7 * T * O] > B.COL_THR), fx["dec_x0"][w])
    r = R.plan()
    assert r["feasible"] == bool(fx["feasible"][w]) and r["status"] == fx["status"][w]
    assert r["iterations"] == fx["iterations"][w]
    np.testing.assert_allclose(r["k_opt"], fx["k_opt"][w], rtol=0, atol=1e-10)


def test_fixture_covers_decisions():
    fx = load()
    assert (~fx["feasible"]).any() and fx["feasible"].any()
    assert fx["near_x0"].sum() + fx["near_kopt"].sum() >= 100
    assert not fx["feasible"][fx["kinds"] == "start"].any()


def test_layout_and_extrema():
    """m = NJ*T*O + 28 (ACMP/NLPclass.cu:45-46); collision rows first, then the constant-acceleration
    extrema (ACMP/Trajectory.cu:83-227) at x = 0: q(t) = q0 + qd0 t, braking to rest at t = 1"""
    fx = load()
    T, O = int(fx["T"]), fx["obstacles"].shape[1]
    q0, qd0 = fx["q0"][0], fx["qd0"][0]
    R = OracleArmtd(*world(fx, 0), T=T, threads=4)
    R.reach()
    g = R.eval(np.zeros(7), jac=False)
    assert g.shape == (7 * T * O + 28,)
    ext = g[7 * T * O:]
    q_peak, q_stop = q0 + 0.5 * qd0, q0 + 0.5 * qd0 + 0.25 * qd0
    np.testing.assert_allclose(ext[:7], np.minimum(q0, np.minimum(q_peak, q_stop)), atol=1e-15)
    np.testing.assert_allclose(ext[7:14], np.maximum(q0, np.maximum(q_peak, q_stop)), atol=1e-15)
    np.testing.assert_allclose(ext[14:21], np.minimum(qd0, 0), atol=1e-15)
    np.testing.assert_allclose(ext[21:], np.maximum(qd0, 0), atol=1e-15)


def test_tables_are_the_reference_offline_jrs():
    """the fixture's tables are the slices of ACMP/offline_jrs/orig_parameterization/JRS_<c_kvi>.mat
    the MATLAB caller makes (KSI/uarmtd_planner.m:260-318)"""
    import offline_jrs as J

    if not os.path.isdir(J.JRS_DIR):
        pytest.skip("reference not present")
    fx = load()
    for w in (0, 3):
        tab, kr = J.armtd_input(fx["qd0"][w])
        np.testing.assert_array_equal(tab, fx["tables"][w])
        np.testing.assert_array_equal(kr, fx["k_range"][w])
