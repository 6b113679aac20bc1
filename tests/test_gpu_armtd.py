"""ARMTD comparison planner on the GPU (armour_create_armtd, armtd_main) against the oracle
(oracle/src/armtd.cpp) on the fixture worlds (tests/golden/armtd_T100_O10.npz: the reference's
offline JRS tables, obstacles on the collision threshold, a start-in-collision world).
Bar as the ARMOUR path: link generators, g and J within 1e-9, every collision decision and the
feasibility re-check identical, solver status / iterations identical, k_opt within 1e-8 (1e-3 for
an infeasible plan ending in line-search failure, tests/test_gpu_boundary.py)."""
import os
import subprocess

import numpy as np
import pytest

import armour_amd as A
import boundary_worlds as B
from conftest import engine
from oracle import OracleArmtd
from test_armtd import load, world

pytestmark = pytest.mark.gpu
TOL = 1e-9
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "armour-dev_amd", "armour_amd", "armtd_main")


@pytest.mark.parametrize("eng", ["lane", "job"])
def test_armtd_parity(eng):
    fx = load()
    T, W, O = int(fx["T"]), len(fx["kinds"]), fx["obstacles"].shape[1]
    worlds = [world(fx, w) for w in range(W)]
    with engine(eng):
        P = A.ArmtdPlanner(T=T, max_obstacles=O, max_worlds=W)
    assert P.num_constraints(O) == 7 * T * O + 28
    P.reach(worlds)
    refs = []
    cs = B.collision_slice(T, 7, O, nt=0)
    for w in range(W):
        R = OracleArmtd(*worlds[w], T=T, threads=8)
        R.reach()
        refs.append(R)
        np.testing.assert_allclose(P.link_generators(w), R.link_gens(), rtol=0, atol=TOL)
        for x in (fx["x0"][w], fx["k_opt"][w], np.linspace(-0.8, 0.8, 7)):
            g, J = P.eval_constraints(w, x)
            go, Jo = R.eval(x)
            np.testing.assert_allclose(g, go, rtol=0, atol=TOL)
            np.testing.assert_allclose(J, Jo, rtol=0, atol=TOL)
            np.testing.assert_array_equal(g[cs] > B.COL_THR, go[cs] > B.COL_THR)
            assert R.feasible(g) == R.feasible(go)
    res, _ = P.plan(worlds)
    for w, (r, R) in enumerate(zip(res, refs)):
        ro = R.plan()
        assert r["feasible"] == ro["feasible"] and r["status"] == ro["status"], w
        assert r["iterations"] == ro["iterations"], (w, r["iterations"], ro["iterations"])
        tol = 1e-8 if (r["status"] == 0 or r["feasible"]) else 1e-3
        np.testing.assert_allclose(r["k_opt"], ro["k_opt"], rtol=0, atol=tol, err_msg=f"world {w}")
        np.testing.assert_allclose(P.constraints(w), R.eval(r["k_opt"], jac=False), rtol=0, atol=1e-7)


def write_armtd_in(path, q0, qd0, q_des, tables, k_range, obstacles):
    """the writer of KSI/uarmtd_planner.m:268-324 (%.10f)"""
    with open(os.path.join(path, "armtd.in"), "w") as f:
        for v in (q0, qd0, q_des):
            f.write(" ".join(f"{x:.10f}" for x in v) + "\n")
        for i in range(7):
            for k in range(6):
                f.write(" ".join(f"{x:.10f}" for x in tables[i][k]) + "\n")
            f.write(f"{k_range[i]:.10f}\n ")
        f.write(f"{len(obstacles)}\n")
        for o in obstacles:
            f.write(" ".join(f"{x:.10f}" for x in o) + "\n")


@pytest.mark.parametrize("w", [0, 3])
def test_armtd_main_protocol(tmp_path, w):
    """armtd_main speaks ACMP/armtd_main.cu's file protocol: k_opt or -1 (the start-in-collision
    world 3), centres, generators, constraints"""
    fx = load()
    T, O = int(fx["T"]), fx["obstacles"].shape[1]
    wd = world(fx, w)
    write_armtd_in(str(tmp_path), *wd)
    r = subprocess.run([EXE, str(tmp_path)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ARMOUR_NUM_TIME_STEPS=str(T)))
    assert r.returncode == 0, r.stderr
    out = [float(v) for v in open(tmp_path / "armtd.out").read().split()]
    rounded = tuple(np.round(np.asarray(a, dtype=np.float64), 10) for a in wd)
    P = A.ArmtdPlanner(T=T, max_obstacles=O, max_worlds=1)
    res, _ = P.plan([rounded])
    if res[0]["feasible"]:
        assert len(out) == 8
        np.testing.assert_allclose(out[:7], res[0]["k_opt"], rtol=1e-9, atol=1e-9)
    else:
        assert out[0] == -1 and len(out) == 2
    assert bool(fx["feasible"][w]) == res[0]["feasible"]
    c = np.loadtxt(tmp_path / "armtd_joint_position_center.out")
    assert c.shape == (T * 7, 3)
    np.testing.assert_allclose(c.reshape(T, 7, 3), P.link_centers(0), rtol=1e-9, atol=1e-9)
    gens = np.loadtxt(tmp_path / "armtd_joint_position_radius.out")
    np.testing.assert_allclose(gens.reshape(T, 7, 3, 6), P.link_generators(0), rtol=1e-9, atol=1e-12)
    cons = np.loadtxt(tmp_path / "armtd_constraints.out")
    assert cons.shape == (7 * T * O + 28,)
    np.testing.assert_allclose(cons, P.constraints(0), rtol=1e-5, atol=1e-5)
