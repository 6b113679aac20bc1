"""The fp32 tolerance-study path (ARMOUR_EVAL_F32: eval_kernel_t<float>, a diagnostic, never the
product path): it must run, stay close to the fp64 evaluation on the same reach sets, and leave the
fp64 path untouched when unset. Bounds from profiles/r01_fp32_study.json, loosened 10x. Two cases:
Kinova at a small size, and BASELINE configs[4] as it is stated — the Fetch arm (its URDF tables,
tests/golden/robot_fetch.json), T = 100, O = 20, fp32."""
import os

import numpy as np
import pytest

import armour_amd as A
from armour_amd import robot_tables as RT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _eval(f32, T, O, W, seed0, robot=None, profile="default"):
    old = os.environ.pop("ARMOUR_EVAL_F32", None)
    try:
        if f32:
            os.environ["ARMOUR_EVAL_F32"] = "1"
        P = A.Planner(T=T, max_obstacles=O, max_worlds=W, robot=robot)
    finally:
        os.environ.pop("ARMOUR_EVAL_F32", None)
        if old is not None:
            os.environ["ARMOUR_EVAL_F32"] = old
    P.reach([A.make_world(seed0 + s, O, profile=profile) for s in range(W)])
    x = np.linspace(-0.6, 0.6, 7)
    return P, [P.eval_constraints(w, x) for w in range(W)]


def _check(T, O, W, seed0, robot=None, torque_tol=3e-4, coll_median=1e-6, coll_max=None, profile="default"):
    Pa, a = _eval(False, T, O, W, seed0, robot, profile)
    Pb, b = _eval(True, T, O, W, seed0, robot, profile)
    nt, nc = 7 * T, T * Pa.NJ * O
    for (g64, J64), (g32, J32) in zip(a, b):
        assert np.all(np.isfinite(g32)) and np.all(np.isfinite(J32))
        assert np.max(np.abs(g32[:nt] - g64[:nt])) < torque_tol              # torque rows
        dc = np.abs(g32[nt:nt + nc] - g64[nt:nt + nc])                        # collision rows
        assert np.median(dc) < coll_median
        if coll_max is not None:
            assert dc.max() < coll_max
        assert not np.array_equal(g32, g64)                                 # it really ran in float
    _, c = _eval(False, T, O, W, seed0, robot, profile)
    for (g0, J0), (g1, J1) in zip(a, c):
        assert np.array_equal(g0, g1) and np.array_equal(J0, J1)            # fp64 unaffected


def test_fp32_eval_close_to_fp64():
    _check(40, 8, 4, 300)


def test_fp32_config5_fetch_full_size():
    """BASELINE configs[4] as stated: the Fetch arm at T = 100, O = 20 in fp32, 8 survey worlds.
    r01's study over 64 Fetch worlds found torque rows within 2.9e-5, collision rows within 4.7e-7
    (no decision flips): held here at 10x (torque 3e-4, collision max 5e-6)."""
    fetch = RT.load_json(os.path.join(GOLD, "robot_fetch.json"))
    _check(100, 20, 8, 600, robot=fetch, coll_max=5e-6, profile="survey")
