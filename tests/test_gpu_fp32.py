"""The fp32 tolerance-study path (ARMOUR_EVAL_F32: eval_kernel_t<float>, a diagnostic, never the
product path): it must run, stay close to the fp64 evaluation on the same reach sets, and leave the
fp64 path untouched when unset. Bounds from profiles/r01_fp32_study.json, loosened 10x."""
import os

import numpy as np
import pytest

import armour_amd as A

pytestmark = pytest.mark.gpu
T, O, W = 40, 8, 4


def _eval(f32):
    old = os.environ.pop("ARMOUR_EVAL_F32", None)
    try:
        if f32:
            os.environ["ARMOUR_EVAL_F32"] = "1"
        P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    finally:
        os.environ.pop("ARMOUR_EVAL_F32", None)
        if old is not None:
            os.environ["ARMOUR_EVAL_F32"] = old
    P.reach([A.make_world(300 + s, O) for s in range(W)])
    x = np.linspace(-0.6, 0.6, 7)
    return [P.eval_constraints(w, x) for w in range(W)]


def test_fp32_eval_close_to_fp64():
    a, b = _eval(False), _eval(True)
    nt = 7 * T
    for (g64, J64), (g32, J32) in zip(a, b):
        assert np.all(np.isfinite(g32)) and np.all(np.isfinite(J32))
        assert np.max(np.abs(g32[:nt] - g64[:nt])) < 3e-4                   # torque rows
        dc = np.abs(g32[nt:nt + T * 7 * O] - g64[nt:nt + T * 7 * O])         # collision rows
        assert np.median(dc) < 1e-6
        assert not np.array_equal(g32, g64)                                 # it really ran in float
    c = _eval(False)
    for (g0, J0), (g1, J1) in zip(a, c):
        assert np.array_equal(g0, g1) and np.array_equal(J0, J1)            # fp64 unaffected
