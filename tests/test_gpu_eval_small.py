"""The small-capacity evaluation kernels (eval_kernel_small, eval_trials_small: LDS sized for the
batch's largest PZs, five blocks per CU) against the full-capacity ones
(ARMOUR_EVAL_FULL=1): constraint values, Jacobians and whole plans bitwise equal, on survey worlds
and on the config 3 decision-boundary fixture (280 pairs, the largest the small kernels take)."""
import numpy as np
import pytest

import armour_amd as A
from conftest import engine
from test_boundary import load, world
from test_gpu_plane_cache import check_eval, check_plan, env

pytestmark = pytest.mark.gpu


def planners(T, O, W, eng=None):
    with engine(eng):
        P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
        with env("ARMOUR_EVAL_FULL", "1"):
            Q = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    return P, Q


def test_eval_small_survey_worlds():
    T, O, W = 100, 20, 40
    worlds = [A.make_world(3000 + s, O, profile="survey") for s in range(W)]
    P, Q = planners(T, O, W, "lane")  # the bundle engine records the PZ sizes
    check_eval(P, Q, worlds, np.random.default_rng(5), n=2)
    check_plan(P, Q, worlds)
    occ = P.occupancy()
    assert occ["link_monomials"][0] <= 16 and occ["torque_monomials"][0] <= 64  # the small kernels ran


def test_eval_small_boundary_config3():
    fx = load("boundary_config3_T200_O40")
    T, W, O = int(fx["T"]), len(fx["kinds"]), fx["obstacles"].shape[1]
    worlds = [world(fx, w) for w in range(W)]
    P, Q = planners(T, O, W)
    check_eval(P, Q, worlds, np.random.default_rng(9), n=3)
    check_plan(P, Q, worlds)
