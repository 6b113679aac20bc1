"""The certified plane cache (plane_cache_kernel) against the full per-evaluation
plane scan of the same library (ARMOUR_PLANE_CACHE=0): constraint values, Jacobians and whole plans
bitwise equal, on survey worlds and on the decision-boundary fixtures, at points inside the
certified box (cached scan) and outside it (full scan in both)."""
import contextlib
import os

import numpy as np
import pytest

import armour_amd as A
from conftest import engine
from test_boundary import load, world

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def env(name, value):
    prev = os.environ.get(name)
    os.environ[name] = value
    try:
        yield
    finally:
        if prev is None:
            os.environ.pop(name, None)
        else:
            os.environ[name] = prev


def planners(T, O, W):
    P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    with env("ARMOUR_PLANE_CACHE", "0"):
        Q = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    return P, Q


def points(rng, n):
    xs = [np.zeros(7), np.ones(7), -np.ones(7), np.array([1, -1, 1, -1, 1, -1, 1.0])]
    xs += [rng.uniform(-1, 1, 7) for _ in range(n)]
    xs += [rng.uniform(-1, 1, 7) * 1.5]  # outside the certified box: the full scan in both
    return xs


def check_eval(P, Q, worlds, rng, n=6):
    P.reach(worlds)
    Q.reach(worlds)
    for x in points(rng, n):
        for w in range(len(worlds)):
            g, J = P.eval_constraints(w, x)
            gq, Jq = Q.eval_constraints(w, x)
            np.testing.assert_array_equal(g, gq)
            np.testing.assert_array_equal(J, Jq)


def check_plan(P, Q, worlds):
    ra, _ = P.plan(worlds)
    rb, _ = Q.plan(worlds)
    for w, (a, b) in enumerate(zip(ra, rb)):
        assert a["feasible"] == b["feasible"] and a["status"] == b["status"], w
        assert a["iterations"] == b["iterations"] and a["evaluations"] == b["evaluations"], w
        np.testing.assert_array_equal(a["k_opt"], b["k_opt"])
        np.testing.assert_array_equal(P.constraints(w), Q.constraints(w))


@pytest.mark.parametrize("eng", ["lane", "job"])
def test_plane_cache_survey_worlds(eng):
    T, O, W = 100, 20, 12
    worlds = [A.make_world(1000 + s, O, profile="survey") for s in range(W)]
    with engine(eng):
        P, Q = planners(T, O, W)
    rng = np.random.default_rng(7)
    check_eval(P, Q, worlds, rng)
    check_plan(P, Q, worlds)


@pytest.mark.parametrize("name", ["boundary_config2_T100_O20", "boundary_config3_T200_O40"])
def test_plane_cache_boundary(name):
    fx = load(name)
    T, W, O = int(fx["T"]), len(fx["kinds"]), fx["obstacles"].shape[1]
    worlds = [world(fx, w) for w in range(W)]
    P, Q = planners(T, O, W)
    rng = np.random.default_rng(11)
    check_eval(P, Q, worlds, rng, n=3)
    check_plan(P, Q, worlds)


def test_plane_cache_stats_survey():
    """kept planes per pair on survey worlds (DESIGN.md section 4 quotes these)"""
    T, O, W = 100, 20, 64
    P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    P.reach([A.make_world(2000 + s, O, profile="survey") for s in range(W)])
    st = P.plane_cache_stats()
    print("plane cache:", st, "mean kept per pair %.2f" % (st["planes_kept"] / st["pairs"]))
    assert st["pairs"] == W * T * 7 * O
    assert st["blocks_cached"] == st["blocks"]
    assert 1 <= st["max_per_pair"] <= 36


def test_plane_cache_pool_regrows():
    """The cache's records live in one pool sized at creation for ARMOUR_PC_K records per pair
    (default 12; the survey workload keeps 5.3). A pool too small for a build (ARMOUR_PC_K=1) is
    grown to what the build needed and the build repeated: every block cached, and the plans and
    constraint values bitwise those of the default pool and of the full scan."""
    T, O, W = 100, 20, 8
    worlds = [A.make_world(3000 + s, O, profile="survey") for s in range(W)]
    P, Q = planners(T, O, W)
    with env("ARMOUR_PC_K", "1"):
        S = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    S.reach(worlds)
    st = S.plane_cache_stats()
    assert st["blocks_cached"] == st["blocks"] and st["pool_records"] >= st["planes_kept"] > W * T * 7 * O
    check_plan(S, Q, worlds)
    check_plan(P, S, worlds)


def test_plane_cache_grow_failure_falls_back_to_full_scan():
    """A build that overflows its pool when the larger pool cannot be allocated
    (ARMOUR_PC_GROW_FAIL simulates the failed allocation) must not leave the cache marked ready:
    the blocks that did not fit have no records at their pool offset. The solve then runs on the
    full scan and the sequential line-search rounds: every plan, constraint value and iteration
    count bitwise those of the full-scan planner, and a later build that fits caches again."""
    T, O, W = 100, 20, 8
    worlds = [A.make_world(3100 + s, O, profile="survey") for s in range(W)]
    P, Q = planners(T, O, W)
    with env("ARMOUR_PC_K", "1"):
        S = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    with env("ARMOUR_PC_GROW_FAIL", "1"):
        check_plan(S, Q, worlds)
        S.reach(worlds)
        st = S.plane_cache_stats()
        assert st["blocks_cached"] < st["blocks"]
        rng = np.random.default_rng(5)
        for x in points(rng, 2):
            for w in range(W):
                g, J = S.eval_constraints(w, x)
                gq, Jq = Q.eval_constraints(w, x)
                np.testing.assert_array_equal(g, gq)
                np.testing.assert_array_equal(J, Jq)
    check_plan(S, P, worlds)
