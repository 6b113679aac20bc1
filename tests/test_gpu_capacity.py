"""Reach-set capacity: headroom at SURVEY §8(d)'s full start-state ranges and at the reference's
debug state (KPR/debug_script.m:29-31), the 4x-buffer retry, and per-world isolation of a world
that still overflows (armour_result.error; the rest of the batch is planned)."""
import os

import numpy as np
import pytest

import armour_amd as A
from conftest import engine

pytestmark = pytest.mark.gpu
DEBUG = (np.array([-1.0, -1, -1, -1, 1, 1, 1]), np.array([1.0, 1, 1, -1, -1, -1, -1]), np.full(7, 2.0))


def debug_world(O):
    base = A.make_world(1, O)
    return DEBUG + (DEBUG[0] + 0.05, base[4])


def rest_world(O):
    q0, _, _, qdes, obs = A.make_world(1, O)
    return q0, np.zeros(7), np.zeros(7), qdes, obs


def test_full_range_headroom():
    """1000 worlds at the full SURVEY §8(d) ranges (T=100, O=20): no capacity failure, and the
    largest use of every buffer stays below 80 % of its capacity"""
    T, O = 100, 20
    B = A.default_batch(T)
    with engine("lane"):  # the last batch (19 worlds) would take the per-job engine
        P = A.Planner(T=T, max_obstacles=O, max_worlds=B)
    worst = {}
    for s0 in range(0, 1000, B):
        worlds = [A.make_world(s, O, profile="survey") for s in range(s0, min(1000, s0 + B))]
        res, _ = P.plan(worlds)
        assert all(r["error"] == 0 for r in res)
        for k, (u, c) in P.occupancy().items():
            worst[k] = (max(u, worst.get(k, (0, c))[0]), c)
    print({k: f"{u}/{c}" for k, (u, c) in worst.items()})
    assert worst["worlds_retried"][0] == 0
    for k in ("arena_hashes", "arena_rows", "operator_terms", "link_monomials", "torque_monomials"):
        assert worst[k][0] < 0.8 * worst[k][1], (k, worst[k])


def test_debug_state_headroom():
    """the reference's debug state (qd0 = +-1, qdd0 = 2) at the drop-in's T = 128"""
    with engine("lane"):  # the bundle engine records occupancy (and has the union inflation)
        P = A.Planner(T=128, max_obstacles=10, max_worlds=1)
    res, _ = P.plan([debug_world(10)])
    occ = P.occupancy()
    print(occ)
    assert res[0]["error"] == 0 and occ["worlds_retried"][0] == 0
    assert occ["arena_rows"][0] < 0.8 * occ["arena_rows"][1]


def _planner(T, O, W, ccap=None):
    if ccap is None:
        os.environ.pop("ARMOUR_LANE_CCAP", None)
    else:
        os.environ["ARMOUR_LANE_CCAP"] = str(ccap)
    try:
        with engine("lane"):
            return A.Planner(T=T, max_obstacles=O, max_worlds=W)
    finally:
        os.environ.pop("ARMOUR_LANE_CCAP", None)


def test_retry_and_per_world_isolation():
    """T = 64: one bundle is one world. With the arena shrunk so that every world overflows the
    first launch, the retry (4x buffers) plans them all bitwise as the full-size arena does; shrunk
    further, only the heavy debug-state world still overflows: it alone reports ARMOUR_E_CAPACITY
    and the other worlds are planned, bitwise as before."""
    T, O = 64, 8
    worlds = [rest_world(O), debug_world(O), rest_world(O)]
    P = _planner(T, O, 3)
    ref, _ = P.plan(worlds)
    use = []
    for w in worlds:
        P.plan([w])
        use.append(P.occupancy()["arena_rows"][0])
    P.close()
    light, heavy = max(use[0], use[2]), use[1]
    assert all(r["error"] == 0 for r in ref)

    P = _planner(T, O, 3, ccap=light // 2)
    res, _ = P.plan(worlds)
    occ = P.occupancy()
    assert occ["worlds_retried"][0] == 3 and occ["worlds_failed"][0] == 0
    for r, r0 in zip(res, ref):
        assert r["error"] == 0 and np.array_equal(r["k_opt"], r0["k_opt"]) and r["iterations"] == r0["iterations"]
    P.close()

    c = (light + heavy) // 8   # 4c >= light, 4c < heavy
    assert 4 * c >= light and 4 * c < heavy
    P = _planner(T, O, 3, ccap=c)
    res, _ = P.plan(worlds)
    occ = P.occupancy()
    assert occ["worlds_retried"][0] == 3 and occ["worlds_failed"][0] == 1
    assert res[1]["error"] == A.ARMOUR_E_CAPACITY and not res[1]["feasible"] and res[1]["status"] == 3
    for w in (0, 2):
        assert res[w]["error"] == 0 and np.array_equal(res[w]["k_opt"], ref[w]["k_opt"])
        assert res[w]["feasible"] == ref[w]["feasible"] and res[w]["iterations"] == ref[w]["iterations"]
