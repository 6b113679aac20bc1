"""The HIP path's reachable sets enclose the reference's definitions (the checks of
tests/test_oracle_containment.py on the GPU's outputs).

After a plan, the library returns at the final iterate x = k_opt: the sliced link centres
(armour_get_link_centers), the residual link generators (armour_get_link_generators), the torque
rows of g = the sliced torque centres (armour_get_constraints) and the torque radius
(armour_get_torque_radius). The independent point models of tests/point_model.py (Bezier
trajectory, point FK of the link boxes, point RNEA with nominal and +-3 % parameters) are sampled
at random times in every interval and tracking errors within the ultimate bounds; every sample
must lie in its set (link: zonotope membership; torque: centre +- (radius - the robust term)).
"""
import os

import numpy as np
import pytest

import armour_amd as A
from armour_amd import robot_tables as RT
from test_oracle_containment import SLACK, containment, fetch, kinova

pytestmark = pytest.mark.gpu


def _check(P, worlds, robot, rng, nmax=None):
    res, _ = P.plan(worlds)
    T = P.T
    n = 0
    worst = [-np.inf, -np.inf]
    for w in range(len(worlds) if nmax is None else nmax):
        x = res[w]["k_opt"]
        g = P.constraints(w)
        lw, tw, k = containment(robot, worlds[w], T, x, P.link_centers(w), P.link_generators(w),
                                g[:7 * T].reshape(T, 7), P.torque_radius(w), rng)
        worst = [max(worst[0], lw), max(worst[1], tw)]
        n += k
    assert worst[0] <= SLACK, f"a link point lies {worst[0]:.3e} m outside its set"
    assert worst[1] <= SLACK, f"a torque lies {worst[1]:.3e} N m outside centre +- radius"
    return n, worst


def test_bench_worlds_sets_contain_point_models():
    """32 worlds of the headline workload (survey profile, T = 100, O = 20) at their k_opt"""
    worlds = [A.make_world(s, 20, profile="survey") for s in range(32)]
    P = A.Planner(T=100, max_obstacles=20, max_worlds=len(worlds))
    n, worst = _check(P, worlds, kinova(), np.random.default_rng(1))
    print(f"{n} time samples x (7 links x 8 corners, 2 torque parameter sets): worst excess {worst}")


def test_drop_in_horizon_sets_contain_point_models():
    """one world at the drop-in's T = 128 (KPR/Parameters.h:17), the per-job engine's batch"""
    worlds = [A.make_world(40, 20, profile="survey")]
    P = A.Planner(T=128, max_obstacles=20, max_worlds=1)
    _check(P, worlds, kinova(), np.random.default_rng(2))


def test_fetch_sets_contain_point_models():
    robot = fetch()
    worlds = [A.make_world(600 + s, 20, robot=RT.geometry(robot), profile="survey") for s in range(8)]
    P = A.Planner(T=100, max_obstacles=20, max_worlds=len(worlds), robot=robot)
    _check(P, worlds, robot, np.random.default_rng(3))
