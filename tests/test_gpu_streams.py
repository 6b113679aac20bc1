"""The reach phase on its own stream: with a CU-masked reach stream (ARMOUR_REACH_CU_RESERVE) and a
high-priority solver stream (ARMOUR_SOLVER_PRIORITY) the solver's stream must still see the reach
phase's outputs (the event wait in planner.hip run_reach; the constraint bounds are formed on the
solver stream by ipm_rows_init). Plans are bitwise those of the default streams, on both engines."""
import numpy as np
import pytest

import armour_amd as A
from conftest import engine
from test_gpu_plane_cache import check_plan, env

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("eng", ["lane", "job"])
def test_cu_masked_reach_stream_plans_bitwise(eng):
    T, O, W = 100, 20, 12
    worlds = [A.make_world(4000 + s, O, profile="survey") for s in range(W)]
    with engine(eng):
        P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
        with env("ARMOUR_REACH_CU_RESERVE", "32"), env("ARMOUR_SOLVER_PRIORITY", "1"):
            Q = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    check_plan(P, Q, worlds)
    # twice more on the masked planner: back-to-back reach phases reuse the same buffers
    ra, _ = P.plan(worlds)
    for _ in range(2):
        rb, _ = Q.plan(worlds)
        for a, b in zip(ra, rb):
            np.testing.assert_array_equal(a["k_opt"], b["k_opt"])
            assert a["iterations"] == b["iterations"]


def test_bundle_kernel_shapes_plan_bitwise():
    """the bundle kernel's two LDS / register shapes (lane_kernel.hip LaneWide, LaneDense; planner.hip
    picks by device sharing and batch size) hold the same arithmetic: plans bitwise equal"""
    T, O, W = 100, 20, 24
    worlds = [A.make_world(4100 + s, O, profile="survey") for s in range(W)]
    with engine("lane"):
        with env("ARMOUR_LANE_SHAPE", "wide"):
            P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
        with env("ARMOUR_LANE_SHAPE", "dense"):
            Q = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    check_plan(P, Q, worlds)
    for w in range(W):
        np.testing.assert_array_equal(P.link_generators(w), Q.link_generators(w))
        np.testing.assert_array_equal(P.torque_radius(w), Q.torque_radius(w))
