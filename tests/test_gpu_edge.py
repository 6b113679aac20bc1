"""Edge cases of the boundary on the GPU: no obstacles, MAX_OBSTACLE_NUM obstacles, single-world
and full batches, argument and state errors, outputs at the solution."""
import numpy as np
import pytest

import armour_amd as A
from oracle import OraclePlanner

pytestmark = pytest.mark.gpu


def test_no_obstacles():
    T = 20
    world = A.make_world(4, 0)
    P = A.Planner(T=T, max_obstacles=0, max_worlds=1)
    res, _ = P.plan([world])
    R = OraclePlanner(*world, T=T, threads=4)
    R.reach()
    ro = R.plan()
    assert P.num_constraints(0) == 7 * T + 28
    assert res[0]["feasible"] == ro["feasible"]
    np.testing.assert_allclose(res[0]["k_opt"], ro["k_opt"], rtol=0, atol=1e-8)


def test_max_obstacles_and_full_batch():
    T, O, W = 10, 40, 3
    worlds = [A.make_world(30 + s, O) for s in range(W)]
    P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    res, _ = P.plan(worlds)
    for w, world in enumerate(worlds):
        R = OraclePlanner(*world, T=T, threads=4)
        R.reach()
        ro = R.plan()
        assert res[w]["feasible"] == ro["feasible"]
        np.testing.assert_allclose(res[w]["k_opt"], ro["k_opt"], rtol=0, atol=1e-8)


def test_outputs_at_solution():
    """armour_joint_position_center.out / armour_constraints.out payloads are those at k_opt"""
    T, O = 20, 5
    world = A.make_world(8, O)
    P = A.Planner(T=T, max_obstacles=O, max_worlds=1)
    res, _ = P.plan([world])
    k = res[0]["k_opt"]
    R = OraclePlanner(*world, T=T, threads=4)
    R.reach()
    g, _, lc = R.eval(k, centers=True)
    np.testing.assert_allclose(P.link_centers(0), lc, rtol=0, atol=1e-9)
    np.testing.assert_allclose(P.constraints(0), g, rtol=0, atol=1e-9)


def test_argument_and_state_errors():
    P = A.Planner(T=10, max_obstacles=3, max_worlds=2)
    with pytest.raises(A.ArmourError, match="state|no reach|plan"):
        P.constraints(0)
    worlds = [A.make_world(s, 3) for s in range(3)]
    with pytest.raises(A.ArmourError, match="num_worlds"):
        P.plan(worlds)                      # more worlds than max_worlds
    with pytest.raises(A.ArmourError, match="max_obstacles"):
        P.plan([A.make_world(0, 4)])        # more obstacles than max_obstacles
    with pytest.raises(A.ArmourError, match="same num_obstacles"):
        P.plan([A.make_world(0, 3), A.make_world(1, 2)])
    P.plan(worlds[:2])
    with pytest.raises(A.ArmourError, match="out of range"):
        P.torque_radius(2)


def test_concurrent_planners_match_sequential():
    # bench.py's default: planners driven from their own host threads (one HIP stream each) must
    # give, world by world, bitwise the results of sequential planning
    import threading
    W, T, O = 6, 40, 8
    batches = [[A.make_world(700 + 10 * b + s, O) for s in range(W)] for b in range(2)]
    seq = [A.Planner(T=T, max_obstacles=O, max_worlds=W).plan(bw)[0] for bw in batches]
    planners = [A.Planner(T=T, max_obstacles=O, max_worlds=W) for _ in range(2)]
    out = [None, None]

    def work(b):
        out[b] = planners[b].plan(batches[b])[0]

    ths = [threading.Thread(target=work, args=(b,)) for b in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for b in range(2):
        assert out[b] is not None
        for r0, r1 in zip(seq[b], out[b]):
            assert np.array_equal(r0["k_opt"], r1["k_opt"]) and r0["iterations"] == r1["iterations"]
            assert r0["feasible"] == r1["feasible"] and r0["status"] == r1["status"]


def test_speculative_line_search_matches_sequential():
    """The tail's speculative line-search round (all remaining trials of the few searching worlds
    at once, planner.hip run_solver) gives bitwise the plans of sequential rounds
    (ARMOUR_NO_SPEC), on full-range worlds whose line searches run long."""
    import os

    T, O = 40, 10
    worlds = [A.make_world(s, O, profile="survey") for s in range(48)]
    P = A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds))
    res_s, _ = P.plan(worlds)
    g_s = [P.constraints(w) for w in range(len(worlds))]
    c_s = [P.link_centers(w) for w in range(len(worlds))]
    os.environ["ARMOUR_NO_SPEC"] = "1"
    try:
        Q = A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds))
    finally:
        del os.environ["ARMOUR_NO_SPEC"]
    res_q, _ = Q.plan(worlds)
    assert sum(r["evaluations"] - r["iterations"] > 1 for r in res_q) > 0, "no world backtracked"
    for w, (a, b) in enumerate(zip(res_s, res_q)):
        assert np.array_equal(a["k_opt"], b["k_opt"]) and a["cost"] == b["cost"]
        assert (a["iterations"], a["evaluations"], a["status"], a["feasible"]) == \
            (b["iterations"], b["evaluations"], b["status"], b["feasible"])
        assert np.array_equal(g_s[w], Q.constraints(w)) and np.array_equal(c_s[w], Q.link_centers(w))


@pytest.mark.parametrize("variant", ["ARMOUR_RESTO_ROUNDS", "ARMOUR_RESTO_INLINE"])
@pytest.mark.parametrize("case", ["survey", "boundary"])
def test_restoration_one_round_matches_rounds(variant, case):
    """The restoration phase's one-round Armijo search (all max_ls trials' values at once, iterations
    launched without a host synchronisation; planner.hip run_resto) and its iterations run inside the
    interior-point loop (ipm_loop, the default) give bitwise the plans of the phase's sequential
    rounds after the loop (ARMOUR_RESTO_ROUNDS) and of the one-round phases after the loop
    (ARMOUR_RESTO_INLINE=0): on full-range worlds a third of which end in local infeasibility
    (status 4), and on the small boundary set, two of whose converging worlds restart the interior
    point at a phase's first iteration (their line search failed at a point within every bound)"""
    import os

    if case == "survey":
        T, O = 40, 10
        worlds = [A.make_world(s, O, profile="survey") for s in range(64)]
    else:
        fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "boundary_small_T20_O6.npz")))
        T, O = int(fx["T"]), fx["obstacles"].shape[1]
        worlds = [(fx["q0"][w], fx["qd0"][w], fx["qdd0"][w], fx["q_des"][w], fx["obstacles"][w])
                  for w in range(len(fx["kinds"]))]
    P = A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds))
    res_s, _ = P.plan(worlds)
    g_s = [P.constraints(w) for w in range(len(worlds))]
    os.environ[variant] = "1" if variant == "ARMOUR_RESTO_ROUNDS" else "0"
    try:
        Q = A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds))
    finally:
        del os.environ[variant]
    res_q, _ = Q.plan(worlds)
    assert sum(r["status"] == 4 for r in res_q) >= (8 if case == "survey" else 3), "too few worlds in the restoration phase"
    for w, (a, b) in enumerate(zip(res_s, res_q)):
        assert np.array_equal(a["k_opt"], b["k_opt"]) and a["cost"] == b["cost"]
        assert (a["iterations"], a["evaluations"], a["status"], a["feasible"]) == \
            (b["iterations"], b["evaluations"], b["status"], b["feasible"]), w
        assert np.array_equal(g_s[w], Q.constraints(w))


@pytest.mark.parametrize("tail", ["16", "1000"])
def test_concurrent_restoration_matches_serial(tail):
    """Restoration phase iterations inside the sync-free tail run on the planner's second stream,
    concurrently with the next interior-point iteration (planner.hip ipm_loop, resto_conc, the
    default): bitwise the plans of phase iterations in order on the planner's stream
    (ARMOUR_RESTO_CONCURRENT=0). "1000" puts every iteration after the first in the tail, so most
    phase iterations overlap an interior-point iteration."""
    import os

    T, O = 40, 10
    worlds = [A.make_world(s, O, profile="survey") for s in range(64)]
    planners = []
    for conc in ("1", "0"):
        os.environ["ARMOUR_TAIL_WORLDS"] = tail
        os.environ["ARMOUR_RESTO_CONCURRENT"] = conc
        try:
            planners.append(A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds)))
        finally:
            del os.environ["ARMOUR_TAIL_WORLDS"]
            del os.environ["ARMOUR_RESTO_CONCURRENT"]
    (res_c, _), (res_s, _) = [P.plan(worlds) for P in planners]
    assert sum(r["status"] == 4 for r in res_s) >= 8, "too few worlds in the restoration phase"
    for w, (a, b) in enumerate(zip(res_c, res_s)):
        assert np.array_equal(a["k_opt"], b["k_opt"]) and a["cost"] == b["cost"]
        assert (a["iterations"], a["evaluations"], a["status"], a["feasible"], a["error"]) == \
            (b["iterations"], b["evaluations"], b["status"], b["feasible"], b["error"]), w
        assert np.array_equal(planners[0].constraints(w), planners[1].constraints(w))


def test_inline_restart_after_other_worlds_finish():
    """A world whose restoration phase restarts the interior point inside ipm_loop (status
    WS_RESTART) while another world is still iterating, after which that other world converges and
    no world is left in a phase: run_solver must still collect and run the restarted world
    (it was left at status 7 and reported 'not planned'). Boundary worlds 1, 8 and 9 of
    the small set restart at iterations 1, 4 and 1 on the oracle; world 4 converges at 24 without
    a phase. Every result matches the oracle's plan and carries no error."""
    import os

    fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "boundary_small_T20_O6.npz")))
    T, O = int(fx["T"]), fx["obstacles"].shape[1]
    world = lambda w: (fx["q0"][w], fx["qd0"][w], fx["qdd0"][w], fx["q_des"][w], fx["obstacles"][w])
    P = A.Planner(T=T, max_obstacles=O, max_worlds=2)
    for pair in ((9, 4), (1, 4), (8, 4), (4, 9)):
        res, _ = P.plan([world(w) for w in pair])
        for w, r in zip(pair, res):
            ref = OraclePlanner(*world(w), T=T, threads=4)
            ref.reach()
            ro = ref.plan()
            assert r["error"] == 0, (pair, w, r)
            assert (r["status"], r["iterations"], r["feasible"]) == (ro["status"], ro["iterations"], ro["feasible"]), (pair, w)
            assert np.abs(r["k_opt"] - ro["k_opt"]).max() < 1e-8, (pair, w)


@pytest.mark.parametrize("search", ["adaptive", "one", "rounds"])
@pytest.mark.parametrize("tail", ["1000", "16"])
def test_sync_free_tail_matches_synchronised(tail, search):
    """Sync-free tail iterations (planner.hip run_solver: bounded grids, device-side list lengths,
    the running count read one iteration later) give bitwise the plans of the loop synchronised
    every iteration (ARMOUR_TAIL_WORLDS=0). "1000" runs every iteration after the first sync-free;
    also one world alone, the drop-in's batch. The tail's line search runs in one round of all
    trials (eval_trials_all, ipm_world_Cs_all: "one"), round by round ("rounds"), or picked per
    iteration by whether worlds backtracked ("adaptive", the default)."""
    import os

    T, O = 40, 10
    for worlds in ([A.make_world(s, O, profile="survey") for s in range(48)], [A.make_world(7, O, profile="survey")]):
        planners = []
        for tw in ("0", tail):
            os.environ["ARMOUR_TAIL_WORLDS"] = tw
            os.environ["ARMOUR_TAIL_SEARCH"] = search
            try:
                planners.append(A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds)))
            finally:
                del os.environ["ARMOUR_TAIL_WORLDS"]
                del os.environ["ARMOUR_TAIL_SEARCH"]
        (res_s, _), (res_t, _) = [P.plan(worlds) for P in planners]
        for w, (a, b) in enumerate(zip(res_s, res_t)):
            assert np.array_equal(a["k_opt"], b["k_opt"]) and a["cost"] == b["cost"]
            assert (a["iterations"], a["evaluations"], a["status"], a["feasible"]) == \
                (b["iterations"], b["evaluations"], b["status"], b["feasible"])
            assert np.array_equal(planners[0].constraints(w), planners[1].constraints(w))
            assert np.array_equal(planners[0].link_centers(w), planners[1].link_centers(w))


@pytest.mark.parametrize("T", [10, 14])
def test_short_horizon_plans_match_oracle(T):
    """Horizons shorter than the 2 NF + 1 = 15 extremum / cost tasks of a trial evaluation: the
    trial kernel (eval_trials_body) spreads them over blocks t = v (mod T), so some blocks take two.
    A batch (the speculative trial path) and single-world plans against the oracle's plans."""
    O = 3
    worlds = [A.make_world(900 + s, O) for s in range(6)]
    P = A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds))
    res, _ = P.plan(worlds)
    for w, r in enumerate(res):
        ro = OraclePlanner(*worlds[w], T=T, threads=4).plan()
        assert r["error"] == 0
        assert (r["feasible"], r["status"]) == (ro["feasible"], ro["status"]), (w, r["status"], ro["status"])
        it_tol = 5 if (r["status"] == 4 and not r["feasible"]) else 0
        assert abs(r["iterations"] - ro["iterations"]) <= it_tol, (w, r["iterations"], ro["iterations"])
        if r["status"] == 0 or r["feasible"]:
            np.testing.assert_allclose(r["k_opt"], ro["k_opt"], rtol=0, atol=1e-8)


@pytest.mark.parametrize("W", [1, 64])
def test_reach_span_on_the_device_clock(W):
    """armour_get_reach_span: the last reach launch's execution span on the device clock (first
    workgroup start to last workgroup end), for the per-job engine (one world) and the bundle engine
    (64 worlds, 6400 jobs): positive, and within the reach phase's host-timed wall time."""
    T, O = 100, 20
    P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
    worlds = [A.make_world(s, O, profile="survey") for s in range(W)]
    for _ in range(2):
        tm = P.reach(worlds)
    span = P.reach_span_ms()
    assert span == tm["reach_span_ms"]
    assert 0.0 < span <= tm["reach_ms"] + 0.05, (span, tm)


def test_row_pass_lds_accumulators_match_registers():
    """The fused row pass's wide-grid form (ipm_rows_DA_lds: the first 20 of pass A's Newton-matrix
    accumulators in LDS, one slot per thread, three waves per SIMD; launched when the grid holds at
    least four blocks per CU) gives bitwise the plans of the register form (ARMOUR_DA_REGS=1): 96
    headline worlds, 15 row blocks each, so the early iterations take the LDS form."""
    import os

    T, O = 100, 20
    worlds = [A.make_world(s, O, profile="survey") for s in range(96)]
    planners = []
    for regs in (False, True):
        if regs:
            os.environ["ARMOUR_DA_REGS"] = "1"
        try:
            planners.append(A.Planner(T=T, max_obstacles=O, max_worlds=len(worlds)))
        finally:
            os.environ.pop("ARMOUR_DA_REGS", None)
    (res_l, _), (res_r, _) = [P.plan(worlds) for P in planners]
    for w, (a, b) in enumerate(zip(res_l, res_r)):
        assert np.array_equal(a["k_opt"], b["k_opt"]) and a["cost"] == b["cost"], w
        assert (a["iterations"], a["evaluations"], a["status"], a["feasible"]) == \
            (b["iterations"], b["evaluations"], b["status"], b["feasible"]), w
        assert np.array_equal(planners[0].constraints(w), planners[1].constraints(w))
