"""The headline workload on the GPU against the oracle, world by world.

bench.py's default step at N = 1 plans seeds 0..3923 of make_world(seed, 20, profile="survey") at
T = 100 as three concurrent planners x 1308 worlds (one host thread and HIP stream each; 2044 64-job
bundles per planner, eight waves of the device's 256 CUs). This test runs exactly that step and compares every world
with the oracle's plan frozen in tests/golden/bench_survey_T100_O20.npz and its extension _ext.npz
(tests/golden/make_bench_worlds.py):

  * feasibility (finalize_solution, KPR/NLPclass.cu:422-538) and solver status identical for all
    3924 worlds;
  * the solver's path (iteration count, and k_opt within 1e-8 for a converged or feasible plan)
    identical for at least 99.5 % of them; see the bar at the end. An infeasible plan writes -1
    (KPR/armour_main.cu:326-334), so its k_opt is not an output; its iterates run through nearly
    singular Newton systems that amplify rounding-level differences of g / J (DESIGN.md §2,
    profiles/r02_ipm_divergence.log), and it is held to identical status and feasibility (its
    iteration count and k_opt difference are reported; it counts against the 0.5 % off-path bar).
"""
import os
import threading

import numpy as np
import pytest

import armour_amd as A
from test_bench_worlds import digest, load, load_step

pytestmark = pytest.mark.gpu


def test_bench_step_matches_oracle_world_by_world():
    fx = load_step()
    T, O, W = int(fx["T"]), int(fx["O"]), len(fx["seed"])
    batch = 1308
    assert 4 * A.default_batch(T) == batch, "the bench's default batch on this device"
    worlds = [A.make_world(int(s), O, profile="survey") for s in fx["seed"]]
    for i in (0, W // 2, W - 1):
        assert np.array_equal(digest(worlds[i]), fx["digest"][i])
    subs = [worlds[p * batch:(p + 1) * batch] for p in range(3)]
    planners = [A.Planner(T=T, max_obstacles=O, max_worlds=batch) for _ in range(3)]
    out, errs = [None] * 3, [None] * 3

    def work(p):
        try:
            out[p] = planners[p].plan(subs[p])[0]
        except BaseException as e:  # noqa: BLE001 (re-raised below)
            errs[p] = e

    for _ in range(2):  # the bench's warm-up step, then the compared step
        ths = [threading.Thread(target=work, args=(p,)) for p in range(3)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        for e in errs:
            if e is not None:
                raise e
    res = [r for o in out for r in o]
    assert len(res) == W
    n_feas = sum(r["feasible"] for r in res)
    assert all(r["error"] == 0 for r in res)
    # decisions: identical for every world
    dec = [i for i, r in enumerate(res) if r["feasible"] != bool(fx["feasible"][i]) or r["status"] != fx["status"][i]]
    assert not dec, [(i, res[i]["feasible"], res[i]["status"], int(fx["status"][i])) for i in dec]
    # the solver's path: iteration counts and k_opt (converged / feasible plans)
    it_diff = [i for i, r in enumerate(res) if r["iterations"] != fx["iterations"][i]]
    ok = [r["status"] == 0 or r["feasible"] for r in res]
    dk = np.array([np.abs(r["k_opt"] - fx["k_opt"][i]).max() for i, r in enumerate(res)])
    dcost = np.array([abs(r["cost"] - fx["cost"][i]) / max(1e-12, abs(fx["cost"][i])) for i, r in enumerate(res)])
    k_diff = [i for i in range(W) if ok[i] and dk[i] > 1e-8]
    for i in sorted(set(it_diff) | set(k_diff)):
        r = res[i]
        print(f"  world {i}: feasible={r['feasible']} status={r['status']} iterations {r['iterations']} "
              f"(oracle {int(fx['iterations'][i])}) |dk_opt|={dk[i]:.2e} |dcost|/cost={dcost[i]:.2e}")
    okm = np.array(ok)
    print(f"bench step: {W} worlds, {n_feas} feasible; identical iteration counts {W - len(it_diff)}/{W}; "
          f"converged/feasible k_opt within 1e-8: {int(okm.sum()) - len(k_diff)}/{int(okm.sum())} "
          f"(max {dk[okm].max():.1e}); infeasible plans' k_opt (not an output) max |dk| {dk[~okm].max():.1e}")
    # Bar: every decision identical (above); at least 99.5 % of the worlds on the oracle's exact
    # solver path (same iteration count, k_opt within 1e-8). The rest are long solves through
    # ill-conditioned Newton systems, where ~1e-14 differences of g / J (summation order of the
    # reach engines) grow to a different path: a converged or feasible plan within 10 iterations
    # and within the solver's tolerance scale (k_opt 1e-4, cost 1e-6 relative). An infeasible
    # plan's output is -1 whatever iteration its line search gives up at; its iteration count is
    # held to within 40 of the oracle's (the largest gap observed is 34). Observed (r05 and r06,
    # 3924 worlds): 7 off the path — infeasible worlds 127, 1479, 3267, 3887, 3913 (2, 34, 1, 1, 1
    # iterations apart) and the 31-iteration converged worlds 489, 1491 (k_opt 1.4e-7 and 3.6e-8
    # away). The seeds off the path are printed above (the set moves with rounding-level changes of
    # the evaluation's arithmetic, so it is bounded, not frozen).
    assert len(set(it_diff) | set(k_diff)) <= W // 200
    assert all(abs(res[i]["iterations"] - int(fx["iterations"][i])) <= 10 for i in it_diff if ok[i])
    assert all(abs(res[i]["iterations"] - int(fx["iterations"][i])) <= 40 for i in it_diff)
    assert dk[okm].max() <= 1e-4 and dcost[okm].max() <= 1e-6
    # the converged plans' KKT error (Ipopt-scaled, as the solver's stopping test) is within tol
    kkt = np.array([r["kkt"] for r in res])
    st = np.array([r["status"] for r in res])
    assert np.all(kkt[st == 0] <= 1e-4)


def test_single_world_plans_match_oracle():
    """The drop-in's batch — one world per call — takes other paths than the bench step: the
    per-job reach engine (reach_kernel<256>), the sync-free tail from the
    second iteration, and restoration phases after the interior-point loop. The first 48 headline
    worlds planned one at a time against the same frozen oracle plans: every decision identical,
    and the solver's path (iterations, k_opt within 1e-8 when converged or feasible) for all but
    at most one of them."""
    fx = load()
    T, O = int(fx["T"]), int(fx["O"])
    n = 48
    P = A.Planner(T=T, max_obstacles=O, max_worlds=1)
    off = []
    for i in range(n):
        (r,), _ = P.plan([A.make_world(int(fx["seed"][i]), O, profile="survey")])
        assert r["feasible"] == bool(fx["feasible"][i]) and r["status"] == fx["status"][i], \
            (i, r["feasible"], r["status"], int(fx["status"][i]), r["iterations"], int(fx["iterations"][i]))
        dk = float(np.abs(r["k_opt"] - fx["k_opt"][i]).max())
        if r["iterations"] != fx["iterations"][i] or ((r["status"] == 0 or r["feasible"]) and dk > 1e-8):
            off.append((i, r["iterations"], int(fx["iterations"][i]), dk))
    print(f"single-world plans: {n - len(off)}/{n} on the oracle's path; off: {off}")
    assert len(off) <= 1, off
