"""The headline workload's oracle fixture (tests/golden/bench_survey_T100_O20.npz, made by
tests/golden/make_bench_worlds.py): the worlds bench.py's default step plans — seeds 0..980 of
make_world(seed, 20, profile="survey") at T = 100 — with the oracle's plan of each.

Here: the generator still produces exactly those worlds (input digests), the oracle still
reproduces a sample of the plans, and the fixture covers what the workload holds (feasible and
infeasible worlds, every solver exit). The extension (seeds 981..3923) completes bench.py's default
step from round 5 on (three planners x 1308 worlds); tests/test_gpu_bench_worlds.py plans all 3924
on the GPU in those three concurrent batches and compares every world."""
import json
import os

import numpy as np
import pytest

import armour_amd as A
from oracle import OraclePlanner

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAME = "bench_survey_T100_O20"


def load():
    """seeds 0..980: the phase-1 and fidelity studies' worlds"""
    return dict(np.load(os.path.join(GOLD, NAME + ".npz")))


def load_step():
    """the worlds of bench.py's default step: the base fixture and its extension (seeds 981..3923,
    tests/golden/make_bench_worlds.py --extend), concatenated"""
    a, b = load(), dict(np.load(os.path.join(GOLD, NAME + "_ext.npz")))
    return {k: (np.concatenate([a[k], b[k]]) if np.ndim(a[k]) else a[k]) for k in a}


def digest(world):
    import hashlib

    h = hashlib.sha1()
    for a in world:
        h.update(np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes())
    return np.frombuffer(h.digest(), dtype=np.uint8)


def bench_world(fx, i):
    return A.make_world(int(fx["seed"][i]), int(fx["O"]), profile="survey")


def test_generator_reproduces_the_fixture_worlds():
    fx = load_step()
    assert list(fx["seed"]) == list(range(3 * 1308))
    for i in range(len(fx["seed"])):
        assert np.array_equal(digest(bench_world(fx, i)), fx["digest"][i]), f"world {i} changed"


def test_fixture_covers_the_workload():
    fx = load()
    st = fx["status"]
    assert 0.5 < fx["feasible"].mean() < 0.75          # ~62 % feasible: the solver works against active limits
    # infeasible worlds end in the restoration phase's local-infeasibility verdict (status 4)
    assert (st == 0).sum() > 500 and (st == 4).sum() > 300
    # every converged plan is a KKT point to the reference's tolerance (IPOPT_OPTIMIZATION_TOLERANCE
    # 1e-4, KPR/Parameters.h:50), with the Ipopt scaling of the error (ipm.cpp)
    assert np.all(fx["kkt"][st == 0] <= 1e-4)
    # converged plans are feasible; an infeasible plan never reports convergence
    assert np.all(fx["feasible"][st == 0])


@pytest.mark.parametrize("i", [1, 5, 55, 300])
def test_oracle_reproduces_fixture_plans(i):
    """converged (1), infeasible (5, 300) and iteration-limit (55) worlds re-planned"""
    assert int(load()["status"][55]) == 1
    fx = load()
    R = OraclePlanner(*bench_world(fx, i), T=int(fx["T"]), threads=8)
    R.reach()
    r = R.plan()
    assert r["feasible"] == bool(fx["feasible"][i]) and r["status"] == fx["status"][i]
    assert r["iterations"] == fx["iterations"][i]
    np.testing.assert_allclose(r["k_opt"], fx["k_opt"][i], rtol=0, atol=1e-10)


def test_cap_study_recorded():
    """the worlds that end at the 100-iteration cap, re-planned with Ipopt's default limit of 3000
    (tests/golden/bench_cap_study.json): every one keeps its verdict (the re-check at the final
    iterate, KPR/NLPclass.cu:449-538), so the cap changes no decision"""
    rec = json.load(open(os.path.join(GOLD, "bench_cap_study.json")))
    fx = load()
    assert len(rec["worlds"]) == int((fx["status"] == 1).sum()) > 0
    for w in rec["worlds"]:
        assert w["cap100"]["feasible"] == w["cap3000"]["feasible"]
        assert w["cap3000"]["iterations"] < 3000
