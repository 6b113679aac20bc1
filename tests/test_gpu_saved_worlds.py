"""The HIP path on the reference's 100 saved worlds at T = 100 (SURVEY.md §8(d) fixed real-world
check) against the oracle's plans in tests/golden/saved_worlds_T100.npz: feasibility, solver status
and iteration counts identical, k_opt within 1e-8. Worlds are batched by obstacle count (a batch
shares num_obstacles)."""
import numpy as np
import pytest

import armour_amd as A
from test_saved_worlds import saved_worlds

pytestmark = pytest.mark.gpu


def test_saved_worlds_match_oracle():
    names, worlds, fx = saved_worlds()
    counts = fx["num_obstacles"]
    done = 0
    for O in sorted(set(counts.tolist())):
        idx = [i for i in range(len(worlds)) if counts[i] == O]
        P = A.Planner(T=100, max_obstacles=O, max_worlds=len(idx))
        res, _ = P.plan([worlds[i] for i in idx])
        for i, r in zip(idx, res):
            assert r["feasible"] == bool(fx["feasible"][i]), names[i]
            assert r["status"] == int(fx["status"][i]), names[i]
            assert r["iterations"] == int(fx["iterations"][i]), names[i]
            np.testing.assert_allclose(r["k_opt"], fx["k_opt"][i], rtol=0, atol=1e-8, err_msg=str(names[i]))
            np.testing.assert_allclose(r["cost"], fx["cost"][i], rtol=1e-8, atol=1e-12, err_msg=str(names[i]))
            done += 1
        P.close()
    assert done == 100


def test_saved_worlds_monotone_barrier_option():
    """The monotone barrier (ARMOUR_MU_STRATEGY=monotone; the default is the reference's adaptive
    strategy, KPR/Parameters.h:57) against the oracle's monotone solve (mu_strategy 0) on the saved
    worlds with 10 obstacles: the same bar as the default, decisions, status and iteration counts
    identical and k_opt within 1e-8."""
    import os

    from oracle import OraclePlanner

    names, worlds, fx = saved_worlds()
    idx = [i for i in range(len(worlds)) if fx["num_obstacles"][i] == 10]
    os.environ["ARMOUR_MU_STRATEGY"] = "monotone"
    try:
        P = A.Planner(T=100, max_obstacles=10, max_worlds=len(idx))
    finally:
        os.environ.pop("ARMOUR_MU_STRATEGY", None)
    res, _ = P.plan([worlds[i] for i in idx])
    its = []
    for i, r in zip(idx, res):
        R = OraclePlanner(*worlds[i], T=100, threads=8)
        R.reach()
        ro = R.plan(mu_strategy=0)
        assert r["feasible"] == ro["feasible"] and r["status"] == ro["status"], names[i]
        assert r["iterations"] == ro["iterations"], names[i]
        np.testing.assert_allclose(r["k_opt"], ro["k_opt"], rtol=0, atol=1e-8, err_msg=str(names[i]))
        its.append((r["iterations"], int(fx["iterations"][i])))
    print(f"{len(idx)} worlds; iterations (monotone, adaptive default): {its}")
