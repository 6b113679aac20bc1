"""The reference's 100 saved worlds (SURVEY.md §8(d) fixed real-world check; fixture
tests/golden/saved_worlds_T100.npz, made by tests/golden/make_saved_worlds.py): the fixture's
worlds are the reference's CSV rows, and the oracle reproduces its plans."""
import os

import numpy as np
import pytest

from oracle import OraclePlanner

HERE = os.path.dirname(os.path.abspath(__file__))


def saved_worlds():
    """(names, worlds, expected) of the fixture; worlds rebuilt from the stored CSV rows"""
    from armour_amd.worlds import csv_world

    fx = np.load(os.path.join(HERE, "golden", "saved_worlds_T100.npz"))
    worlds = []
    for r in fx["rows"]:
        n = int(np.max(np.nonzero(~np.all(np.isnan(r), axis=1))[0])) + 1  # drop the padding rows
        worlds.append(csv_world(r[:n]))
    return fx["names"], worlds, fx


def test_fixture_is_the_reference_world_set():
    names, worlds, fx = saved_worlds()
    assert len(names) == 100 and len(set(names.tolist())) == 100 and int(fx["T"]) == 100
    for (q0, qd0, qdd0, qdes, obs), n in zip(worlds, fx["num_obstacles"]):
        assert obs.shape == (n, 12) and np.all(qd0 == 0) and np.all(qdd0 == 0)
        np.testing.assert_allclose(np.linalg.norm(qdes - q0), 0.1, rtol=1e-12)


@pytest.mark.parametrize("i", [0, 37, 99])
def test_oracle_reproduces_saved_world(i):
    names, worlds, fx = saved_worlds()
    P = OraclePlanner(*worlds[i], T=100, threads=4)
    P.reach()
    r = P.plan()
    assert r["feasible"] == bool(fx["feasible"][i]), names[i]
    assert r["status"] == int(fx["status"][i]) and r["iterations"] == int(fx["iterations"][i]), names[i]
    np.testing.assert_allclose(r["k_opt"], fx["k_opt"][i], rtol=0, atol=1e-10)
