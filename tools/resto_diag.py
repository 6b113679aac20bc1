"""Diagnostics: per-world status / iterations / evaluations of a boundary fixture under the
restoration variants (default inline phases, ARMOUR_RESTO_INLINE=0, ARMOUR_RESTO_ROUNDS=1,
ARMOUR_RESTORATION=0) and both reach engines, next to the frozen fixture's oracle counts.
usage: python tools/resto_diag.py [fixture]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "boundary_small_T20_O6"
fx = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz")))
T, W, O = int(fx["T"]), len(fx["kinds"]), fx["obstacles"].shape[1]
worlds = [(fx["q0"][w], fx["qd0"][w], fx["qdd0"][w], fx["q_des"][w], fx["obstacles"][w]) for w in range(W)]
assert str(fx.get("robot", "kinova")) == "kinova", "Kinova fixtures only"
tables = None
print("fixture iterations", [int(v) for v in fx["iterations"]], flush=True)
for eng in ("lane", "job"):
    for env in ({}, {"ARMOUR_RESTO_INLINE": "0"}, {"ARMOUR_RESTO_ROUNDS": "1"}, {"ARMOUR_RESTORATION": "0"},
                {"ARMOUR_TAIL_WORLDS": "0"}, {"ARMOUR_NO_SPEC": "1"}):
        env = dict(env, ARMOUR_ENGINE=eng)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            P = A.Planner(T=T, max_obstacles=O, max_worlds=W, robot=tables)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
        res, _ = P.plan(worlds)
        print(env, [(r["status"], r["iterations"], r["evaluations"]) for r in res], flush=True)
