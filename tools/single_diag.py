"""Diagnostics: single-world plans (one world per call, the drop-in's batch) of survey worlds under
environment variants, as (status, iterations) per world, for comparison with the oracle's.
usage: python tools/single_diag.py [n] [T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
worlds = [A.make_world(s, 20, profile="survey") for s in range(n)]
for env in ({}, {"ARMOUR_LDS_ARENA": "0"}, {"ARMOUR_TAIL_WORLDS": "0"}, {"ARMOUR_ENGINE": "lane"},
            {"ARMOUR_RESTORATION": "0"}, {"ARMOUR_NO_SPEC": "1"}):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        P = A.Planner(T=T, max_obstacles=20, max_worlds=1)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    out = []
    for w in worlds:
        (r,), _ = P.plan([w])
        out.append((r["status"], r["iterations"]))
    print(env, out, flush=True)
