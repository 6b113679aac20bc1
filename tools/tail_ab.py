"""A/B of a solver option that is read at planner creation (development tool): two planners in one
process, one created with ENV=VALUE set, planning the same survey worlds alternately; prints the
median solver (nlp) and total times per batch size and checks that the plans are bitwise equal.

usage: python tools/tail_ab.py ENV=VALUE [reps]    e.g. ARMOUR_TAIL_ROUNDS=1"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

key, val = sys.argv[1].split("=", 1)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for W in (1, 8, 32):
    Ps = []
    for on in (False, True):
        if on:
            os.environ[key] = val
        try:
            Ps.append(A.Planner(T=100, max_obstacles=20, max_worlds=W))
        finally:
            os.environ.pop(key, None)
    times = {0: [], 1: []}
    for r in range(reps + 1):
        ws = [A.make_world(70_000 + 97 * r + s, 20, profile="survey") for s in range(W)]
        outs = []
        for i, P in enumerate(Ps):
            res, tm = P.plan(ws)
            outs.append(res)
            if r > 0:
                times[i].append((tm["nlp_ms"], tm["total_ms"], max(x["iterations"] for x in res)))
        for a, b in zip(*outs):
            assert np.array_equal(a["k_opt"], b["k_opt"]) and a["cost"] == b["cost"], "plans differ"
            assert (a["iterations"], a["evaluations"], a["status"]) == (b["iterations"], b["evaluations"], b["status"])
    for i, name in ((0, "default"), (1, f"{key}={val}")):
        t = np.array(times[i])
        print(f"W={W:3d} {name:24s} nlp {np.median(t[:, 0]):7.2f} ms  total {np.median(t[:, 1]):7.2f} ms  "
              f"(max iterations median {np.median(t[:, 2]):.0f}; nlp/iteration {np.median(t[:, 0] / t[:, 2]) * 1e3:.0f} us)",
              flush=True)
    for P in Ps:
        P.close()
print("plans bitwise equal")
