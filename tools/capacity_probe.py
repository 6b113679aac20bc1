"""Reach-set capacity headroom (armour_get_reach_occupancy) over world families: per world alone at
T=64 (one bundle = one world), then batches of SURVEY §8(d) full-range worlds. Prints JSON lines."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import armour_amd as A  # noqa: E402

DEBUG = (np.array([-1.0, -1, -1, -1, 1, 1, 1]), np.array([1.0, 1, 1, -1, -1, -1, -1]), np.full(7, 2.0))


def main():
    n_survey = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    T, O = 64, 20
    P = A.Planner(T=T, max_obstacles=O, max_worlds=1)
    fam = {"default": A.make_world(1, O), "survey": A.make_world(1, O, profile="survey"),
           "rest": (A.make_world(1, O)[0], np.zeros(7), np.zeros(7)) + A.make_world(1, O)[3:],
           "debug": DEBUG + (DEBUG[0] + 0.05, A.make_world(1, O)[4])}
    for k, w in fam.items():
        P.reach([w])
        print(json.dumps(dict(family=k, T=T, occ=P.occupancy())), flush=True)
    P.close()
    T = 100
    B = A.default_batch(T)
    P = A.Planner(T=T, max_obstacles=O, max_worlds=B)
    worst = {}
    failed = 0
    t0 = time.time()
    for s0 in range(0, n_survey, B):
        worlds = [A.make_world(s, O, profile="survey") for s in range(s0, min(n_survey, s0 + B))]
        res, tm = P.plan(worlds)
        occ = P.occupancy()
        failed += sum(r["error"] != 0 for r in res)
        for k, (u, c) in occ.items():
            worst[k] = (max(u, worst.get(k, (0, c))[0]), c)
        print(json.dumps(dict(batch=s0, n=len(worlds), occ=occ, feasible=sum(r["feasible"] for r in res),
                              reach_ms=tm["reach_ms"], nlp_ms=tm["nlp_ms"])), flush=True)
    print(json.dumps(dict(summary="survey", worlds=n_survey, failed=failed, worst=worst, seconds=time.time() - t0)))


if __name__ == "__main__":
    main()
