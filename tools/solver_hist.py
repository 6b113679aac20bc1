"""Diagnostics: solver status / iteration / evaluation histogram of one batch of survey worlds."""
import os, sys, collections
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
import armour_amd as A
W = int(sys.argv[1]) if len(sys.argv) > 1 else 327
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
worlds = [A.make_world(s, 20, profile="survey") for s in range(W)]
res, tm = P.plan(worlds)
print("timing", tm)
st = collections.Counter((r["status"], r["feasible"]) for r in res)
print("status,feasible:", dict(st))
it = np.array([r["iterations"] for r in res]); ev = np.array([r["evaluations"] for r in res])
fe = np.array([r["feasible"] for r in res]).astype(bool)
for name, m in (("feasible", fe), ("infeasible", ~fe)):
    print(name, m.sum(), "iters mean %.1f max %d" % (it[m].mean(), it[m].max()), "evals mean %.1f" % ev[m].mean(),
          "iter hist", np.histogram(it[m], bins=[0, 10, 20, 30, 50, 75, 99, 101])[0].tolist())
print("plane cache", P.plane_cache_stats())
