"""One planner, one warm-up and one traced plan of a batch (for rocprofv3 --kernel-trace timelines of
the solver). Usage: nlp_trace.py [profile] [W]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

prof = sys.argv[1] if len(sys.argv) > 1 else "survey"
T, O = 100, 20
W = int(sys.argv[2]) if len(sys.argv) > 2 else A.default_batch(T)
P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
worlds = [A.make_world(s, O, profile=prof) for s in range(W)]
P.plan(worlds)
res, tm = P.plan(worlds)
print(tm, flush=True)
