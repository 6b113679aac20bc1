"""Diagnostics for PMC passes on eval_kernel: one planner, the bench batch of SURVEY §8(d) worlds,
reach once, then 5 full evaluations (g and the dense Jacobian) at one point."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else A.default_batch(100)
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
P.reach([A.make_world(s, 20, profile="survey") for s in range(W)])
for _ in range(5):
    P.eval_constraints(0, np.full(7, 0.2))
print(f"eval_pmc: W={W}", flush=True)
