"""Diagnostics: time armour_eval_constraints (one eval_kernel over the whole batch) at W worlds."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
import armour_amd as A
W = int(sys.argv[1]) if len(sys.argv) > 1 else 256
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
P.reach([A.make_world(s, 20) for s in range(W)])
x = np.full(7, 0.2)
P.eval_constraints(0, x)
n = 10
t0 = time.perf_counter()
for _ in range(n):
    P.eval_constraints(0, x, jac=False)
dt = (time.perf_counter() - t0) / n
print(f"skip={os.environ.get('ARMOUR_EVAL_SKIP', '0')} W={W}: {dt * 1e3:.3f} ms per eval call (incl. host copies)")
