"""Bitwise A/B of whole plans (k_opt, status, iterations, evaluations, cost, KKT error, final link
centres) between two
library builds, at the bench configuration (development tool).
usage: python tools/plan_ab.py <lib_a> <lib_b> [worlds]"""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(%r, 'armour-dev_amd'))
import armour_amd as A
W = int(sys.argv[2])
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
res, _ = P.plan([A.make_world(1000 + s, 20) for s in range(W)])
np.save(sys.argv[1], np.array([np.concatenate([r["k_opt"], [r["feasible"], r["status"], r["iterations"],
                                               r["evaluations"], r["cost"], r["kkt"]], P.link_centers(w).ravel()])
                               for w, r in enumerate(res)]))
'''
W = sys.argv[3] if len(sys.argv) > 3 else "64"
outs = []
for i, lib in enumerate(sys.argv[1:3]):
    f = f"/tmp/plan_ab_{i}.npy"
    subprocess.run([sys.executable, "-c", code % ROOT, f, W], env=dict(os.environ, ARMOUR_LIB=os.path.abspath(lib)),
                   check=True, timeout=300)
    outs.append(np.load(f))
a, b = outs
same = np.array_equal(a, b)
print(f"plans bitwise equal: {same}  worlds {len(a)}  differing worlds {int(np.sum(np.any(a != b, axis=1)))}"
      f"  max |dk| {np.max(np.abs(a[:, :7] - b[:, :7])):.3g}  iterations equal {np.array_equal(a[:, 9], b[:, 9])}")
sys.exit(0 if same else 1)
