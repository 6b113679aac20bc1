"""Bitwise A/B of armour_eval_constraints between two library builds (development tool).
usage: python tools/eval_ab.py <lib_a> <lib_b>"""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(%r, 'armour-dev_amd'))
import armour_amd as A
W, T, O = 6, 40, 20
P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
P.reach([A.make_world(s, O) for s in range(W)])
out = []
for x in [np.zeros(7), np.linspace(-0.8, 0.8, 7), np.full(7, 0.37)]:
    for w in range(W):
        g, J = P.eval_constraints(w, x)
        out.append(np.concatenate([g, J.ravel()]))
np.save(sys.argv[1], np.stack(out))
'''
outs = []
for i, lib in enumerate(sys.argv[1:3]):
    f = f"/tmp/eval_ab_{i}.npy"
    subprocess.run([sys.executable, "-c", code % ROOT, f], env=dict(os.environ, ARMOUR_LIB=os.path.abspath(lib)),
                   check=True, timeout=300)
    outs.append(np.load(f))
a, b = outs
print("bitwise equal:", np.array_equal(a, b), "max |diff|", np.abs(a - b).max(), "values", a.size)
