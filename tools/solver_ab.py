"""A/B of two library builds on the solver's latency (development tool): one planner, survey worlds,
T=100, O=20, batches of 1, 8 and 32 worlds (the drop-in's plan and config 4's shares), each build in
its own process, alternating twice; prints the median solver (nlp) and total times and checks that
both builds plan bitwise alike.

usage: python tools/solver_ab.py <lib_a.so> <lib_b.so> [reps]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.join(%r, "armour-dev_amd"))
import armour_amd as A
W, reps = %d, %d
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
t, plans = [], []
for r in range(reps + 1):
    ws = [A.make_world(70_000 + 97 * r + s, 20, profile="survey") for s in range(W)]
    res, tm = P.plan(ws)
    if r > 0:
        t.append((tm["nlp_ms"], tm["total_ms"]))
    plans.append([(list(map(float, x["k_opt"])), x["iterations"], x["status"]) for x in res])
t = np.array(t)
print(json.dumps({"nlp": float(np.median(t[:, 0])), "total": float(np.median(t[:, 1])), "plans": plans}))
'''
libs = sys.argv[1:3]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
for W in (1, 8, 32):
    got = {}
    for rep in range(2):
        for lib in libs:
            env = dict(os.environ, ARMOUR_LIB=os.path.abspath(lib))
            r = subprocess.run([sys.executable, "-c", code % (ROOT, W, reps)], env=env, capture_output=True, text=True,
                               timeout=300)
            if r.returncode != 0:
                raise SystemExit(r.stderr[-2000:])
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            got.setdefault(lib, []).append(rec)
            print(f"W={W:3d} {os.path.basename(lib):28s} nlp {rec['nlp']:7.2f} ms  total {rec['total']:7.2f} ms", flush=True)
    a, b = (got[lib][0]["plans"] for lib in libs)
    assert a == b, f"plans differ at W={W}"
print("plans bitwise equal")
