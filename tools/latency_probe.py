"""Diagnostics: the drop-in's single-plan latency (one world per call) split into the planner's own
phases (armour_timing: reach, solver, total incl. copies) and the host wall time, at T = 100 and
128, survey worlds (the bench's latency leg, bench.py latency()).

usage: python tools/latency_probe.py [n_plans]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
for T in (100, 128):
    P = A.Planner(T=T, max_obstacles=20, max_worlds=1)
    ws = [[A.make_world(50_000 + s, 20, profile="survey")] for s in range(n)]
    P.plan(ws[0])
    rows = []
    for w in ws:
        t0 = time.perf_counter()
        res, tm = P.plan(w)
        wall = (time.perf_counter() - t0) * 1e3
        rows.append((wall, tm["total_ms"], tm["reach_ms"], tm["reach_kernel_ms"], tm["nlp_ms"], res[0]["iterations"]))
    a = np.array(rows)
    med = np.median(a, 0)
    print(f"T={T}: wall {med[0]:.2f} ms (max {a[:, 0].max():.2f}), total {med[1]:.2f}, reach {med[2]:.2f} "
          f"(kernel {med[3]:.2f}), nlp {med[4]:.2f}, iterations median {med[5]:.0f} max {a[:, 5].max():.0f}", flush=True)
    for r in rows[:6]:
        print("   wall %.2f total %.2f reach %.2f kernel %.2f nlp %.2f it %d" % r)
    P.close()
