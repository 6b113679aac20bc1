"""Diagnostics: the per-job engine's LDS-arena reach (ARMOUR_LDS_ARENA=1) against the HBM arena
(the default), bit for bit, over single-world reaches; prints mismatching jobs.
usage: python tools/lds_check.py [n] [T] [repeats]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rep = int(sys.argv[3]) if len(sys.argv) > 3 else 2
worlds = [A.make_world(s, 20, profile="survey") for s in range(n)]
H = A.Planner(T=T, max_obstacles=20, max_worlds=1)
os.environ["ARMOUR_LDS_ARENA"] = "1"
L = A.Planner(T=T, max_obstacles=20, max_worlds=1)
del os.environ["ARMOUR_LDS_ARENA"]
bad = 0
for s, w in enumerate(worlds):
    H.reach([w])
    ref = H.link_generators(0).reshape(T, -1), H.torque_radius(0).reshape(T, -1)
    for r in range(rep):
        L.reach([w])
        got = L.link_generators(0).reshape(T, -1), L.torque_radius(0).reshape(T, -1)
        jobs = sorted(set(np.where(np.any(ref[0] != got[0], axis=1))[0]) | set(np.where(np.any(ref[1] != got[1], axis=1))[0]))
        if jobs:
            bad += 1
            d0 = np.abs(ref[0] - got[0]).max(axis=1)
            d1 = np.abs(ref[1] - got[1]).max(axis=1)
            j = jobs[0]
            print(f"world {s} repeat {r}: {len(jobs)} jobs differ, first {[int(v) for v in jobs[:8]]}; "
                  f"max |d link gens| {d0.max():.3e} (job {int(d0.argmax())}), max |d torque radius| {d1.max():.3e}; "
                  f"job {int(j)}: {np.where(ref[0][j] != got[0][j])[0][:12].tolist()} ref {ref[0][j][:4]} got {got[0][j][:4]}",
                  flush=True)
print(f"{n} worlds x {rep}: {bad} mismatching reaches", flush=True)
