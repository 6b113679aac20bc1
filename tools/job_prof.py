"""Diagnostics: per-op and per-phase cycle profile of the per-job reach engine (reach_kernel.hip)
on the latency workload: W survey worlds (default 1), T = 100, O = 20, ARMOUR_ENGINE=job.

usage: python tools/job_prof.py [W] [T]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
os.environ["ARMOUR_ENGINE"] = "job"
import armour_amd as A  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1
T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
NAMES = ["JRS", "MAKE1D", "MAKEROT", "MAKEBOX", "CONST", "ZERO", "VIEW", "TRANSPOSE", "MUL", "ADD", "STACK3", "ADD1D",
         "EMIT_LINK", "EMIT_TORQUE", "TORQUE_RADIUS", "CROSS_C", "CROSS_PP"]
worlds = [A.make_world(s, 20, profile="survey") for s in range(W)]

P = A.Planner(T=T, max_obstacles=20, max_worlds=W)
P.reach(worlds)
ts = [P.reach(worlds)["reach_kernel_ms"] for _ in range(5)]
print(f"W={W} T={T}: reach kernel {min(ts):.3f} ms (min of 5), {np.median(ts):.3f} median", flush=True)
P.close()

os.environ["ARMOUR_PROFILE_OPS"] = "1"
P = A.Planner(T=T, max_obstacles=20, max_worlds=W)
P.reach(worlds)
prof, _ = P.reach_profile()
codes = P.reach_program()
prof = prof.astype(np.float64)
jobs = W * T
tot = prof[:, 0].sum()
print(f"profile: {len(codes)} ops, {tot / jobs:.4g} cycles/job (thread 0, includes the stamps)")
for c in range(len(NAMES)):
    m = codes == c
    if m.any():
        print(f"  {NAMES[c]:14s} n={m.sum():4d} cycles/job {prof[m, 0].sum() / jobs:9.0f} ({100 * prof[m, 0].sum() / tot:5.1f}%)"
              f" terms/job {prof[m, 1].sum() / jobs:8.0f}")
terms = prof[:, 1] / jobs
for lo, hi in [(-1, 0), (0, 16), (16, 64), (64, 256), (256, 1024), (1024, 1 << 30)]:
    m = (((codes >= 8) & (codes <= 11)) | (codes >= 15)) & (terms > lo) & (terms <= hi)
    print(f"  terms in ({lo},{hi}]: ops {m.sum():4d} cycles/job {prof[m, 0].sum() / jobs:9.0f}"
          f" ({100 * prof[m, 0].sum() / tot:5.1f}%) per op {prof[m, 0].sum() / jobs / max(m.sum(), 1):7.0f}")
for k in np.argsort(-prof[:, 0])[:12]:
    print(f"  op {k:4d} {NAMES[codes[k]]:8s} cycles/job {prof[k, 0] / jobs:8.0f} terms/job {prof[k, 1] / jobs:7.1f}")
P.close()

os.environ["ARMOUR_PROFILE_OPS"] = "2"
P = A.Planner(T=T, max_obstacles=20, max_worlds=W)
P.reach(worlds)
_, phase = P.reach_profile()
ph = phase.astype(np.float64) / jobs
print("big-path phases cycles/job [-, order, pass1, scan+alloc, pass2, blocksum, stage, -]:", ph[:8].round(0))
print("small-path phases cycles/job [load, sort, groups, keep+write, reduce+finish]:", ph[8:13].round(0),
      "between ops", ph[13].round(0), "headers", ph[14].round(0), "other", ph[15].round(0))
print("sum of phases", ph.sum().round(0))
P.close()
