"""Bitwise A/B of two library builds (development tool): the same worlds planned by the in-tree
library and by a variant next to it (armour-dev_amd/armour_amd/<variant>.so, loaded through
ARMOUR_LIB in a child process each), then k_opt, cost, iterations, evaluations, status and the
constraint values compared bit for bit.

usage: python tools/plan_ab.py <variant .so name> [W] [T] [profile] [batch]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def child(lib, W, T, profile, batch, out):
    os.environ["ARMOUR_LIB"] = os.path.join(ROOT, "armour-dev_amd", "armour_amd", lib)
    sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
    import armour_amd as A

    worlds = [A.make_world(s, 20, profile=profile) for s in range(W)]
    P = A.Planner(T=T, max_obstacles=20, max_worlds=batch)
    rec = {k: [] for k in ("k", "cost", "it", "ev", "st", "g")}
    for b0 in range(0, W, batch):
        res, _ = P.plan(worlds[b0:b0 + batch])
        for w, r in enumerate(res):
            rec["k"].append(r["k_opt"]); rec["cost"].append(r["cost"]); rec["it"].append(r["iterations"])
            rec["ev"].append(r["evaluations"]); rec["st"].append(r["status"]); rec["g"].append(P.constraints(w))
    np.savez(out, **{k: np.array(v) for k, v in rec.items()})


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], int(sys.argv[6]), sys.argv[7])
        sys.exit(0)
    var = sys.argv[1]
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 96
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    profile = sys.argv[4] if len(sys.argv) > 4 else "survey"
    batch = int(sys.argv[5]) if len(sys.argv) > 5 else W
    os.makedirs(OUT, exist_ok=True)
    outs = []
    for lib in ("libarmour_hip.so", var):
        o = os.path.join(OUT, f"plan_ab_{lib}.npz")
        subprocess.run([sys.executable, __file__, "--child", lib, str(W), str(T), profile, str(batch), o], check=True)
        outs.append(dict(np.load(o)))
    a, b = outs
    bad = [k for k in a if not np.array_equal(a[k], b[k])]
    nw = int(np.sum(np.any(a["k"] != b["k"], axis=1) | (a["it"] != b["it"])))
    print(f"{W} worlds (T={T}, {profile}, batches of {batch}): fields differing {bad or 'none'}, worlds differing {nw}")
    sys.exit(1 if bad else 0)
