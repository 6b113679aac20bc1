"""First solver iteration where the HIP armour-IPM and the oracle's leave each other, per world of a
boundary fixture (plans capped at k iterations, k = 1, 2, ...). Diagnostics."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("armour-dev_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import armour_amd as A  # noqa: E402
from oracle import OraclePlanner  # noqa: E402
from test_boundary import load, world  # noqa: E402


FULL = bool(os.environ.get("DIVERGE_FULL"))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "boundary_small_T20_O6"
    only = [int(v) for v in sys.argv[2:]]
    fx = load(name)
    T, W, O = int(fx["T"]), len(fx["kinds"]), fx["obstacles"].shape[1]
    for w in (only or range(W)):
        wd = world(fx, w)
        R = OraclePlanner(*wd, T=T, threads=8)
        R.reach()
        full = R.plan()
        first = None
        rows = []
        for k in range(1, full["iterations"] + 2):
            P = A.Planner(T=T, max_obstacles=O, max_worlds=1, max_iter=k)
            r = P.plan([wd])[0][0]
            ro = R.plan(max_iter=k)
            dx = float(np.abs(r["k_opt"] - ro["k_opt"]).max())
            rows.append((k, r["iterations"], ro["iterations"], r["status"], ro["status"], dx, r["cost"], ro["cost"]))
            P.close()
            if first is None and (dx > 1e-10 or r["status"] != ro["status"] or r["iterations"] != ro["iterations"]):
                first = k
                if not FULL:
                    break
        print(json.dumps(dict(world=w, kind=str(fx["kinds"][w]), oracle_iters=full["iterations"], first_divergence=first,
                              trace=rows if FULL else rows[-3:])), flush=True)


if __name__ == "__main__":
    main()
