"""Generate tests/golden/saved_worlds_T100.npz (run from the repo root in the build container):

    python tests/golden/make_saved_worlds.py [--ref /root/reference]

SURVEY.md §8(d)'s fixed real-world check: all 100 saved worlds of the reference
(kinova_src/saved_worlds/random/scene_<O>_<i>.csv, 13-40 box obstacles; parsed numbers only, the
CSV rows are stored as data) as first replans at T = 100 (armour_amd.worlds.csv_world: rest start,
straight-line waypoint), with the CPU restatement's plan of each (oracle/): k_opt, feasibility,
solver status, iterations, evaluations, cost. tests/test_saved_worlds.py pins the oracle against
the fixture; tests/test_gpu_saved_worlds.py the HIP path. Parity with the reference itself is
unpinned (it ships no outputs)."""
from __future__ import annotations

import argparse
import glob
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from armour_amd.worlds import csv_world  # noqa: E402
from oracle import OraclePlanner  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "saved_worlds_T100.npz")
T = 100


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.ref, "kinova_src", "saved_worlds", "random", "scene_*.csv")))
    assert len(files) == 100, len(files)
    tabs = [np.genfromtxt(fn, delimiter=",") for fn in files]
    R = max(t.shape[0] for t in tabs)
    rows = np.full((len(tabs), R, 7), np.nan)
    for i, t in enumerate(tabs):
        rows[i, :t.shape[0], :t.shape[1]] = t
    names = np.array([os.path.basename(f)[:-4] for f in files])
    out = {k: [] for k in ("k_opt", "feasible", "status", "iterations", "evaluations", "cost", "num_obstacles")}
    t0 = time.time()
    for i, t in enumerate(tabs):
        q0, qd0, qdd0, qdes, obs = csv_world(t)
        P = OraclePlanner(q0, qd0, qdd0, qdes, obs, T=T, threads=a.threads)
        P.reach()
        r = P.plan()
        out["k_opt"].append(r["k_opt"])
        out["feasible"].append(int(r["feasible"]))
        out["status"].append(r["status"])
        out["iterations"].append(r["iterations"])
        out["evaluations"].append(r["evaluations"])
        out["cost"].append(r["cost"])
        out["num_obstacles"].append(obs.shape[0])
        print(f"{names[i]}: O={obs.shape[0]} feasible={r['feasible']} status={r['status']} it={r['iterations']} "
              f"({time.time() - t0:.0f} s)", flush=True)
    np.savez_compressed(OUT, names=names, rows=rows, T=np.int64(T), **{k: np.array(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
