"""Generate the golden fixtures in tests/golden/ (run from the repo root in the build container).

    python tests/golden/make_golden.py [--ref /root/reference]

The reference ships no golden vectors for this path; it cannot be compiled or
imported here. So the fixtures hold (1) the reference's own INPUT data for the path — the
10-obstacle example of kinova_planner_realtime/armour_main.cu:19-34, the slice point of
PZ_tests.cu:198 and saved worlds from kinova_src/saved_worlds/random/*.csv (parsed numbers
only) — and (2) the outputs of the CPU restatement (oracle/) on those inputs: torque radius,
link generators, monomial counts, constraints and dense Jacobian at three points, feasibility
decisions and the solver's result. They pin the oracle against drift (tests/test_golden.py) and
the HIP path against the oracle (tests/test_gpu_parity.py). Parity with the reference itself is
unpinned (no reference outputs exist to compare with).
"""
from __future__ import annotations

import argparse
import glob
import json
import zlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from armour_amd.worlds import csv_world, example_world, make_world  # noqa: E402
from oracle import OraclePlanner  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SLICE_POINT = np.array([0.5, 0.6, 0.7, 0.0, -0.5, -0.6, -0.7])  # PZ_tests.cu:198 / armour_main.cu:207
CSV_SCENES = ["scene_013_001.csv", "scene_013_002.csv", "scene_037_005.csv"]


def points(seed):
    rng = np.random.default_rng(1000 + seed)
    return np.stack([np.zeros(7), SLICE_POINT, rng.uniform(-1, 1, 7)])


def record(name, world, T, full=True):
    q0, qd0, qdd0, qdes, obs = world
    P = OraclePlanner(q0, qd0, qdd0, qdes, obs, T=T, threads=8)
    P.reach()
    NJ = 7
    rec = dict(q0=q0, qd0=qd0, qdd0=qdd0, q_des=qdes, obstacles=np.asarray(obs, dtype=np.float64).reshape(-1, 12),
               T=np.int64(T), torque_radius=P.torque_radius(), link_gens=P.link_gens())
    rec["link_monomials"] = np.array([[len(P.pz(0, l * T + t)["hashes"]) for l in range(NJ)] for t in range(T)])
    rec["torque_monomials"] = np.array([[len(P.pz(1, j * T + t)["hashes"]) for j in range(7)] for t in range(T)])
    if full:
        X = points(zlib.crc32(name.encode()) % 1000)
        gs, Js, feas = [], [], []
        for x in X:
            g, J = P.eval(x)
            gs.append(g)
            Js.append(J)
            feas.append(P.feasible(g))
        rec.update(x=X, g=np.array(gs), J=np.array(Js), feasible_at_x=np.array(feas))
    r = P.plan()
    rec.update(k_opt=r["k_opt"], feasible=np.int64(r["feasible"]), iterations=np.int64(r["iterations"]),
               evaluations=np.int64(r["evaluations"]), status=np.int64(r["status"]), cost=np.float64(r["cost"]),
               g_opt=np.asarray(r["g"]))
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **rec)
    print(f"{name}: T={T} O={rec['obstacles'].shape[0]} feasible={r['feasible']} it={r['iterations']} "
          f"max link monomials={rec['link_monomials'].max()} max torque monomials={rec['torque_monomials'].max()}")
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    names = []
    names.append(record("example_T10", example_world(), 10))
    names.append(record("random0_T10_O10", make_world(0, 10), 10))
    names.append(record("random1_T10_O10", make_world(1, 10), 10))
    names.append(record("random2_T20_O0", make_world(2, 0), 20))
    scenes = sorted(glob.glob(os.path.join(a.ref, "kinova_src", "saved_worlds", "random", "*.csv")))
    for fn in scenes:
        base = os.path.basename(fn)
        if base not in CSV_SCENES:
            continue
        rows = np.genfromtxt(fn, delimiter=",")
        names.append(record("csv_" + base[:-4] + "_T10", csv_world(rows), 10))
    names.append(record("config2_random0_T100_O20", make_world(0, 20), 100, full=False))
    json.dump({"fixtures": names, "generator": "tests/golden/make_golden.py",
               "oracle": "oracle/ (CPU restatement); parity with the reference unpinned"},
              open(os.path.join(OUT, "index.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
