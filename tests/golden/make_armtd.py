"""Generate the ARMTD comparison-planner fixtures tests/golden/armtd_T100_O10.npz (build container,
repo root; needs /root/reference for the offline JRS files):

    python tests/golden/make_armtd.py

Inputs follow the MATLAB caller (KSI/uarmtd_planner.m:260-318): q0 / q_des / obstacles from the
ARMOUR world generator, qd0 within the offline JRS grid, and per joint the reference's own
precomputed JRS (ACMP/offline_jrs/orig_parameterization/JRS_<c_kvi>.mat, read as data by
tests/offline_jrs.py) of the c_kvi closest to qd0_i. Half of the worlds get obstacles tuned with the
oracle onto the collision threshold at x = 0 (tests/boundary_worlds.py), one starts in collision.
Outputs are the oracle's (CPU restatement, oracle/src/armtd.cpp): collision decisions at x = 0,
near-threshold row counts, the plan. Parity with the reference itself is unpinned (no Ipopt, no
reference outputs).
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("armour-dev_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import boundary_worlds as B  # noqa: E402
import offline_jrs as J  # noqa: E402
from armour_amd.worlds import make_world  # noqa: E402
from oracle import OracleArmtd  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
T, O, N = 100, 10, 8


def main():
    rec = {k: [] for k in ("kinds", "q0", "qd0", "q_des", "tables", "k_range", "obstacles", "x0", "feasible", "status",
                           "iterations", "k_opt", "cost", "near_x0", "near_kopt", "dec_x0")}
    for s in range(N):
        rng = np.random.default_rng(20_000 + s)
        kind = ["plain", "graze", "graze", "start", "plain", "graze", "graze", "plain"][s]
        q0, _, _, q_des, obs = make_world(100 + s, O)
        qd0 = rng.uniform(-1.0, 1.0, 7) if s % 2 else rng.uniform(-0.2, 0.2, 7)
        tab, kr = J.armtd_input(qd0)
        x0 = np.zeros(7)
        R = OracleArmtd(q0, qd0, q_des, tab, kr, obs, T=T, threads=8)
        R.reach()
        _, _, lc = R.eval(x0, centers=True)
        obs = np.array(obs)
        if kind == "graze":
            for k in range(O // 2):
                obs[k] = B.tune_obstacle(R, rng, lc, x0, T, 7, B.COL_THR + rng.uniform(-3e-3, 6e-4), t_lo=0.5, nt=0)
        if kind == "start":
            obs[-1] = B.start_obstacle(B.KINOVA, q0, rng)
        R.set_obstacles(obs)
        g0 = R.eval(x0, jac=False)
        r = R.plan()
        gk = R.eval(r["k_opt"], jac=False)
        for k, v in zip(("q0", "qd0", "q_des", "tables", "k_range", "obstacles", "x0"), (q0, qd0, q_des, tab, kr, obs, x0)):
            rec[k].append(np.asarray(v, dtype=np.float64))
        rec["kinds"].append(kind)
        rec["feasible"].append(r["feasible"])
        rec["status"].append(r["status"])
        rec["iterations"].append(r["iterations"])
        rec["k_opt"].append(r["k_opt"])
        rec["cost"].append(r["cost"])
        rec["near_x0"].append(B.near_threshold_rows(g0, T, 7, O, nt=0))
        rec["near_kopt"].append(B.near_threshold_rows(gk, T, 7, O, nt=0))
        rec["dec_x0"].append(np.packbits(g0[:7 * T * O] > B.COL_THR))
        print(f"armtd {s} {kind:6s} feasible={r['feasible']!s:5} status={r['status']} it={r['iterations']:3d} "
              f"near@x0={rec['near_x0'][-1]} near@kopt={rec['near_kopt'][-1]}", flush=True)
    out = {k: np.array(v) for k, v in rec.items()}
    out["T"] = np.int64(T)
    np.savez_compressed(os.path.join(OUT, "armtd_T100_O10.npz"), **out)


if __name__ == "__main__":
    main()
