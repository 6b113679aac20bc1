"""fp32 tolerance study (BASELINE config 5): the constraint evaluation (slicing + collision rows,
eval_kernel_t<float>, ARMOUR_EVAL_F32=1) in float against the fp64 product path, on the same fp64
reach sets. Reports per row family the largest |g32 - g64| and |J32 - J64|, collision decisions at the
reference's violation threshold that flip, and what the solver makes of it (feasibility, k_opt,
iterations). Development tool; needs a GPU.
usage: python tools/fp32_study.py [worlds] [out.json]"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COL_THR = 1e-4   # COLLISION_AVOIDANCE_CONSTRAINT_VIOLATION_THRESHOLD (Parameters.h:38)
T, O = 100, 20

child = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(%r, 'armour-dev_amd'))
import armour_amd as A
from armour_amd import robot_tables as RT
robot_name, W, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
robot = RT.load_json(os.path.join(%r, 'tests', 'golden', 'robot_fetch.json')) if robot_name == 'fetch' else None
geo = RT.geometry(robot) if robot is not None else A.KINOVA
worlds = [A.make_world(2000 + s, %d, robot=geo) for s in range(W)]
P = A.Planner(T=%d, max_obstacles=%d, max_worlds=W, robot=robot)
P.reach(worlds)
rng = np.random.default_rng(7)
xs = [np.zeros(7), np.full(7, 0.5), rng.uniform(-1, 1, 7), rng.uniform(-1, 1, 7)]
g = np.stack([np.stack([P.eval_constraints(w, x)[0] for w in range(W)]) for x in xs])
J = np.stack([np.stack([P.eval_constraints(w, x)[1] for w in range(W)]) for x in xs])
res, _ = P.plan(worlds)
np.savez(out, g=g, J=J, k=np.array([r["k_opt"] for r in res]), feas=np.array([r["feasible"] for r in res]),
         it=np.array([r["iterations"] for r in res]), status=np.array([r["status"] for r in res]))
'''


def run(robot, W, f32):
    out = f"/tmp/fp32_study_{robot}_{int(f32)}.npz"
    env = dict(os.environ)
    env.pop("ARMOUR_EVAL_F32", None)
    if f32:
        env["ARMOUR_EVAL_F32"] = "1"
    subprocess.run([sys.executable, "-c", child % (ROOT, ROOT, O, T, O), robot, str(W), out], env=env, check=True,
                   timeout=600)
    return np.load(out)


def study(robot, W):
    a, b = run(robot, W, False), run(robot, W, True)
    nt, nc = 7 * T, T * (8 if robot == "fetch" else 7) * O
    fam = {"torque": slice(0, nt), "collision": slice(nt, nt + nc), "extrema": slice(nt + nc, None)}
    rep = {"robot": robot, "worlds": W, "T": T, "O": O, "points": int(a["g"].shape[0])}
    for name, sl in fam.items():
        dg = np.abs(b["g"][:, :, sl] - a["g"][:, :, sl])
        dJ = np.abs(b["J"][:, :, sl] - a["J"][:, :, sl])
        rep[f"{name}_max_abs_dg"] = float(dg.max())
        rep[f"{name}_max_abs_dJ"] = float(dJ.max())
    cg64, cg32 = a["g"][:, :, fam["collision"]], b["g"][:, :, fam["collision"]]
    dcg = np.abs(cg32 - cg64)
    rep["collision_dg_p50"] = float(np.percentile(dcg, 50))
    rep["collision_dg_p99_9"] = float(np.percentile(dcg, 99.9))
    rep["collision_rows_dg_over_1e-6"] = int(np.sum(dcg > 1e-6))
    rep["collision_rows_dg_over_1e-3"] = int(np.sum(dcg > 1e-3))
    # g <= 0 is clearance: fp32 below fp64 claims more clearance than there is (unsafe direction)
    rep["collision_rows_fp32_less_conservative_over_1e-3"] = int(np.sum(cg32 < cg64 - 1e-3))
    rep["collision_rows_fp32_more_conservative_over_1e-3"] = int(np.sum(cg32 > cg64 + 1e-3))
    big = np.argwhere(dcg > 1e-3)[:5]
    rep["collision_largest_dg_rows"] = [dict(point=int(i), world=int(w), row=int(r), g64=float(cg64[i, w, r]),
                                             g32=float(cg32[i, w, r])) for i, w, r in big]
    rep["collision_rows"] = int(cg64.size)
    rep["collision_decision_flips"] = int(np.sum((cg64 > COL_THR) != (cg32 > COL_THR)))
    rep["collision_rows_within_1e-4_of_threshold"] = int(np.sum(np.abs(cg64 - COL_THR) < 1e-4))
    rep["plans_feasibility_differs"] = int(np.sum(a["feas"] != b["feas"]))
    rep["plans_status_differs"] = int(np.sum(a["status"] != b["status"]))
    rep["plans_iterations_differ"] = int(np.sum(a["it"] != b["it"]))
    dk = np.abs(b["k"] - a["k"]).max(axis=1)
    rep["k_opt_max_abs_diff"] = float(dk.max())
    rep["k_opt_median_abs_diff"] = float(np.median(dk))
    rep["feasible_fp64"] = int(a["feas"].sum())
    rep["feasible_fp32"] = int(b["feas"].sum())
    return rep


if __name__ == "__main__":
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = [study("fetch", W), study("kinova", W)]
    for r in reps:
        print(json.dumps(r))
    if len(sys.argv) > 2:
        json.dump({"study": "constraint evaluation (slicing + collision) in fp32 on fp64 reach sets, "
                            "against the fp64 path; eval_kernel_t<float> via ARMOUR_EVAL_F32=1",
                   "command": "python tools/fp32_study.py " + " ".join(sys.argv[1:]), "results": reps},
                  open(sys.argv[2], "w"), indent=1)
