"""Phases of the traced plan of tools/nlp_trace.py (rocprofv3 --kernel-trace CSV): the solver's
interior-point loops and restoration phases (planner.hip run_solver / run_resto) as wall-clock
segments after the last reach launch, with their kernel counts. Development tool.
usage: solver_phases.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "reach_kernel" in r["Kernel_Name"]]
R = rows[idx[-1] + 1:]


def kind(name):
    if "resto_" in name:
        return "restoration"
    if "ipm_collect" in name:
        return "collect"
    if "feasible_kernel" in name:
        return "feasible"
    if "plane_cache" in name:
        return "plane cache"
    return "interior point"


segs = []
for r in R:
    k = kind(r["Kernel_Name"])
    if k == "collect":
        continue
    # eval / trial kernels of a restoration phase belong to it
    if segs and segs[-1][0] == "restoration" and k == "interior point" and "ipm_" not in r["Kernel_Name"]:
        k = "restoration"
    if not segs or segs[-1][0] != k:
        segs.append([k, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0])
    segs[-1][2] = int(r["End_Timestamp"])
    segs[-1][3] += 1
t0 = segs[0][1]
print(f"solver span {(segs[-1][2] - t0) / 1e6:.2f} ms")
for k, a, b, n in segs:
    print(f"  {k:15s} {(a - t0) / 1e6:8.2f} .. {(b - t0) / 1e6:8.2f} ms  ({(b - a) / 1e6:7.2f} ms, {n} kernels)")
