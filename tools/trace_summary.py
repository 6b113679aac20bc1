"""Summary of a rocprofv3 --kernel-trace CSV of tools/nlp_trace.py: per-kernel totals over the traced
plan (from the second reach launch), busy vs idle time, and per-iteration costs."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "reach_kernel" in r["Kernel_Name"]]
R = rows[idx[-1]:]
t0 = int(R[0]["Start_Timestamp"])
names = ["eval_kernel", "eval_trials_kernel", "ipm_world_Cs", "ipm_rows_A", "ipm_rows_DA", "ipm_rows_B",
         "ipm_rows_D", "ipm_world_A", "ipm_world_B", "ipm_world_C", "ipm_world_D", "lane_reach", "reach_kernel",
         "bounds", "feasible", "jrs", "ipm_world_init", "ipm_rows_init"]


def nm(r):
    for k in names:
        if k in r["Kernel_Name"]:
            return k
    return r["Kernel_Name"][:30]


tot = collections.defaultdict(float)
cnt = collections.Counter()
busy = 0
last_end = t0
for r in R:
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    d = (b - a) / 1e6
    tot[nm(r)] += d
    cnt[nm(r)] += 1
    busy += (b - max(a, last_end)) / 1e6 if b > last_end else 0
    last_end = max(last_end, b)
span = (last_end - t0) / 1e6
print(f"span {span:.2f} ms, GPU busy {busy:.2f} ms, idle {span - busy:.2f} ms")
for k in sorted(tot, key=lambda k: -tot[k]):
    print(f"  {k:18s} {cnt[k]:6d} {tot[k]:9.2f} ms  avg {tot[k] / cnt[k] * 1e3:8.1f} us")
