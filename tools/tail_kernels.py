"""Per-kernel time of the solver's iterations with a given number of running worlds, from a
rocprofv3 --kernel-trace CSV of tools/nlp_trace.py (development tool; iterations start at each
ipm_rows_A / ipm_rows_DA launch, as tools/iter_profile.py). Concurrent kernels (the restoration
phase's second stream) count in their own rows, so the rows may sum past the iteration's span.
usage: tail_kernels.py <kernel_trace.csv> <min worlds> <max worlds>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "reach_kernel" in r["Kernel_Name"]]
R = rows[idx[-1] + 1:]
its = [i for i, r in enumerate(R) if "ipm_rows_A" in r["Kernel_Name"] or "ipm_rows_DA" in r["Kernel_Name"]]
lo, hi = int(sys.argv[2]), int(sys.argv[3])
agg = collections.defaultdict(lambda: [0, 0.0])
n = span = 0
for a, b in zip(its[:-1], its[1:]):
    seg = R[a:b]
    if not lo <= int(seg[0]["Grid_Size_Y"]) <= hi:
        continue
    n += 1
    span += int(R[b]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])
    for r in seg:
        k = r["Kernel_Name"].split("(")[0].replace("armour::", "")[:40]
        agg[k][0] += 1
        agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print(f"{n} iterations with {lo}-{hi} worlds running, {span / max(n, 1) / 1e3:.1f} us per iteration")
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:42s} {c / n:5.2f}/it {t / c / 1e3:7.1f} us avg {t / n / 1e3:7.1f} us/it")
