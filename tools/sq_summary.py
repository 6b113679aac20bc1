"""Per-kernel SQ counter summary of rocprofv3 --pmc passes (counter_collection CSVs, one pass each):
for every kernel, launches and each counter's mean per wave (SQ_WAVES of the same pass), plus
SQ_WAIT_ANY / SQ_WAVE_CYCLES as a percentage when both are there. Diagnostics.

usage: python tools/sq_summary.py <out.txt> <title> <counter_collection.csv> [...]"""
import csv
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("armour::", "")
            key = (k, row.get("Dispatch_Id") or row.get("Correlation_Id"))
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    return per


out, title, paths = sys.argv[1], sys.argv[2], sys.argv[3:]
kern = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-wave values
launches = defaultdict(int)
for p in paths:
    for (k, _), cs in load(p).items():
        if p == paths[0]:
            launches[k] += 1
        waves = cs.get("SQ_WAVES", 0.0)
        for c, v in cs.items():
            if c == "SQ_WAVES":
                kern[k][c].append(v)
            elif waves > 0:
                kern[k][c].append(v / waves)
lines = [f"# {title}", "# per kernel: launches, mean per wave of each counter (SQ_WAVES: per launch)"]
order = sorted(kern, key=lambda k: -launches[k] * (sum(kern[k].get("SQ_WAVE_CYCLES", [0])) or 1))
for k in order:
    cs = kern[k]
    mean = {c: sum(v) / len(v) for c, v in cs.items() if v}
    parts = [f"{k[:36]:36s} launches {launches[k]:5d}"]
    for c in sorted(mean):
        parts.append(f"{c.replace('SQ_', '')} {mean[c]:.0f}")
    if "SQ_WAIT_ANY" in mean and mean.get("SQ_WAVE_CYCLES"):
        parts.append(f"wait_any% {100 * mean['SQ_WAIT_ANY'] / mean['SQ_WAVE_CYCLES']:.1f}")
    lines.append("  ".join(parts))
open(out, "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:12]))
