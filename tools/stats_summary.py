"""Summarise a rocprofv3 --kernel-trace --stats run (run_kernel_stats.csv) as a fixed-width table.
usage: python tools/stats_summary.py <run_kernel_stats.csv> <out.txt> <header line>..."""
import csv
import sys

src, dst = sys.argv[1:3]
rows = list(csv.DictReader(open(src)))
with open(dst, "w") as f:
    for h in sys.argv[3:]:
        f.write(f"# {h}\n")
    f.write(f"{'Name':72s} {'Calls':>6s} {'TotalDurationNs':>16s} {'AverageNs':>14s} {'MinNs':>12s} {'MaxNs':>12s} {'Percentage':>10s}\n")
    for r in rows:
        f.write(f"{r['Name'][:72]:72s} {int(r['Calls']):6d} {int(float(r['TotalDurationNs'])):16d} {float(r['AverageNs']):14.1f} "
                f"{int(float(r['MinNs'])):12d} {int(float(r['MaxNs'])):12d} {float(r['Percentage']):10.2f}\n")
