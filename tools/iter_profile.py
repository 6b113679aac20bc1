"""Per-iteration time of the traced plan of tools/nlp_trace.py (rocprofv3 --kernel-trace CSV): the
iterations start at each ipm_rows_A / ipm_rows_DA launch; prints worlds running, wall span and eval share per
iteration bucket. Development tool. usage: iter_profile.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "reach_kernel" in r["Kernel_Name"]]
R = rows[idx[-1] + 1:]
its = [i for i, r in enumerate(R) if "ipm_rows_A" in r["Kernel_Name"] or "ipm_rows_DA" in r["Kernel_Name"]]
its.append(len(R))
out = []
for a, b in zip(its[:-1], its[1:]):
    seg = R[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(R[b]["Start_Timestamp"]) if b < len(R) else int(seg[-1]["End_Timestamp"])
    ev = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg if "eval_kernel" in r["Kernel_Name"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    out.append((int(seg[0]["Grid_Size_Y"]), (t1 - t0) / 1e3, ev / 1e3, busy / 1e3, len(seg)))
buckets = [(200, 10**9), (65, 199), (17, 64), (5, 16), (1, 4)]
tot = sum(o[1] for o in out)
print(f"iterations {len(out)}, solver span {tot / 1e3:.2f} ms")
for lo, hi in buckets:
    s = [o for o in out if lo <= o[0] <= hi]
    if not s:
        continue
    span = sum(o[1] for o in s)
    print(f"  worlds {lo:3d}-{hi if hi < 10**9 else 'max':>3}: {len(s):3d} iterations, {span / 1e3:6.2f} ms "
          f"({100 * span / tot:4.1f} %), per iteration {span / len(s):7.1f} us, eval {sum(o[2] for o in s) / len(s):7.1f} us, "
          f"kernels {sum(o[4] for o in s) / len(s):4.1f}, busy {sum(o[3] for o in s) / len(s):7.1f} us")
