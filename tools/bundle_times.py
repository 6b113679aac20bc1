"""Bundle-engine load balance (development tool): every bundle's start / end wall clock (100 MHz,
ARMOUR_PROFILE_OPS=3) of one reach launch; prints the duration distribution against the kernel time.
usage: python3 tools/bundle_times.py [worlds] [profile]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
os.environ['ARMOUR_PROFILE_OPS'] = '3'
import armour_amd as A  # noqa: E402

T, O = 100, 20
W = int(sys.argv[1]) if len(sys.argv) > 1 else A.default_batch(T)
prof = sys.argv[2] if len(sys.argv) > 2 else 'survey'
P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
ws = [A.make_world(s, O, profile=prof) for s in range(W)]
P.reach(ws)
tm = P.reach(ws)
n = A.lib().armour_get_reach_profile(P.h, None, 0)
nb = (W * T + 63) // 64
cap = n + 8 + 4 * 17 + nb
buf = (ctypes.c_ulonglong * (2 * cap))()
A.lib().armour_get_reach_profile(P.h, buf, cap)
bt = np.array(buf[2 * n + 16 + 8 * 17:2 * n + 16 + 8 * 17 + 2 * nb], dtype=np.int64).reshape(nb, 2)
dur = (bt[:, 1] - bt[:, 0]) / 100.0  # us at 100 MHz
span = (bt[:, 1].max() - bt[:, 0].min()) / 100.0
print(f"W={W} bundles={nb} reach_kernel_ms={tm['reach_kernel_ms']:.2f} span_ms={span / 1e3:.2f}")
print(f"bundle ms: mean {dur.mean() / 1e3:.2f} min {dur.min() / 1e3:.2f} p10 {np.percentile(dur, 10) / 1e3:.2f} "
      f"p50 {np.median(dur) / 1e3:.2f} p90 {np.percentile(dur, 90) / 1e3:.2f} max {dur.max() / 1e3:.2f}")
wl = np.array([dur[b] for b in range(nb)])
per_world = [wl[(w * T) // 64:((w + 1) * T - 1) // 64 + 1].max() for w in range(W)]
order = np.argsort(-dur)[:10]
print("slowest bundles:", [(int(b), round(dur[b] / 1e3, 2)) for b in order])
start = (bt[:, 0] - bt[:, 0].min()) / 1e5
print(f"start spread ms: max {start.max():.2f}")
