"""Diagnostics: reach kernel time at W worlds (bench workload T=100, O=20)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
import armour_amd as A
W = int(sys.argv[1]) if len(sys.argv) > 1 else 256
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
worlds = [A.make_world(s, 20) for s in range(W)]
P.reach(worlds)
ts = []
for _ in range(3):
    tm = P.reach(worlds)
    ts.append(tm['reach_kernel_ms'])
print(f"wg/cu={os.environ.get('ARMOUR_REACH_WG_PER_CU', '4')} W={W}: reach kernel {min(ts):.2f} ms")
