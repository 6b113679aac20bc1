"""Diagnostics: two bundle-engine reach launches of W survey worlds (for profilers)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
os.environ.setdefault('ARMOUR_ENGINE', 'lane')
import armour_amd as A
W = int(sys.argv[1]) if len(sys.argv) > 1 else 327
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
ws = [A.make_world(s, 20, profile="survey") for s in range(W)]
for _ in range(2):
    print(P.reach(ws), flush=True)
