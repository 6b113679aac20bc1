"""A/B reach-kernel timing of two library builds in one process pair (development tool).
usage: python tools/reach_ab.py <lib_a> <lib_b> [W]"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys
sys.path.insert(0, os.path.join(%r, 'armour-dev_amd'))
import armour_amd as A
W = %d
P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
ws = [A.make_world(100 + s, 20) for s in range(W)]
P.reach(ws)
ts = [P.reach(ws)["reach_kernel_ms"] for _ in range(3)]
print(os.environ["ARMOUR_LIB"].split("/")[-1], " ".join(f"{t:.2f}" for t in ts), flush=True)
'''
W = int(sys.argv[3]) if len(sys.argv) > 3 else 256
for rep in range(2):
    for lib in sys.argv[1:3]:
        env = dict(os.environ, ARMOUR_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, "-c", code % (ROOT, W)], env=env, check=True, timeout=300)
