import os, sys
ROOT = '/root/repo' if os.path.exists('/root/repo') else os.environ['GRAFT_REPO_ROOT']
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', ROOT), 'armour-dev_amd'))
import armour_amd as A
T, O, W = 200, 40, 163
P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
worlds = [A.make_world(s, O, profile="survey") for s in range(W)]
P.plan(worlds)
res, tm = P.plan(worlds)
print(tm, flush=True)
