# concurrent planners: reach CU reserve x solver stream priority (plans/s of the default bench workload)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # planners reserve priority
  ARMOUR_REACH_CU_RESERVE=$2 ARMOUR_SOLVER_PRIORITY=$3 timeout -k 10 300 python3 bench.py --planners $1 --cpu-seconds 0 --no-extras --steps 5 > gpurun_out/ov.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ov.log').read().strip().splitlines()[-1]); print('planners $1 reserve $2 prio $3:', round(d['value']), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['breakdown_ms'].items()})"
}
run 2 0 0; run 2 0 1; run 2 16 0; run 2 16 1; run 2 32 1; run 2 64 1; run 3 16 1; run 3 32 1
