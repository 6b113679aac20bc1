# plans/s of the default bench workload by concurrent planners per GPU (no extras)
set -o pipefail
cd $GRAFT_REPO_ROOT
for P in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --planners $P --cpu-seconds 0 --no-extras --steps 5 > gpurun_out/sweep_p$P.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_p$P.log').read().strip().splitlines()[-1]); print($P, round(d['value']), round(d['ms_per_step'],1), d['breakdown_ms'])"
done
