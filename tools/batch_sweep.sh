# plans/s at several worlds-per-step batch sizes (development tool)
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 256 327 491 655; do
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 --steps 3 --batch $b > gpurun_out/sweep.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1])
print($b, round(d['value']), 'plans/s', round(d['ms_per_step'],1), 'ms/step', {k: round(v,1) for k,v in d['breakdown_ms'].items()})"
done
