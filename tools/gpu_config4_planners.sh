set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/config4; mkdir -p $O; cd $R
for n in 32 64 128; do for p in 2 4 6; do
  timeout -k 10 300 python3 bench.py --total-worlds $n --planners $p --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/tw${n}_p${p}.json 2> $O/tw${n}_p${p}.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/tw${n}_p${p}.json').read().strip().splitlines()[-1]); print($n, $p, round(d['value'],1), round(d['ms_per_step'],2))"
done; done
