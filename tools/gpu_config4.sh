# Config 4 (SURVEY/BASELINE: 256 worlds in total, sharded over 8 GPUs) on one GPU: the whole job at
# N = 1, and each rank's share at N = 2, 4, 8 (128, 64, 32 worlds), which is what a rank plans per
# step in the strong-scaling run. Bench lines under gpurun_out/config4/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/config4
mkdir -p $O
cd $R
for n in 256 128 64 32; do
  for p in 3 1; do
    timeout -k 10 300 python3 bench.py --total-worlds $n --planners $p --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/tw${n}_p${p}.json 2> $O/tw${n}_p${p}.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/tw${n}_p${p}.json').read().strip().splitlines()[-1]); print($n, $p, round(d['value'],1), round(d['ms_per_step'],2))"
  done
done
