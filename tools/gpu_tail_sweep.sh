# Sync-free tail threshold sweep (development tool): solver timeline and bench per ARMOUR_TAIL_WORLDS.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tails
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for tw in ${TAILS:-16 64 400}; do
  export ARMOUR_TAIL_WORLDS=$tw
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tw$tw -o run -- python3 $R/tools/nlp_trace.py survey 327 > $O/tw$tw.log 2>&1 || exit 1
  echo "== tail $tw: $(python3 $R/tools/iter_profile.py $O/tw$tw/run_kernel_trace.csv | sed -n 1,1p)"
  timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-extras > $O/bench_tw$tw.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_tw$tw.json').read().strip().splitlines()[-1]); print('   bench', round(d['value'],1))"
done
done
