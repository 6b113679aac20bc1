# Sync-free solver tail A/B (development tool): GPU suite with the default library, then one
# planner's solver timeline (327 survey worlds) and the bench's latency / config-4 legs with the
# sync-free tail off (ARMOUR_TAIL_WORLDS=0) and on (default), twice each. Outputs under gpurun_out/tail/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tail
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for tw in 0 16; do
  export ARMOUR_TAIL_WORLDS=$tw
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tw$tw -o run -- python3 $R/tools/nlp_trace.py survey 327 > $O/tw$tw.log 2>&1 || exit 1
  echo "== tail $tw: $(python3 $R/tools/iter_profile.py $O/tw$tw/run_kernel_trace.csv | sed -n 1,1p)"
  timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_tw$tw.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_tw$tw.json').read().strip().splitlines()[-1]); print('   bench', round(d['value'],1), 'latency', {k: round(v,2) for k,v in d['latency'].items()})"
  timeout -k 10 300 python3 $R/bench.py --total-worlds 32 --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/c4_tw$tw.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c4_tw$tw.json').read().strip().splitlines()[-1]); print('   32 worlds', round(d['ms_per_step'],2), 'ms')"
done
done
