# eval_kernel duration of the current build (mode 0, 256 worlds; tools/eval_time.py) and the
# solver timeline of one planner (development tool). usage: bash tools/gpu_eval_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/evalab
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/evalab/t -o run -- python3 $R/tools/eval_time.py 256 > $R/gpurun_out/evalab/t.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/evalab/nlp -o run -- python3 $R/tools/nlp_trace.py survey 327 > $R/gpurun_out/evalab/nlp.log 2>&1 || exit 1
cd $R
python3 - gpurun_out/evalab/t/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'eval_kernel' in r['Name']:
        print('eval mode 0, 256 worlds: avg us', float(r['AverageNs']) / 1e3, 'min', float(r['MinNs']) / 1e3)
PY
python3 tools/iter_profile.py gpurun_out/evalab/nlp/run_kernel_trace.csv 
python3 tools/trace_summary.py gpurun_out/evalab/nlp/run_kernel_trace.csv 
