# Round evidence (usage: bash tools/gpu_prof_round.sh r02): rocprofv3 kernel stats of the bench
# command, FETCH_SIZE / WRITE_SIZE passes of one planner's reach launch (traffic record for this
# library build), an fp64 VALU pass on eval_kernel. Outputs under gpurun_out/prof_<round>/.
set -o pipefail
RND=${1:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$RND
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py > $O/trace.log 2>&1 || { echo trace failed; tail -5 $O/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --planners 1 --steps 1 --warmup 0 --cpu-seconds 0 --no-extras > $O/fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --planners 1 --steps 1 --warmup 0 --cpu-seconds 0 --no-extras > $O/write.log 2>&1 || { echo write failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/evalpmc -o run -- python3 $R/tools/eval_pmc.py > $O/evalpmc.log 2>&1 || { echo evalpmc failed; tail -3 $O/evalpmc.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/evaltrace -o run -- python3 $R/tools/eval_pmc.py > $O/evaltrace.log 2>&1 || { echo evaltrace failed; exit 1; }
cd $R
python3 tools/stats_summary.py $O/trace/run_kernel_stats.csv profiles/${RND}_kernel_stats.txt "rocprofv3 --kernel-trace --stats -- python3 bench.py (defaults), $RND" > /dev/null
cp $O/trace/run_kernel_stats.csv profiles/${RND}_kernel_stats.csv
grep "^{\"metric\"" $O/trace.log | tail -1 > profiles/${RND}_bench_profiled.json
python3 tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv lane_reach_kernel profiles/${RND}_reach_traffic.json $RND 327 survey > /dev/null
python3 tools/eval_valu.py $O/evalpmc/run_counter_collection.csv $O/evaltrace/run_kernel_trace.csv profiles/${RND}_eval_valu.json > /dev/null
mkdir -p gpurun_out/profiles_new && cp profiles/${RND}_* gpurun_out/profiles_new/
head -12 profiles/${RND}_kernel_stats.txt
cat profiles/${RND}_reach_traffic.json | head -8
python3 -c "import json; d=json.load(open('profiles/${RND}_eval_valu.json')); print({k: d[k] for k in ('fp64_tflops','frac_of_fp64_peak','valu_busy','median_duration_s')})"
# solver timeline of one planner (one traced plan of the bench batch): per-iteration buckets and kernel totals
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_$RND/nlp -o run -- python3 $R/tools/nlp_trace.py survey 327 > $R/gpurun_out/prof_$RND/nlp.log 2>&1 || { echo nlp trace failed; exit 1; }
cd $R
{ echo "# one planner, 327 survey worlds, T=100, O=20: rocprofv3 --kernel-trace -- python3 tools/nlp_trace.py survey 327 ($RND)"; python3 tools/iter_profile.py gpurun_out/prof_$RND/nlp/run_kernel_trace.csv; python3 tools/trace_summary.py gpurun_out/prof_$RND/nlp/run_kernel_trace.csv; } > profiles/${RND}_solver_timeline.txt
cp profiles/${RND}_solver_timeline.txt gpurun_out/profiles_new/
cat profiles/${RND}_solver_timeline.txt | head -8
