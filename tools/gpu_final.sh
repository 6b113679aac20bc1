# Round evidence in one call: rocprofv3 kernel stats + PMC traffic passes, the traffic record for
# this exact library (tools/pmc_traffic.py, so bench.py reports roofline.traffic), GPU tests, smoke,
# the default bench and the config-5 (Fetch) bench. Outputs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
bash tools/gpu_prof.sh > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/prof/fetch/run_counter_collection.csv gpurun_out/prof/write/run_counter_collection.csv \
    lane_reach_kernel profiles/r01_reach_traffic.json r01 327 > /dev/null && cp profiles/r01_reach_traffic.json gpurun_out/r01_reach_traffic.json || exit 1
bash tools/gpu_round.sh || exit 1
timeout -k 10 600 python3 bench.py --robot fetch --batch 256 > gpurun_out/bench_fetch.log 2>&1 || exit 1
tail -1 gpurun_out/bench_fetch.log
