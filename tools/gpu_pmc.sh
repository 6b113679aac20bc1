# PMC passes (separate runs) for the reach kernel's HBM traffic, plus a kernel-trace stats run
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc/fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/pmc/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc/write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/pmc/write.log 2>&1
rc=$?
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc/fetch/run_counter_collection.csv gpurun_out/pmc/write/run_counter_collection.csv reach_kernel gpurun_out/pmc/traffic.json r01 && cat gpurun_out/pmc/traffic.json
exit $rc
