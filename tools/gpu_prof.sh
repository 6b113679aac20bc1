# rocprofv3: kernel trace + stats (csv) and two PMC passes for the reach kernel's traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/trace -o run -- python3 $R/bench.py > $R/gpurun_out/prof/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/prof/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/prof/write.log 2>&1
rc=$?
find $R/gpurun_out/prof -name "*.csv" | head -20
echo rc=$rc
exit $rc
