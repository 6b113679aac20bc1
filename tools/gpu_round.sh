# round evidence: GPU tests, smoke, bench (stdout JSON line) into gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log gpurun_out/bench.log | tail -3
echo rc=$rc
exit $rc
