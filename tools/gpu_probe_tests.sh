set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/workload_probe.py > gpurun_out/workload2.log 2>&1 || exit 1
cat gpurun_out/workload2.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; exit $rc
