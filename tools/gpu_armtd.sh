set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_armtd.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_armtd.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_armtd.log | head -30; tail -3 gpurun_out/pytest_armtd.log; exit $rc
