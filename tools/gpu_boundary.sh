# decision-boundary and capacity GPU tests (round 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_boundary.py -v -s --timeout 600 --timeout-method thread > gpurun_out/pytest_b.log 2>&1
rc=$?; tail -40 gpurun_out/pytest_b.log; exit $rc
