set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python3 tools/reach_time.py 256 > gpurun_out/reach_time.log 2>&1 && \
ARMOUR_PROFILE_OPS=2 timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick_phase.log 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/bench.log 2>&1
echo rc=$?
