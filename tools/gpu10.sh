set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/dump_ops.py gpu > gpurun_out/dump.log 2>&1 && \
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick.log 2>&1
echo rc=$?
