set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
for s in 0 1 2 3; do ARMOUR_EVAL_SKIP=$s timeout -k 10 120 python3 tools/eval_time.py 256 || exit 1; done > gpurun_out/eval_time.log 2>&1
echo rc=$?
