set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 -m pytest tests/test_gpu_wave.py -x -q > gpurun_out/wave.log 2>&1
echo rc=$?
