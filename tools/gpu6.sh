set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 -m pytest tests/test_gpu_wave.py -x -q > gpurun_out/wave.log 2>&1 && \
timeout -k 10 200 python3 tools/dump_ops.py gpu > gpurun_out/dump.log 2>&1 && \
timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick.log 2>&1 && \
ARMOUR_PROFILE_OPS=2 timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick_phase.log 2>&1 && \
ARMOUR_PROFILE_OPS=1 timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick_prof.log 2>&1
echo rc=$?
