set -o pipefail
cd $GRAFT_REPO_ROOT
ARMOUR_PROFILE_OPS=2 timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick_phase.log 2>&1 && \
ARMOUR_PROFILE_OPS=1 timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick_prof.log 2>&1
echo rc=$?
