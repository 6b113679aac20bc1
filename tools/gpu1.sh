set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick.log 2>&1 && \
ARMOUR_PROFILE_OPS=1 timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick_prof.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
echo rc=$?
