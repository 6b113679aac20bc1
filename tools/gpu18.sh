set -o pipefail
cd $GRAFT_REPO_ROOT
{ timeout -k 10 200 python3 tools/reach_time.py 256 && ARMOUR_ENGINE_MODE=2 timeout -k 10 200 python3 tools/reach_time.py 256 ; } > gpurun_out/reach_mode.log 2>&1
echo rc=$?
