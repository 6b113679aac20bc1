# GPU suite with the in-tree library, then a same-box A/B against a variant build (development tool)
# usage: bash tools/gpu_suite_ab.sh <variant .so in armour-dev_amd/armour_amd/> "<kernel regex>"
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1 || { tail -30 gpurun_out/suite.log; exit 1; }
tail -1 gpurun_out/suite.log
bash tools/lib_ab.sh "$1" "$2" > gpurun_out/suite_ab.log 2>&1
