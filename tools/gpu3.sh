set -o pipefail
cd $GRAFT_REPO_ROOT
for m in 3 1 2 0; do
  echo "== mode $m"
  ARMOUR_ENGINE_MODE=$m timeout -k 10 200 python3 tools/gpu_quick.py 2>&1 | head -4 || exit 1
done > gpurun_out/modes.log 2>&1
echo rc=$?
