# A/B of the plan step (reach + NLP ms) of two library builds on one box (development tool)
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for lib in armour-dev_amd/armour_amd/libarmour_hip_base.so armour-dev_amd/armour_amd/libarmour_hip.so; do
  ARMOUR_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --cpu-seconds 0 --steps 3 > gpurun_out/ab.log 2>&1 || exit 1
  echo "$(basename $lib) $(grep -o 'breakdown_ms[^}]*' gpurun_out/ab.log)"
done
done
