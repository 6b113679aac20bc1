set -o pipefail
cd $GRAFT_REPO_ROOT
{ timeout -k 10 200 python3 tools/reach_time.py 256 && \
  for n in 4 6 8; do ARMOUR_LIB=$PWD/armour-dev_amd/armour_amd/libarmour_hip_t64.so ARMOUR_REACH_WG_PER_CU=$n timeout -k 10 200 python3 tools/reach_time.py 256 || exit 1; done && \
  ARMOUR_LIB=$PWD/armour-dev_amd/armour_amd/libarmour_hip_t64.so timeout -k 10 300 python3 tools/gpu_quick.py ; } > gpurun_out/reach_conc.log 2>&1
echo rc=$?
