set -o pipefail
cd $GRAFT_REPO_ROOT
L=$PWD/armour-dev_amd/armour_amd/libarmour_hip_t128w3.so
{ timeout -k 10 200 python3 tools/reach_time.py 256 && \
  for n in 4 6; do ARMOUR_LIB=$L ARMOUR_REACH_WG_PER_CU=$n timeout -k 10 200 python3 tools/reach_time.py 256 || exit 1; done ; } > gpurun_out/reach_w3.log 2>&1
echo rc=$?
