# A/B of two library builds on one box (development tool): one planner's solver timeline (327
# survey worlds) with the in-tree library and with a variant next to it, twice each.
# usage: bash tools/lib_ab.sh <variant .so in armour-dev_amd/armour_amd/> "<kernel regex>"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for L in libarmour_hip.so $1; do
  export ARMOUR_LIB=$R/armour-dev_amd/armour_amd/$L
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$L -o run -- python3 $R/tools/nlp_trace.py survey 327 > $O/$L.log 2>&1 || exit 1
  echo "== $L"
  python3 $R/tools/iter_profile.py $O/$L/run_kernel_trace.csv > $O/$L.iter && sed -n 1,1p $O/$L.iter
  python3 $R/tools/trace_summary.py $O/$L/run_kernel_trace.csv > $O/$L.sum && grep -E "$2" $O/$L.sum
done
done
