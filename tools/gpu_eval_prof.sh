# eval_kernel duration with its parts switched off (ARMOUR_EVAL_SKIP bit 0: slicing, bit 1: collision)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/evalprof
cd /tmp && export TMPDIR=/tmp
for k in 0 1 2 3; do
  ARMOUR_EVAL_SKIP=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/evalprof/s$k -o run -- python3 $R/tools/eval_time.py 256 > $R/gpurun_out/evalprof/s$k.log 2>&1 || exit 1
  grep eval_kernel $R/gpurun_out/evalprof/s$k/run_kernel_stats.csv | cut -d, -f1-5
done
