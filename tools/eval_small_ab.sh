# small- vs full-capacity evaluation kernels (ARMOUR_EVAL_FULL=1), one planner's solver timeline on
# one box (development tool)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/esab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for f in 0 1; do
  export ARMOUR_EVAL_FULL=$f
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/f$f -o run -- python3 $R/tools/nlp_trace.py survey 327 > $O/f$f.log 2>&1 || exit 1
  echo "== full=$f"
  python3 $R/tools/iter_profile.py $O/f$f/run_kernel_trace.csv > $O/f$f.iter && sed -n 1,1p $O/f$f.iter
  python3 $R/tools/trace_summary.py $O/f$f/run_kernel_trace.csv > $O/f$f.sum && grep -E "eval|mono" $O/f$f.sum
done
done
