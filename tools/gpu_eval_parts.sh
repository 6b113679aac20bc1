# eval_kernel per-part duration and per-wave instruction counts (ARMOUR_EVAL_SKIP bit 0: slicing,
# bit 1: collision) of one build (development tool). usage: bash tools/gpu_eval_parts.sh [lib]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/evalparts
cd /tmp && export TMPDIR=/tmp
[ -n "$1" ] && export ARMOUR_LIB=$R/$1
for k in 0 1 2 3; do
  export ARMOUR_EVAL_SKIP=$k
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/evalparts/t$k -o run -- python3 $R/tools/eval_time.py 256 > $R/gpurun_out/evalparts/t$k.log 2>&1 || exit 1
  echo "skip=$k $(grep eval_kernel $R/gpurun_out/evalparts/t$k/run_kernel_stats.csv | cut -d, -f2-5)"
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $R/gpurun_out/evalparts/p$k -o run -- python3 $R/tools/eval_time.py 256 > $R/gpurun_out/evalparts/p$k.log 2>&1 || exit 1
  python3 - $R/gpurun_out/evalparts/p$k/run_counter_collection.csv <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'eval_kernel' in r.get('Kernel_Name', ''):
        tot[r['Counter_Name']] += float(r['Counter_Value'])
w = tot['SQ_WAVES']
print('  per wave:', ' '.join(f"{k[3:]}={v / w:.0f}" for k, v in sorted(tot.items()) if k != 'SQ_WAVES'))
PY
done
