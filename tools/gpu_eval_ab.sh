# eval_kernel duration and VALU/LDS instruction counts of two library builds (development tool)
# usage: bash tools/gpu_eval_ab.sh <lib_a> <lib_b>
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/evalab
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  export ARMOUR_LIB=$R/$lib
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/evalab/t$i -o run -- python3 $R/tools/eval_time.py 256 > $R/gpurun_out/evalab/t$i.log 2>&1 || exit 1
  echo "$lib $(grep eval_kernel $R/gpurun_out/evalab/t$i/run_kernel_stats.csv | cut -d, -f2-5)"
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/evalab/p$i -o run -- python3 $R/tools/eval_time.py 256 > $R/gpurun_out/evalab/p$i.log 2>&1 || exit 1
  python3 - $R/gpurun_out/evalab/p$i/run_counter_collection.csv <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'eval_kernel' in r.get('Kernel_Name', ''):
        tot[r['Counter_Name']] += float(r['Counter_Value'])
w = tot['SQ_WAVES']
print('  per wave:', ' '.join(f"{k[3:]}={v / w:.0f}" for k, v in sorted(tot.items()) if k != 'SQ_WAVES'))
PY
done
