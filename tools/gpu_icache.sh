# instruction-fetch behaviour of the reach kernel (separate --pmc passes)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ic
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/ic/p$i -o run -- python3 $R/tools/reach_time.py 256 > $R/gpurun_out/ic/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/ic/p$i.log; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in glob.glob('gpurun_out/ic/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'lane_reach' in r.get('Kernel_Name', ''):
            tot[r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(tot.items()): print(f'{k:32s} {v:.4g}')
PY
