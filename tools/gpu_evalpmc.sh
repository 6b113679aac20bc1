# eval_kernel PMC passes (separate runs)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ep
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_VALU_FMA_F64" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/ep/p$i -o run -- python3 $R/tools/eval_time.py 256 > $R/gpurun_out/ep/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/ep/p$i.log; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob('gpurun_out/ep/p*/run_counter_collection.csv'):
    seen = set()
    for r in csv.DictReader(open(f)):
        if 'eval_kernel' in r.get('Kernel_Name', ''):
            tot[r['Counter_Name']] += float(r['Counter_Value'])
            seen.add(r.get('Dispatch_Id'))
    for k in list(tot):
        pass
    print(f, 'dispatches', len(seen))
for k, v in sorted(tot.items()): print(f'{k:28s} {v:.4g}')
PY
