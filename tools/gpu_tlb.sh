# address-translation counters of the reach kernel (development tool): one PMC pass
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tlb
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $R/gpurun_out/tlb/list.txt 2>&1 || true
grep -o "TCP_UTCL1[A-Z_]*\|TCP_TCP_LATENCY[A-Z_]*\|TCP_TA_[A-Z_]*STALL[A-Z_]*\|TCP_PENDING[A-Z_]*" $R/gpurun_out/tlb/list.txt | sort -u | head -30
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $R/gpurun_out/tlb/p1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/tlb/p1.log 2>&1 || { echo "pmc failed"; tail -3 $R/gpurun_out/tlb/p1.log; exit 0; }
python3 - $R/gpurun_out/tlb/p1/run_counter_collection.csv <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'lane_reach' in r.get('Kernel_Name', ''):
        tot[r['Counter_Name']] += float(r['Counter_Value'])
print(dict(tot))
PY
