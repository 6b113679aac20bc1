# average memory latencies seen by the reach kernel (development tool): TCP->TCC read latency and
# TCC->EA (HBM) read latency, one PMC pass each
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/lat
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $R/gpurun_out/lat/list.txt 2>&1 || true
grep -o "TCP_TCC_READ_REQ_LATENCY[A-Z_]*\|TCP_TCC_READ_REQ[A-Z_]*\|TCC_EA0_RDREQ_LEVEL[A-Z_]*\|TCC_EA0_RDREQ[A-Z_0-9]*\|TCP_TCR_TCP_STALL[A-Z_]*\|TCP_READ_TAGCONFLICT_STALL[A-Z_]*" $R/gpurun_out/lat/list.txt | sort -u | head -20
i=0
for set in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/lat/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/lat/p$i.log 2>&1 || { echo "pass $i failed"; tail -2 $R/gpurun_out/lat/p$i.log; continue; }
  python3 - $R/gpurun_out/lat/p$i/run_counter_collection.csv <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'lane_reach' in r.get('Kernel_Name', ''):
        tot[r['Counter_Name']] += float(r['Counter_Value'])
print(dict(tot))
PY
done
