# Cache behaviour of the bundle reach kernel (development tool): L2 hit rate (TCC_HIT / TCC_MISS)
# and the L1-to-L2 request counts, one PMC pass each, over tools/reach_only.py (327 survey worlds,
# two launches). Outputs under gpurun_out/cache/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cache
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/l2 -o run -- python3 $R/tools/reach_only.py 327 > $O/l2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --output-format csv -d $O/l1 -o run -- python3 $R/tools/reach_only.py 327 > $O/l1.log 2>&1
rc=$?
cd $R && python3 - <<'PY'
import csv, glob, collections
for tag in ("l2", "l1"):
    for f in glob.glob(f"gpurun_out/cache/{tag}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for row in csv.DictReader(open(f)):
            if "lane_reach" in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
        print(tag, {k: [f"{x:.4g}" for x in v] for k, v in acc.items()})
PY
exit $rc
