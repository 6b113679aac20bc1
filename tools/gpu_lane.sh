set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/lane_check.py > gpurun_out/lane_check.log 2>&1 && \
timeout -k 10 300 python3 -u tools/lane_prof.py > gpurun_out/lane_prof.log 2>&1
rc=$?
tail -8 gpurun_out/lane_check.log; cat gpurun_out/lane_prof.log
exit $rc
