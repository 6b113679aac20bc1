#!/usr/bin/env bash
# One parameterised GPU-box runner (replaces the per-experiment tools/gpu_*.sh wrappers).
#
#   gpurun -- bash tools/gpu.sh 'STEP ARGS' ['STEP ARGS' ...]
#
# Steps run in order, each under its own time limit, and the first failure ends the call (no GPU
# step runs after a fault, abort or time-out). Output of step n goes to gpurun_out/<n>_<step>.*
#   pytest ARGS         python -m pytest -m gpu -x -v --timeout 300 --timeout-method thread ARGS
#   smoke               __graft_entry__.smoke()
#   bench ARGS          python bench.py ARGS (the JSON line -> gpurun_out/<n>_bench.json)
#   py SCRIPT ARGS      python -u SCRIPT ARGS
#   stats SCRIPT ARGS   rocprofv3 --kernel-trace --stats of python SCRIPT ARGS (csv under gpurun_out/<n>_stats/)
#   pmc 'CTRS' SCRIPT ARGS  one rocprofv3 --pmc pass (counters within one pass's block limits);
#                       SCRIPT may also be a built executable (tools/micro/...), run directly
#   traffic TAG BATCH   FETCH_SIZE and WRITE_SIZE passes over one bench step, then tools/pmc_traffic.py
#                       writes gpurun_out/<TAG>_reach_traffic.json for this library build
#   sweep 'ARGS' V...   bench.py ARGS once per value V, "{}" in ARGS replaced by V (planner counts,
#                       batch sizes; an env sweep: 'env ARMOUR_ROW_CHUNK={} ...' is not supported,
#                       put the variable in ARGS as --flag or use envab); one line per value
#   libab VARIANT RE    one planner's solver timeline (tools/nlp_trace.py, 327 survey worlds) under
#                       rocprofv3 with the in-tree library and with armour_amd/VARIANT, twice each,
#                       iteration profile and the kernels matching RE (same-box A/B)
#   envab NAME V0 V1 RE the same timeline A/B between two values of environment variable NAME
# Environment for a step: prefix it, e.g. 'env ARMOUR_ENGINE=job py tools/reach_time.py 32'.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  eval "set -- $step"
  envs=()
  if [ "$1" = env ]; then
    shift
    while [[ "$1" == *=* ]]; do envs+=("$1"); shift; done
  fi
  kind=$1; shift
  tag=$(printf "%02d_%s" $n "$kind")
  echo "== step $n: $step" | tee -a "$OUT/gpu_sh.log"
  case $kind in
    pytest)
      env "${envs[@]}" timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/$tag.log" 2>&1
      rc=$?; grep -E "passed|failed|error" "$OUT/$tag.log" | tail -3 ;;
    smoke)
      env "${envs[@]}" timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/$tag.log" 2>&1
      rc=$?; tail -1 "$OUT/$tag.log" ;;
    bench)
      env "${envs[@]}" timeout -k 10 900 python3 bench.py "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err"
      rc=$?; tail -c 600 "$OUT/$tag.json" ;;
    py)
      env "${envs[@]}" timeout -k 10 600 python3 -u "$@" > "$OUT/$tag.log" 2>&1
      rc=$?; tail -5 "$OUT/$tag.log" ;;
    stats)
      (cd /tmp && env "${envs[@]}" timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/$tag" -o run -- python3 "$R/$1" "${@:2}") > "$OUT/$tag.log" 2>&1
      rc=$?
      [ $rc -eq 0 ] && python3 tools/stats_summary.py "$OUT/$tag/run_kernel_stats.csv" "$OUT/$tag.txt" "$step" \
          "lib_sha1 $(python3 -c 'import hashlib; print(hashlib.sha1(open("armour-dev_amd/armour_amd/libarmour_hip.so","rb").read()).hexdigest()[:16])')" \
          && head -14 "$OUT/$tag.txt" ;;
    pmc)
      ctrs=$1; shift
      prog=(python3 "$R/$1"); [[ "$1" == *.py ]] || prog=("$R/$1")
      (cd /tmp && env "${envs[@]}" timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv \
          -d "$OUT/$tag" -o run -- "${prog[@]}" "${@:2}") > "$OUT/$tag.log" 2>&1
      rc=$? ;;
    traffic)
      ttag=$1; batch=$2
      (cd /tmp && env "${envs[@]}" timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/${tag}_fetch" -o run -- \
          python3 "$R/bench.py" --batch "$batch" --steps 1 --warmup 0 --cpu-seconds 0 --no-extras) > "$OUT/${tag}_fetch.log" 2>&1 && \
      (cd /tmp && env "${envs[@]}" timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/${tag}_write" -o run -- \
          python3 "$R/bench.py" --batch "$batch" --steps 1 --warmup 0 --cpu-seconds 0 --no-extras) > "$OUT/${tag}_write.log" 2>&1 && \
      python3 tools/pmc_traffic.py "$OUT/${tag}_fetch/run_counter_collection.csv" "$OUT/${tag}_write/run_counter_collection.csv" \
          lane_reach_kernel "$OUT/${ttag}_reach_traffic.json" "$ttag" "$batch" survey
      rc=$?; [ $rc -eq 0 ] && cat "$OUT/${ttag}_reach_traffic.json" ;;
    sweep)
      args=$1; shift; rc=0
      for v in "$@"; do
        env "${envs[@]}" timeout -k 10 600 python3 bench.py ${args//\{\}/$v} > "$OUT/${tag}_$v.json" 2> "$OUT/${tag}_$v.err" || { rc=$?; break; }
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value'], 1), round(d['ms_per_step'], 2), {k: round(v, 2) for k, v in d['breakdown_ms'].items()})" "$OUT/${tag}_$v.json" "$v"
      done ;;
    libab|envab)
      rc=0; mkdir -p "$OUT/$tag"
      if [ "$kind" = libab ]; then names=(libarmour_hip.so "$1"); re=$2; else names=("$2" "$3"); re=$4; fi
      for rep in 1 2; do
        for nm in "${names[@]}"; do
          if [ "$kind" = libab ]; then ev=(ARMOUR_LIB="$R/armour-dev_amd/armour_amd/$nm"); else ev=("$1=$nm"); fi
          (cd /tmp && env "${envs[@]}" "${ev[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
              -d "$OUT/$tag/$nm.$rep" -o run -- python3 "$R/tools/nlp_trace.py" survey 327) > "$OUT/$tag/$nm.$rep.log" 2>&1 || { rc=$?; break 2; }
          echo "== $nm (rep $rep)"
          python3 tools/iter_profile.py "$OUT/$tag/$nm.$rep/run_kernel_trace.csv" | sed -n 1,1p
          python3 tools/trace_summary.py "$OUT/$tag/$nm.$rep/run_kernel_trace.csv" | grep -E "$re"
        done
      done ;;
    *)
      echo "unknown step kind: $kind"; rc=2 ;;
  esac
  echo "== step $n rc=$rc" | tee -a "$OUT/gpu_sh.log"
  [ $rc -eq 0 ] || exit $rc
done
