# NLP time vs the IPM row-pass chunk (ARMOUR_ROW_CHUNK), bench defaults (development tool)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in 2048 1024 512 256; do
  ARMOUR_ROW_CHUNK=$c timeout -k 10 200 python3 bench.py --cpu-seconds 0 --steps 3 > gpurun_out/chunk.log 2>&1 || exit 1
  echo "chunk $c $(grep -o '"value": [0-9.]*' gpurun_out/chunk.log) $(grep -o 'breakdown_ms[^}]*' gpurun_out/chunk.log)"
done
