#!/bin/bash
# side-lane stream priorities (DFX_LOC_PRIO / DFX_AUX_PRIO: 0 low, 1 high, 2 normal) on a bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for cfg in "1 1" "2 2" "2 1" "1 2" "0 0" "1 1"; do
  set -- $cfg
  DFX_LOC_PRIO=$1 DFX_AUX_PRIO=$2 timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/prio.log 2>&1 || exit 1
  echo "loc=$1 aux=$2 $(grep -o '"value": [0-9.]*' gpurun_out/prio.log)"
done
