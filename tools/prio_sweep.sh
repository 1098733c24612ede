#!/bin/bash
# side-lane stream priorities (DFX_LOC_PRIO / DFX_AUX_PRIO: 0 low, 1 high, 2 normal) on a bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for cfg in ${PRIO_CFGS:-"1,1" "2,2" "2,1" "1,2" "0,0" "1,1"}; do
  IFS=, read lp ap <<< "$cfg"
  DFX_LOC_PRIO=$lp DFX_AUX_PRIO=$ap timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/prio.log 2>&1 || exit 1
  echo "loc=$lp aux=$ap $(grep -o '"value": [0-9.]*' gpurun_out/prio.log) $(grep -o '"initv": [0-9.]*\|"eval_auc": [0-9.]*' gpurun_out/prio.log | tr '\n' ' ')"
done
