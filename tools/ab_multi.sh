#!/bin/bash
# Same-box multi-library A/B (bisection): each VARIANT is name|libpath|ctx-kwargs
# (libpath empty = in-tree library). Variants alternate, ROUNDS times, so box variance
# does not decide a comparison. Prints one summary line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
IFS=';' read -ra VS <<< "$VARIANTS"
logs=()
for i in $(seq 1 $ROUNDS); do
  for v in "${VS[@]}"; do
    IFS='|' read -r name lib ctx <<< "$v"
    log=gpurun_out/abm_${name}_$i.log
    if [ -n "$lib" ]; then
      DFX_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --ctx "$ctx" $BENCH_ARGS > $log 2>&1 || exit 1
    else
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --ctx "$ctx" $BENCH_ARGS > $log 2>&1 || exit 1
    fi
    logs+=($log)
  done
done
python3 tools/ab_summary.py "${logs[@]}"
