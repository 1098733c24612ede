#!/bin/bash
# Same-box A/B over bench ARGUMENTS (not library builds): each VARIANT is name|bench-args;
# variants alternate ROUNDS times so box variance does not decide a comparison.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
IFS=';' read -ra VS <<< "$VARIANTS"
logs=()
for i in $(seq 1 $ROUNDS); do
  for v in "${VS[@]}"; do
    IFS='|' read -r name args <<< "$v"
    log=gpurun_out/aba_${name}_$i.log
    timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > $log 2>&1 || exit 1
    logs+=($log)
  done
done
python3 tools/ab_summary.py "${logs[@]}"
