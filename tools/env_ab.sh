#!/bin/bash
# Same-box A/B of a runtime switch: bench with $AB_ENV unset (A) and set (B), alternating.
#   AB_ENV="DFX_XVP_ROW=1" bash tools/env_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/eab_A$i.log 2>&1 || exit 1
  timeout -k 10 200 env $AB_ENV python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/eab_B$i.log 2>&1 || exit 1
done
for f in gpurun_out/eab_A*.log gpurun_out/eab_B*.log; do
  echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"launch_ms": [0-9.]*' $f | head -1) $(grep -o '"forward": [0-9.]*' $f | head -1)"
done
