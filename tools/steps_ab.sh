#!/bin/bash
# bench at the default K and at longer timed windows, alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in 1 2; do for k in 20 100; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $k --warmup 10 $BENCH_ARGS > gpurun_out/steps.log 2>&1 || exit 1
  echo "steps=$k $(grep -o '"value": [0-9.]*\|"launch_ms": [0-9.]*' gpurun_out/steps.log | tr '\n' ' ')"
done; done
