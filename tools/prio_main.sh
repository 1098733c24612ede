#!/bin/bash
# compute-stream priority A/B (bench --main-prio), alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in 1 2; do for p in normal high; do for sh in "" "--sharded"; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --main-prio $p $sh > gpurun_out/pm.log 2>&1 || { tail -5 gpurun_out/pm.log; exit 1; }
  echo "prio=$p $sh $(grep -o '"value": [0-9.]*' gpurun_out/pm.log)"
done; done; done
