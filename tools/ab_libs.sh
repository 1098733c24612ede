#!/bin/bash
# Same-box A/B/...: bench each library in $LIBS (paths; "tree" = the in-tree build) in turn,
# ROUNDS interleaved rounds (default 2), $BENCH_ARGS each; prints value and phases per run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  n=0
  for lib in $LIBS; do
    n=$((n + 1))
    log=gpurun_out/abl_${n}_$i.log
    if [ "$lib" = tree ]; then
      timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > $log 2>&1 || exit 1
    else
      DFX_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > $log 2>&1 || exit 1
    fi
    python3 - "$log" "$lib" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(j["value"] / 1e6, 2), "M", j.get("phases_ms_per_step"), "cold", j.get("cold_epoch_ms_per_step"))
PY
  done
done
