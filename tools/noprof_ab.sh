#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in 1 2; do for e in "" 1; do
  DFX_NOPROF=$e timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/np.log 2>&1 || exit 1
  echo "noprof=$e $(grep -o '"value": [0-9.]*' gpurun_out/np.log)"
done; done
