#!/bin/bash
# closing kwarg sweep on the final tree (C3, same box, 3 interleaved rounds): the backward's LDS
# reservation (bwd_lds, default 16384) below its default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
for i in 1 2 3; do
  for ctx in "" "bwd_lds=8192" "bwd_lds=12288" "bwd_lds=14336"; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 ${ctx:+--ctx $ctx} > gpurun_out/r5/sw_$i.log 2>&1 || exit 1
    python3 - gpurun_out/r5/sw_$i.log "${ctx:-default}" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(j["value"] / 1e6, 2), j["phases_ms_per_step"]["forward"], j["phases_ms_per_step"]["backward_update"])
PY
  done
done
