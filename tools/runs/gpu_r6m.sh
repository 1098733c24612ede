#!/bin/bash
# round 6: the split step at N = 1 with every exchange through RCCL (--force-collectives: the
# N > 1 code path), rows in 1 slice (default) against 2 slices, interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6m
for i in 1 2; do
  for s in 0 2; do
    timeout -k 10 400 python3 bench.py --no-cpu-baseline --sharded --force-collectives --slices $s --steps 40 --warmup 5 > gpurun_out/r6m/fc_s${s}_$i.log 2>&1 || exit 1
    python3 - gpurun_out/r6m/fc_s${s}_$i.log fc_s${s}_$i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"] / 1e6, 2), d["phases_ms_per_step_rank0"], {k: round(v["value"] / 1e6, 2) for k, v in d["collectives"].items()})
PY
  done
done
