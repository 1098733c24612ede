#!/bin/bash
# round 6: the other configs on the tree at 8be763c against build/ab (276bc7a: separate
# finalize), ABBA x 1 each (C2, C5, C4 shard, B = 10^4), then the sharded step at N = 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=r6l_c2 ROUNDS=1 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6l_c5 ROUNDS=1 BENCH_ARGS="--config c5 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6l_c4 ROUNDS=1 BENCH_ARGS="--config c4shard --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6l_b1e4 ROUNDS=1 BENCH_ARGS="--batch 10000 --steps 300 --warmup 30" bash tools/abba.sh || exit 1
mkdir -p gpurun_out/r6l
timeout -k 10 400 python3 bench.py --no-cpu-baseline --sharded --steps 40 --warmup 5 > gpurun_out/r6l/sharded.log 2>&1 || exit 1
python3 - gpurun_out/r6l/sharded.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("sharded", round(d["value"] / 1e6, 2), d["phases_ms_per_step_rank0"], {k: round(v["value"] / 1e6, 2) for k, v in d["collectives"].items()})
PY
