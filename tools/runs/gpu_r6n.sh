#!/bin/bash
# round 6: four split slots (the owner Localizer lane gated on the device at the step three back,
# the host's run-ahead wait after the next step's Begin): the split / dist GPU tests, then ABBA
# against build/ab (the tree before) on the sharded step at N = 1, plain and with every exchange
# forced through RCCL
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6n
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6n/tests.log 2>&1 || { tail -30 gpurun_out/r6n/tests.log; exit 1; }
tail -3 gpurun_out/r6n/tests.log
TAG=r6n_sh BENCH_ARGS="--sharded --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6n_fc BENCH_ARGS="--sharded --force-collectives --steps 20 --warmup 5" bash tools/abba.sh || exit 1
for f in gpurun_out/r6n_fc/*.log; do python3 - $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], round(d["value"] / 1e6, 2), d["phases_ms_per_step_rank0"])
PY
done
