#!/bin/bash
# round-5 closing verification: the whole GPU suite, smoke, the default bench line, then one
# line per other config (c2, c5, c4shard, B = 10^4) and the sharded step at N = 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5f
bash tools/gpu_round.sh || exit $?
cp gpurun_out/bench.log gpurun_out/r5f/bench_default.log
CONFIGS="c2 c5 c4shard b1e4" bash tools/bench_configs.sh > gpurun_out/cfg_all.log 2>&1; rc=$?
cat gpurun_out/cfg_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline --sharded > gpurun_out/r5f/sharded.log 2>&1 || exit $?
tail -c 600 gpurun_out/r5f/sharded.log
