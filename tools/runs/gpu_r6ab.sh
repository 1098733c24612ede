#!/bin/bash
# round 6: the split combine's AUC snapshot double-buffered (as the fused step's): the split /
# dist / fused-parity GPU tests, then ABBA against build/ab (HEAD before) on the sharded step at
# N = 1, plain and with the collectives forced, and C3 fused (the shared event bookkeeping)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6ab
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_dist.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6ab/tests.log 2>&1 || { tail -30 gpurun_out/r6ab/tests.log; exit 1; }
tail -2 gpurun_out/r6ab/tests.log
TAG=r6ab_sh BENCH_ARGS="--sharded --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6ab_fc BENCH_ARGS="--sharded --force-collectives --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6ab_c3 ROUNDS=1 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
