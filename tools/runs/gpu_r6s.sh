#!/bin/bash
# round 6: the split driver waits on the library's slot event (dfx_split_slot_event) instead
# of recording its own at the same point of a training step: the split / dist GPU tests, then
# ABBA against build/ab (HEAD before), sharded at N = 1, plain and with the collectives forced
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6s
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6s/tests.log 2>&1 || { tail -30 gpurun_out/r6s/tests.log; exit 1; }
tail -2 gpurun_out/r6s/tests.log
TAG=r6s_sh BENCH_ARGS="--sharded --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6s_fc BENCH_ARGS="--sharded --force-collectives --steps 20 --warmup 5" bash tools/abba.sh || exit 1
