#!/bin/bash
# round 6: the split step with two event records, one copy and one cross-stream wait fewer on
# the main stream (the forward's and backward's slot-free records dropped for training steps,
# the capacity guard's counts written by the ranked InitV draw's last block and its event
# freeing the slot, the AUC join on the owner Localizer lane, the run-ahead bound on the slots'
# own events): the split / dist GPU tests, then ABBA against build/ab (HEAD before), sharded
# at N = 1, plain and with every exchange forced through RCCL
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6p
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6p/tests.log 2>&1 || { tail -30 gpurun_out/r6p/tests.log; exit 1; }
tail -2 gpurun_out/r6p/tests.log
TAG=r6p_sh BENCH_ARGS="--sharded --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6p_fc BENCH_ARGS="--sharded --force-collectives --steps 20 --warmup 5" bash tools/abba.sh || exit 1
