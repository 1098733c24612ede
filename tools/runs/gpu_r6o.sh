#!/bin/bash
# round 6: the fused step with one cross-stream wait and two event records fewer on its main
# stream (the AUC join moved onto the Localizer lane, the AUC lane started from the backward's
# phase mark, the parity's free event shared with the capacity guard's): the GPU suite, then
# ABBA against build/ab (HEAD before) at the driver command, C3 and B = 10^4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6o/tests.log 2>&1 || { tail -30 gpurun_out/r6o/tests.log; exit 1; }
tail -2 gpurun_out/r6o/tests.log
TAG=r6o_c3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6o_b1e4 BENCH_ARGS="--steps 20 --warmup 5 --batch 10000" bash tools/abba.sh || exit 1
