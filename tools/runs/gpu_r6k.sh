#!/bin/bash
# round 6: the finalize folded into the fused InitV launch, without the per-block fences (they
# wrote back each XCD's L2 in every step that drew a V row): the GPU suite, then ABBA x 3 at the
# driver's command (A = build/ab: 276bc7a with the separate finalize; B = the tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6k
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6k/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6k/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=r6k ROUNDS=3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh
