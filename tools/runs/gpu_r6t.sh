#!/bin/bash
# round 6: the fused step's chunk plan and chunk kernels only when the batch two back on the
# same parity had a long segment (host-visible pinned flag, read after that batch's Localizer):
# the GPU suite, then ABBA against build/ab (HEAD before) at the driver command for C3, B = 10^4,
# C2 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6t
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6t/tests.log 2>&1 || { tail -30 gpurun_out/r6t/tests.log; exit 1; }
tail -2 gpurun_out/r6t/tests.log
TAG=r6t_c3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6t_b1e4 BENCH_ARGS="--steps 20 --warmup 5 --batch 10000" bash tools/abba.sh || exit 1
TAG=r6t_c2 ROUNDS=1 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6t_c5 ROUNDS=1 BENCH_ARGS="--config c5 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
