#!/bin/bash
# round 6: as gpu_r6w.sh, but the guess read from the Localizer's pinned word as it stands (no
# event query): test_gpu_r6 and the fused-step parity tests, then ABBA against build/ab (HEAD
# before) at the driver command for C3, B = 10^4, C2 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6x
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_r6.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6x/tests.log 2>&1 || { tail -30 gpurun_out/r6x/tests.log; exit 1; }
tail -2 gpurun_out/r6x/tests.log
TAG=r6x_c3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6x_b1e4 BENCH_ARGS="--steps 20 --warmup 5 --batch 10000" bash tools/abba.sh || exit 1
TAG=r6x_c2 ROUNDS=1 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6x_c5 ROUNDS=1 BENCH_ARGS="--config c5 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
