#!/bin/bash
# round 6: the fused step's chunk kernels on one block each when the newest Localizer the host
# saw finish found no long segment (no host wait; same partials on any grid): the fused-step GPU
# tests (test_gpu_r6, parity, r5, r3, full size), then ABBA against build/ab (HEAD before) at
# the driver command for C3, B = 10^4, C2 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6v
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_r6.py tests/test_gpu_parity.py tests/test_gpu_r5.py tests/test_gpu_r3.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6v/tests.log 2>&1 || { tail -30 gpurun_out/r6v/tests.log; exit 1; }
tail -2 gpurun_out/r6v/tests.log
TAG=r6v_c3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6v_b1e4 BENCH_ARGS="--steps 20 --warmup 5 --batch 10000" bash tools/abba.sh || exit 1
TAG=r6v_c2 ROUNDS=1 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6v_c5 ROUNDS=1 BENCH_ARGS="--config c5 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
