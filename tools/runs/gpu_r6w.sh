#!/bin/bash
# round 6: the hot keys' pre-sum kernels (k_chunk_hotgroup / hotsum) skipped when the newest
# Localizer the host saw finish found no long segment, the backward pre-summing a hot key itself
# when they did not run (fm.hip hot_presum: the same sums): the fused-step and split GPU tests,
# then ABBA against build/ab (HEAD before) at the driver command for C3, B = 10^4, C2 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6w
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_r6.py tests/test_gpu_parity.py tests/test_gpu_r5.py tests/test_gpu_r3.py tests/test_gpu_fullsize.py tests/test_gpu_split.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6w/tests.log 2>&1 || { tail -30 gpurun_out/r6w/tests.log; exit 1; }
tail -2 gpurun_out/r6w/tests.log
TAG=r6w_c3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6w_b1e4 BENCH_ARGS="--steps 20 --warmup 5 --batch 10000" bash tools/abba.sh || exit 1
TAG=r6w_c2 ROUNDS=1 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6w_c5 ROUNDS=1 BENCH_ARGS="--config c5 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
