#!/bin/bash
# the fat forward's key recompute taken from 32 k rows only: forward tests, then B = 10^4 (3
# rounds) and C3 (2 rounds) against 12a2abf (no recompute anywhere)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "fwd or forward or parity or fused_full or walk or fat" > gpurun_out/r5/t_r5zi.log 2>&1 || { tail -40 gpurun_out/r5/t_r5zi.log; exit 1; }
tail -1 gpurun_out/r5/t_r5zi.log
ROUNDS=3 LIBS="build/ab_12a2abf/libdifacto_amd.so tree" BENCH_ARGS="--batch 10000 --steps 300 --warmup 30" tools/ab_libs.sh || exit 1
ROUNDS=2 LIBS="build/ab_12a2abf/libdifacto_amd.so tree" BENCH_ARGS="--steps 20 --warmup 5" tools/ab_libs.sh
