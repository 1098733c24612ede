#!/bin/bash
# the fat forward's keys recomputed instead of held (no spills, 107 VGPRs) and at 5 blocks per
# CU (96 VGPRs, spills): forward tests, then C3 A / B / C (3 rounds) and B = 10^4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "fwd or forward or parity or fused_full or walk or fat" > gpurun_out/r5/t_r5ze.log 2>&1 || { tail -40 gpurun_out/r5/t_r5ze.log; exit 1; }
tail -1 gpurun_out/r5/t_r5ze.log
ROUNDS=3 LIBS="build/ab/libdifacto_amd.so build/abB/libdifacto_amd.so tree" BENCH_ARGS="--steps 20 --warmup 5" tools/ab_libs.sh || exit 1
ROUNDS=1 LIBS="build/ab/libdifacto_amd.so build/abB/libdifacto_amd.so tree" BENCH_ARGS="--batch 10000 --steps 300 --warmup 30" tools/ab_libs.sh
