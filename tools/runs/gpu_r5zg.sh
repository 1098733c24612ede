#!/bin/bash
# this session's changes against its starting tree (build/ab = 0afea54), same box:
# B = 10^4 (3 rounds), C3 and C5 (2 rounds each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
ROUNDS=3 LIBS="build/ab/libdifacto_amd.so tree" BENCH_ARGS="--batch 10000 --steps 300 --warmup 30" tools/ab_libs.sh || exit 1
ROUNDS=2 LIBS="build/ab/libdifacto_amd.so tree" BENCH_ARGS="--steps 20 --warmup 5" tools/ab_libs.sh || exit 1
ROUNDS=2 LIBS="build/ab/libdifacto_amd.so tree" BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab_libs.sh
