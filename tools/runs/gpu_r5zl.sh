#!/bin/bash
# the one-kernel fused backward's LDS reservation 16 -> 12 KiB (kBwdLdsCapFused): C3 (3 rounds),
# C2 and the C4 shard (2 rounds each) against build/ab (16 KiB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
ROUNDS=3 LIBS="build/ab/libdifacto_amd.so tree" BENCH_ARGS="--steps 40 --warmup 5" tools/ab_libs.sh || exit 1
ROUNDS=2 LIBS="build/ab/libdifacto_amd.so tree" BENCH_ARGS="--config c2 --steps 20 --warmup 5" tools/ab_libs.sh || exit 1
ROUNDS=2 LIBS="build/ab/libdifacto_amd.so tree" BENCH_ARGS="--config c4shard --steps 20 --warmup 5" tools/ab_libs.sh
