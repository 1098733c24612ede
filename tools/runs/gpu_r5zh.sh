#!/bin/bash
# B = 10^4 bisection over this session's commits (same box, 3 rounds): 0afea54 (start),
# 7f70c1b (pass V items), 671bcf3 (InitV 8192-key tiles), 12a2abf (striped counters), tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
ROUNDS=3 LIBS="build/ab/libdifacto_amd.so build/ab_7f70c1b/libdifacto_amd.so build/ab_671bcf3/libdifacto_amd.so build/ab_12a2abf/libdifacto_amd.so tree" BENCH_ARGS="--batch 10000 --steps 300 --warmup 30" tools/ab_libs.sh
