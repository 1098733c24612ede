#!/bin/bash
# pass W's block counts folded by pass V (no per-block atomics on the step's counters), with and
# without 6 waves / SIMD: tests, then C5 A / B / C
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "c5 or two_pass or fused_full or split" > gpurun_out/r5/t_r5y.log 2>&1 || { tail -40 gpurun_out/r5/t_r5y.log; exit 1; }
tail -1 gpurun_out/r5/t_r5y.log
LIBS="build/ab/libdifacto_amd.so build/abB/libdifacto_amd.so tree" BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab_libs.sh
