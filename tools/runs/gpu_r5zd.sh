#!/bin/bash
# pass V with 16 lanes per key (two float4 each): its tests, then C5 / C4 shard A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "c5 or two_pass or fused_full or split" > gpurun_out/r5/t_r5zd.log 2>&1 || { tail -40 gpurun_out/r5/t_r5zd.log; exit 1; }
tail -1 gpurun_out/r5/t_r5zd.log
LIBS="build/ab/libdifacto_amd.so tree" BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab_libs.sh
