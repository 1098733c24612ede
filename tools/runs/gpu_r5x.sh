#!/bin/bash
# One-word atomics on MI355X (tools/membench/atombench), then the block-aggregated pass-W
# append: its tests, then C5 / C3 A/B against build/ab
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 120 ./tools/membench/atombench 20 > gpurun_out/r5/atombench.txt 2>&1 || { cat gpurun_out/r5/atombench.txt; exit 1; }
cat gpurun_out/r5/atombench.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "c5 or two_pass or fused_full" > gpurun_out/r5/t_r5x.log 2>&1 || { tail -40 gpurun_out/r5/t_r5x.log; exit 1; }
tail -1 gpurun_out/r5/t_r5x.log
BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab.sh || exit 1
