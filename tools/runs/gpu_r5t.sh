#!/bin/bash
# the backward's p from the compact per-row array at V_dim >= 64: the GPU tests that cover the
# wide-V backward, then C5 / C4shard / C3 A/B against build/ab
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c5 or c4 or 128 or 64 or chunk or hot or dist or calcgrad or deferred or fullsize" \
  > gpurun_out/r5/t_r5t.log 2>&1 || { tail -40 gpurun_out/r5/t_r5t.log; exit 1; }
tail -1 gpurun_out/r5/t_r5t.log
BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--config c4shard --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--steps 20 --warmup 5" tools/ab.sh || exit 1
