#!/bin/bash
# InitV drawn a coordinate per thread: the whole GPU suite, then C5 / C3 A/B against build/ab
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5/t_r5u.log 2>&1 || { tail -40 gpurun_out/r5/t_r5u.log; exit 1; }
tail -1 gpurun_out/r5/t_r5u.log
BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--steps 20 --warmup 5" tools/ab.sh || exit 1
