#!/bin/bash
# splitter map with the interleaved descent: its tests, then same-box A/B against the key-map
# build (build/ab) on C5 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r3.py -x -q \
  --timeout 300 --timeout-method thread -k "bucket" \
  > gpurun_out/r5/t_r5j.log 2>&1 || { tail -40 gpurun_out/r5/t_r5j.log; exit 1; }
tail -1 gpurun_out/r5/t_r5j.log
BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--config c3 --steps 20 --warmup 5" tools/ab.sh || exit 1
ROUNDS=1 VARIANTS="c5|--config c5 --steps 20 --warmup 5;c5locl|--config c5 --steps 20 --warmup 5 --ctx lane_prio=loc_low;c5noloc|--config c5 --steps 20 --warmup 5 --ctx diag=noloc" tools/ab_args.sh
