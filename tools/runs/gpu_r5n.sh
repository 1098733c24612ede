#!/bin/bash
# HOT as a template switch: bucket tests, then C3 (3 rounds) and C5 A/B against build/ab
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r3.py -x -q \
  --timeout 300 --timeout-method thread -k "bucket" \
  > gpurun_out/r5/t_r5n.log 2>&1 || { tail -40 gpurun_out/r5/t_r5n.log; exit 1; }
tail -1 gpurun_out/r5/t_r5n.log
BENCH_ARGS="--config c3 --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--config c3 --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab.sh || exit 1
