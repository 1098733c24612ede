#!/bin/bash
# the hot-key map: Localizer parity tests, the C5 Localizer lane alone, then C5 / C3 A/B against
# build/ab (the round's tree before the map)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r3.py -x -q \
  --timeout 300 --timeout-method thread -k "bucket" \
  > gpurun_out/r5/t_r5l.log 2>&1 || { tail -40 gpurun_out/r5/t_r5l.log; exit 1; }
tail -1 gpurun_out/r5/t_r5l.log
tools/runs/gpu_r5k.sh || exit 1
BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab.sh || exit 1
