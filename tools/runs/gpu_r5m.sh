#!/bin/bash
# chunk plan as reduce / scan / apply and the hot map's rank sort: Localizer + chunk parity
# tests, the C5 Localizer lane alone, then C5 and C3 A/B against build/ab
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r3.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "bucket or c5 or chunk or hot or zipf or skew" \
  > gpurun_out/r5/t_r5m.log 2>&1 || { tail -40 gpurun_out/r5/t_r5m.log; exit 1; }
tail -1 gpurun_out/r5/t_r5m.log
tools/runs/gpu_r5k.sh || exit 1
BENCH_ARGS="--config c5 --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--config c3 --steps 20 --warmup 5" tools/ab.sh || exit 1
