#!/bin/bash
# round 6: the fused step's AUC snapshot double-buffered at every batch size (the next forward
# then waits, through the Localizer lane's join, for the AUC of two steps back instead of the
# previous step's): the fused-step parity tests, then ABBA against build/ab (HEAD) at the driver
# command for C3 and C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6y
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_r3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6y/tests.log 2>&1 || { tail -30 gpurun_out/r6y/tests.log; exit 1; }
tail -2 gpurun_out/r6y/tests.log
TAG=r6y_c3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6y_c2 ROUNDS=1 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
