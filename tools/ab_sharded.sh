#!/bin/bash
# sharded-store GPU tests, then a same-box A/B of the sharded bench (build/ab = A)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_host_cpp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dist_tests.log 2>&1; rc=$?; tail -3 gpurun_out/dist_tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--sharded ${BENCH_ARGS:-}" bash tools/ab.sh
