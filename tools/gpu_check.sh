#!/bin/bash
# all GPU tests, smoke, then the default bench and the sharded bench (N=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
timeout -k 10 300 python -u bench.py --sharded --no-cpu-baseline > gpurun_out/bench_sharded.log 2>&1 || exit $?
tail -1 gpurun_out/bench_sharded.log
