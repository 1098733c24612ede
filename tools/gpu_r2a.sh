#!/bin/bash
# round 2: the pageable-copy probe, every GPU test, the default bench and the sharded bench
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 60 ./build/pageable_probe > gpurun_out/pageable_probe.log 2>&1; cat gpurun_out/pageable_probe.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3; grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r2a.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r2a.log
timeout -k 10 300 python -u bench.py --sharded --no-cpu-baseline > gpurun_out/bench_sharded_r2a.log 2>&1 || exit $?
tail -1 gpurun_out/bench_sharded_r2a.log
