#!/bin/bash
# all GPU tests, then the C3 and C5 bench lines
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s > gpurun_out/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
CONFIGS="${CONFIGS:-b1e5 c5}" bash tools/bench_configs.sh
