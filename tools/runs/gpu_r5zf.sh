#!/bin/bash
# the cold-model counters test (striped backward counters, pass W's folded counts)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py -x -v --timeout 200 --timeout-method thread \
  -k "cold_model" > gpurun_out/r5/t_r5zf.log 2>&1; rc=$?; tail -15 gpurun_out/r5/t_r5zf.log; exit $rc
