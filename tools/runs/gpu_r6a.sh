#!/bin/bash
# round 6: where the driver's 20-step window loses against 100 steps — the same tree on one box
# at the driver's command, at 100 steps, and with a long warmup; per-step window shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6a
b() {  # label, bench args
  local lab=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/r6a/$lab.log 2>&1 || { tail -20 gpurun_out/r6a/$lab.log; exit 1; }
  python3 tools/bline.py gpurun_out/r6a/$lab.log $lab
}
b k20w5_a --steps 20 --warmup 5
b k100w10 --steps 100 --warmup 10
b k20w50 --steps 20 --warmup 50
b k20w5_b --steps 20 --warmup 5
b k100w10_b --steps 100 --warmup 10
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_r5.py -x -q --timeout 120 --timeout-method thread -k "splitter" > gpurun_out/r6a/t_splitter.log 2>&1; rc=$?; tail -3 gpurun_out/r6a/t_splitter.log; exit $rc
