#!/bin/bash
# round 3: GPU tests of this round's files, then a same-box sweep (SWEEP) of context kwargs
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r3.py -q --timeout 200 --timeout-method thread > gpurun_out/r3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ctx_sweep.sh > gpurun_out/sweep.log 2>&1; rc=$?; tail -20 gpurun_out/sweep.log; exit $rc
