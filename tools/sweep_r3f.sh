#!/bin/bash
# this round's GPU tests, A/B against the round-2 library (build/ab), Localizer-mode sweep
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r3.py -q --timeout 300 --timeout-method thread -s > gpurun_out/r3_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r3_tests.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab.sh > gpurun_out/ab_c3.txt 2>&1 || exit $?
python3 tools/ab_summary.py gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log
SWEEP="loc_bucket=0;loc_bucket=1;loc_bucket=2" bash tools/ctx_sweep.sh > gpurun_out/sweep.log 2>&1; rc=$?; tail -6 gpurun_out/sweep.log; exit $rc
