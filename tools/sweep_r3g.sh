#!/bin/bash
# round-3 GPU tests, then the Localizer-mode A/B against the round-2 library
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_parity.py -q -s --timeout 300 --timeout-method thread -x > gpurun_out/r3_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r3_tests.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/r3_tests.log | head; exit $rc; fi
VARIANTS="r2|build/ab/r2/libdifacto_amd.so|;b0||loc_bucket=0;b1||loc_bucket=1;b2||loc_bucket=2;op0||loc_bucket=0,loc_onepass=1" bash tools/ab_multi.sh
