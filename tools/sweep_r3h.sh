#!/bin/bash
# round-3 GPU tests (C5 drift against the exact trajectory), then the Localizer lane on a CU
# subset (loc_cus) A/B
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py -q -s --timeout 200 --timeout-method thread -x -k "c5_model_drift or bucket" > gpurun_out/r3_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r3_tests.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/r3_tests.log | head; exit $rc; fi
VARIANTS="all||;s128||loc_cus=128;s64||loc_cus=64;s32||loc_cus=32;b64||loc_cus=64,loc_cu_block=1;b32||loc_cus=32,loc_cu_block=1" bash tools/ab_multi.sh
