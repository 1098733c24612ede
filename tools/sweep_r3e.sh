#!/bin/bash
# all GPU tests, then same-box A/B (build/ab = the previous library) for C3 and C5
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -s > gpurun_out/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab.sh | tee gpurun_out/ab_c3.txt
python3 tools/ab_summary.py gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log
BENCH_ARGS="--config c5" bash tools/ab.sh | tee gpurun_out/ab_c5.txt
python3 tools/ab_summary.py gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log
