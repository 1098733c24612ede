#!/bin/bash
# [GPU tests unless SKIP_TESTS=1], then same-box A/B/C: A = build/ab library, B = in-tree,
# C = in-tree + context kwargs $C_CTX
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_A$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_B$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --ctx "$C_CTX" > gpurun_out/ab_C$i.log 2>&1 || exit 1
done
python3 tools/ab_summary.py gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_C1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log gpurun_out/ab_C2.log
