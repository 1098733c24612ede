#!/bin/bash
# GPU tests, then a same-box A/B of the bench: A = build/ab/libdifacto_amd.so, B = in-tree
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh
