#!/bin/bash
# round 6: the split and a2a paths record snapshot buffer 0's last-reader event too (a fused step
# of the same context, double-buffered at every size now, waits on it): the split / dist /
# fused-parity GPU tests and the smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6aa
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_dist.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6aa/tests.log 2>&1 || { tail -30 gpurun_out/r6aa/tests.log; exit 1; }
tail -2 gpurun_out/r6aa/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6aa/smoke.log 2>&1 || { tail -20 gpurun_out/r6aa/smoke.log; exit 1; }
tail -1 gpurun_out/r6aa/smoke.log
