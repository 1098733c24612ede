#!/bin/bash
# round 5: the new kernels' parity, a same-box A/B (tiled forward, AUC lane after the backward),
# then the whole GPU suite (look-back tickets restored, switches pruned this round)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_gpu_r5.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r5/t_r5.log 2>&1 || { tail -30 gpurun_out/r5/t_r5.log; exit 1; }
tail -3 gpurun_out/r5/t_r5.log
SWEEP="base;fwd_tile=1;auc_lane=after;fwd_tile=1,auc_lane=after" timeout -k 10 900 bash tools/ctx_sweep.sh > gpurun_out/r5/sweep_tile.txt 2>&1 || exit 1
tail -12 gpurun_out/r5/sweep_tile.txt
DFX_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --ctx fwd_tile=1 > gpurun_out/r5/serial_tile.json 2>&1 && \
DFX_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r5/serial_base.json 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r5/gpu_tests.log
exit $rc
