#!/bin/bash
# round 5: the walk forward (fwd_tile=2, default) against round 4's fat forward (fwd_tile=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
timeout -k 10 100 ./tools/membench/fwdreal > gpurun_out/r5/fwdreal3.txt 2>&1 || exit 1
cat gpurun_out/r5/fwdreal3.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5/t_r5c.log 2>&1 || { tail -30 gpurun_out/r5/t_r5c.log; exit 1; }
tail -2 gpurun_out/r5/t_r5c.log
SWEEP="base;fwd_tile=0" timeout -k 10 600 bash tools/ctx_sweep.sh > gpurun_out/r5/sweep_walk.txt 2>&1 || exit 1
tail -6 gpurun_out/r5/sweep_walk.txt
BENCH_ARGS="--batch 10000 --steps 300" SWEEP="base;fwd_tile=0" timeout -k 10 600 bash tools/ctx_sweep.sh > gpurun_out/r5/sweep_walk_b1e4.txt 2>&1 || exit 1
tail -6 gpurun_out/r5/sweep_walk_b1e4.txt
