#!/bin/bash
# round 3: the new kernels' GPU tests, then a same-box sweep of the forward / AUC variants and
# the side lanes' headroom (diag=...), then serialised forward timings
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_r3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
export SWEEP="${SWEEP:-base;fwd_lanes=2,fat_nb=4;fwd_lanes=4,fat_nb=4;fwd_lanes=4,fat_nb=6;auc_sort=block;diag=noauc;diag=noloc;diag=noauc_noloc}"
bash tools/ctx_sweep.sh > gpurun_out/sweep1.log 2>&1; rc=$?; tail -20 gpurun_out/sweep1.log; [ $rc -ne 0 ] && exit $rc
for c in "" "fwd_lanes=2,fat_nb=4" "fwd_lanes=4,fat_nb=4"; do
  DFX_SERIAL=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 30 --ctx "$c" > "gpurun_out/ser_$c.log" 2>&1 || exit 1
  echo "serial [$c]"; python3 tools/ab_summary.py "gpurun_out/ser_$c.log"
done
