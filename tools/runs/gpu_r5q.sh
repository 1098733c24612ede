#!/bin/bash
# key-first bucket sorts: Localizer parity tests, the Localizer alone (uniform, Zipf), C3 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r3.py -x -q \
  --timeout 300 --timeout-method thread -k "bucket" \
  > gpurun_out/r5/t_r5q.log 2>&1 || { tail -40 gpurun_out/r5/t_r5q.log; exit 1; }
tail -1 gpurun_out/r5/t_r5q.log
for kw in "" "loc_bucket=0"; do
  timeout -k 10 60 ./build/locbench 100000 39 24 20 "$kw" || exit 1
  timeout -k 10 60 ./build/locbench 100000 39 24 20 "$kw" zipf || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_locu -o trace \
  --output-format csv -- ./build/locbench 100000 39 24 20 "" > gpurun_out/prof_locu.log 2>&1 || exit 1
grep -E "wbucket|lb_scatter|lb_hist" gpurun_out/prof_locu/trace_kernel_stats.csv | cut -d, -f1-5
BENCH_ARGS="--config c3 --steps 20 --warmup 5" tools/ab.sh || exit 1
BENCH_ARGS="--config c3 --steps 20 --warmup 5" tools/ab.sh || exit 1
