#!/bin/bash
# Round 4 evidence: the small-batch regime (B = 10^4: two bench runs and a kernel trace) and
# the split's loopback N = 8 schedules (pipelined vs 1-step-stale) under a kernel trace, for
# tools/timeline.py.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --batch 10000 --steps 100 --warmup 10 --no-cpu-baseline \
    > gpurun_out/b1e4_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/b1e4_$i.log | cut -c1-200
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4_b1e4 -o trace \
  --output-format csv -- python3 bench.py --batch 10000 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/prof_r4_b1e4.log 2>&1 || exit $?
echo "trace b1e4 ok"
for st in 0 1; do
  timeout -k 10 300 python3 tools/split_loopback.py 8 $st 12 12500 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4_loop8_$st -o trace \
    --output-format csv -- python3 tools/split_loopback.py 8 $st 12 12500 \
    > gpurun_out/prof_r4_loop8_$st.log 2>&1 || exit $?
  echo "trace loopback N=8 stale=$st ok"
done
