#!/bin/bash
# the split's loopback N = 8 with one issuing thread per shard: split tests, then the harness
# (pipelined / stale; threads / one thread) and kernel traces for tools/split_timeline.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
true || timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5/t_r5r.log 2>&1 || { tail -30 gpurun_out/r5/t_r5r.log; exit 1; }
tail -1 gpurun_out/r5/t_r5r.log
# (GPU_MAX_HW_QUEUES=16: 595 ms per step — the queues time-sliced; the default 4 is kept)
for st in 0 1; do
  timeout -k 10 120 python3 tools/split_loopback.py 8 $st 20 12500 || exit 1

  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_lb8_$st -o trace --output-format csv \
    -- python3 tools/split_loopback.py 8 $st 20 12500 > gpurun_out/prof_r5_lb8_$st.log 2>&1 || exit 1
  python3 tools/split_timeline.py gpurun_out/prof_r5_lb8_$st/trace_kernel_trace.csv 8 5 10
done
