#!/bin/bash
# round 6: kernel trace of the small-batch regime (C3 at B = 10^4 per GPU), for the per-launch
# evidence in DESIGN.md (d): profiles/r6/kernel_summary_b1e4.md
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6_b1e4 -o trace \
  --output-format csv -- python3 bench.py --batch 10000 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/prof_r6_b1e4.log 2>&1 && echo "trace b1e4 ok"
