#!/bin/bash
# round 6: the tightened pins (C5 full-size model drift bound, the a2a reordered keys' norm),
# then the small batch (B = 10^4) unprofiled and under a kernel trace (per-launch gaps of the
# main stream: tools/timeline.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6h
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_dist.py -x -q -s --timeout 300 --timeout-method thread -k "c5 or concatenated" > gpurun_out/r6h/tests.log 2>&1
rc=$?; grep -E "drift|passed|failed" gpurun_out/r6h/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch 10000 --steps 300 --warmup 30 > gpurun_out/r6h/b1e4.log 2>&1 || exit 1
python3 tools/bline.py gpurun_out/r6h/b1e4.log b1e4
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6h/prof_b1e4 -o trace --output-format csv \
  -- python3 bench.py --no-cpu-baseline --batch 10000 --steps 100 --warmup 20 > gpurun_out/r6h/prof_b1e4.log 2>&1 || exit 1
python3 tools/bline.py gpurun_out/r6h/prof_b1e4.log b1e4_traced
