#!/bin/bash
# round 6: the step's finalize folded into the fused InitV launch (its last block; one launch
# less per step) and the split worker's loss sum + progress in one launch: the GPU suite, then
# A = build/ab (276bc7a, separate finalize) against B = the tree at the driver's command and at
# B = 10^4, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6i
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6i/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6i/tests.log; [ $rc -eq 0 ] || exit $rc
ab() {  # label, bench args
  local lab=$1; shift
  DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/r6i/A_$lab.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6i/A_$lab.log A_$lab
  timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/r6i/B_$lab.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6i/B_$lab.log B_$lab
}
for i in 1 2 3; do ab c3_$i --steps 20 --warmup 5; done
for i in 1 2; do ab b1e4_$i --batch 10000 --steps 300 --warmup 30; done
