#!/bin/bash
# round 6: the GPU suite on the tree with the late Localizer wait (a training step's forward
# waits for its batch only, the backward for the Localizer) and ADVICE r5's fixes; then the
# driver's command, A = build/ab (HEAD 85b4640) against B = the tree, 3 interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6d
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6d/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6d/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6d/A$i.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6d/A$i.log A$i
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6d/B$i.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6d/B$i.log B$i
done
