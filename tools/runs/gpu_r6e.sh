#!/bin/bash
# round 6: the split owner's ranked InitV in two launches (was six) and the pruned kwargs /
# variants: the whole GPU suite (InitV draws pinned to the oracle's rand_r sequence), then the
# sharded step at N = 1 (C++ driver, pipelined), A = build/headtree (8564017) against B = the
# tree, 2 interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6e
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6e/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6e/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  (cd build/headtree && timeout -k 10 300 python3 bench.py --no-cpu-baseline --sharded --steps 40 --warmup 5) > gpurun_out/r6e/A$i.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6e/A$i.log A$i
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --sharded --steps 40 --warmup 5 > gpurun_out/r6e/B$i.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6e/B$i.log B$i
done
