#!/bin/bash
# round 6: the finalize folded into the fused InitV launch, ABBA x 3 at the driver's command
# (A = build/ab: 276bc7a with the separate finalize; B = the tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=r6j ROUNDS=3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh
