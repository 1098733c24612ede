#!/bin/bash
# round 6: re-check the context kwargs tuned in earlier rounds on the tree with fewer stream
# events (driver command, same box, two interleaved rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SWEEP="base;nt=1;nt=8;bwd_lds=16384;bwd_lds=8192;lb_hnt=512" BENCH_ARGS="--steps 20 --warmup 5" bash tools/ctx_sweep.sh
