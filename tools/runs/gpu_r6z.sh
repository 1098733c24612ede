#!/bin/bash
# round 6: the AUC snapshot double-buffered at every batch size (as gpu_r6y.sh), a second box:
# ABBA against build/ab (HEAD) at the driver command for C2, C3 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=r6z_c2 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6z_c3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/abba.sh || exit 1
TAG=r6z_c5 ROUNDS=1 BENCH_ARGS="--config c5 --steps 20 --warmup 5" bash tools/abba.sh || exit 1
