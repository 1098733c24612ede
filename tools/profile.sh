#!/bin/bash
# rocprofv3 evidence for the bench command: kernel-trace stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, the L2's memory-side request counters) — never combined with
# tracing (pool rule).  Every GPU step has its own time limit; the chain stops at the first
# failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r2}
ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline}
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, then the bench arguments
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$name -o trace \
    --output-format csv -- python3 bench.py "$@" > gpurun_out/prof_${TAG}_$name.log 2>&1 \
    || exit $?
  echo "trace $name ok"
}
pmc() {  # name, counters, then the bench arguments
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 200 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_$name -o pmc \
    --output-format csv -- python3 bench.py "$@" > gpurun_out/pmc_${TAG}_$name.log 2>&1 \
    || exit $?
  echo "pmc $name ok"
}
SHORT="--steps 3 --warmup 1 --no-cpu-baseline"
run fused $ARGS
DFX_SERIAL=1 run serial $ARGS
run split --sharded $ARGS
run a2a --sharded --collective a2a $ARGS
pmc fetch FETCH_SIZE $SHORT
pmc write WRITE_SIZE $SHORT
pmc req "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" $SHORT
pmc fetch_split FETCH_SIZE --sharded $SHORT
pmc write_split WRITE_SIZE --sharded $SHORT
