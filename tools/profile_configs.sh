#!/bin/bash
# rocprofv3 evidence for the bench's other BASELINE configs (bench.py --config c2|c5|c4shard):
# a kernel-trace run each, then separate FETCH_SIZE / WRITE_SIZE passes (never combined with
# tracing); bench.py reads profiles/<PMC_ROUND>/pmc_hbm_<config>.json for its traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r3}
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CONFIGS:-c2 c5 c4shard}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$c -o trace \
    --output-format csv -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/prof_${TAG}_$c.log 2>&1 || exit $?
  echo "trace $c ok"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_${c}_$ctr -o pmc \
      --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/pmc_${TAG}_${c}_$ctr.log 2>&1 || exit $?
    echo "pmc $c $ctr ok"
  done
done
