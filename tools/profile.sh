#!/bin/bash
# rocprofv3 evidence for the bench command: kernel-trace stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) — never combined with tracing (pool rule).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r1}
ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace \
  --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_bench.log 2>&1 || exit $?
echo "trace ok"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o pmc \
  --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || exit $?
echo "fetch ok"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o pmc \
  --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/pmc_write_${TAG}.log 2>&1 || exit $?
echo "write ok"
# the lanes serialised (per-kernel cost in isolation), and the sharded store's synchronous step
DFX_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_serial \
  -o trace --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_serial.log 2>&1 \
  || exit $?
echo "serial ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_sharded -o trace \
  --output-format csv -- python3 bench.py --sharded --sync $ARGS \
  > gpurun_out/prof_${TAG}_sharded.log 2>&1 || exit $?
echo "sharded ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_sharded_pipe -o trace \
  --output-format csv -- python3 bench.py --sharded $ARGS \
  > gpurun_out/prof_${TAG}_sharded_pipe.log 2>&1 || exit $?
echo "sharded pipelined ok"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG}_sharded -o pmc \
  --output-format csv -- python3 bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/pmc_fetch_${TAG}_sharded.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG}_sharded -o pmc \
  --output-format csv -- python3 bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/pmc_write_${TAG}_sharded.log 2>&1 || exit $?
echo "sharded pmc ok"
