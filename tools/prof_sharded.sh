#!/bin/bash
# sharded-store bench (pipelined, N=1 RCCL) + its kernel trace + a host-side Python profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sh}
timeout -k 10 300 python3 bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
DFX_PYPROF=gpurun_out/${TAG}_pyprof.out timeout -k 10 300 python3 bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_pyprof.log 2>&1 || exit $?
[ -n "$NOTRACE" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o trace --output-format csv -- python3 bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
