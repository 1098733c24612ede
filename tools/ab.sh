#!/bin/bash
# Same-box A/B: bench with build/ab/libdifacto_amd.so (A) and the in-tree library (B),
# alternating, so box-to-box variance does not decide a comparison.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_A$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_B$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log; do
  echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"
done
