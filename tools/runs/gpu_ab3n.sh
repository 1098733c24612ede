#!/bin/bash
# same-box A/B/C, ROUNDS interleaved rounds (default 3): A = build/ab library, B = in-tree,
# C = in-tree + context kwargs $C_CTX
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
logs=()
for i in $(seq 1 ${ROUNDS:-3}); do
  DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_A$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_B$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --ctx "$C_CTX" > gpurun_out/ab_C$i.log 2>&1 || exit 1
  logs+=(gpurun_out/ab_A$i.log gpurun_out/ab_B$i.log gpurun_out/ab_C$i.log)
done
python3 tools/ab_summary.py "${logs[@]}"
