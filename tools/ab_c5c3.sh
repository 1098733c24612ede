#!/bin/bash
# Parity tests, then same-box A/Bs alternating: library A (build/ab), B (in-tree), B with kwargs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_par.log
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c5 c4shard}; do
  logs=()
  for i in 1 2; do
    DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --config $c > gpurun_out/abx_A_${c}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --config $c > gpurun_out/abx_B_${c}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --config $c ${KW:+--ctx $KW} > gpurun_out/abx_K_${c}_$i.log 2>&1 || exit 1
    logs+=(gpurun_out/abx_A_${c}_$i.log gpurun_out/abx_B_${c}_$i.log gpurun_out/abx_K_${c}_$i.log)
  done
  python3 tools/ab_summary.py "${logs[@]}"
done
