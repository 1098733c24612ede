#!/bin/bash
# Parity tests of the backward, then same-box library A/Bs (build/ab = A) on the benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_par.log
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c5 c4shard}; do
  BENCH_ARGS="--config $c" bash tools/ab.sh || exit 1
  python3 tools/ab_summary.py gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log
done
