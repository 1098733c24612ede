#!/bin/bash
# Parity tests of the backward, then same-box A/Bs of context kwargs on the C5 / C4-shard benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_par.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="cpl4|--config c5 --ctx bwd_cpl=4;cpl8|--config c5" bash tools/ab_args.sh || exit 1
VARIANTS="cpl4|--config c4shard --ctx bwd_cpl=4;cpl8|--config c4shard" bash tools/ab_args.sh
