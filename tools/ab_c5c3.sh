#!/bin/bash
# Parity tests of the backward, then same-box A/Bs of context kwargs on the benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py -k "eight_coords or bad_kwargs" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_par.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="c5cpl8|--config c5;c5cpl16|--config c5 --ctx bwd_cpl=16" bash tools/ab_args.sh || exit 1
VARIANTS="c4cpl8|--config c4shard;c4cpl16|--config c4shard --ctx bwd_cpl=16" bash tools/ab_args.sh
