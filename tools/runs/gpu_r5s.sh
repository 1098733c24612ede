#!/bin/bash
# hot rows in LDS for the V_dim >= 64 forward: bit-identity and C5 tests, then C5 A/B on the
# same box (fwd_hot=0 / 1) and a C5 trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_fullsize.py tests/test_gpu_r3.py -x -q \
  --timeout 300 --timeout-method thread -k "hot or c5" \
  > gpurun_out/r5/t_r5s.log 2>&1 || { tail -40 gpurun_out/r5/t_r5s.log; exit 1; }
tail -1 gpurun_out/r5/t_r5s.log
ROUNDS=2 VARIANTS="c5|--config c5 --steps 20 --warmup 5;c5nohot|--config c5 --steps 20 --warmup 5 --ctx fwd_hot=0" tools/ab_args.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_c5hot -o trace \
  --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/prof_r5_c5hot.log 2>&1 || exit 1
grep -E "fwd|stage" gpurun_out/prof_r5_c5hot/trace_kernel_stats.csv | cut -d, -f1-4
