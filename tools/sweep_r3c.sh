#!/bin/bash
# round 3: this round's GPU tests, the other configs' bench lines, a pipelined kernel trace
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r3.py -q --timeout 200 --timeout-method thread -s > gpurun_out/r3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/bench_configs.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3x -o trace --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r3x.log 2>&1 || exit $?
echo trace ok
