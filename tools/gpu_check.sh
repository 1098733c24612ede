#!/bin/bash
# One GPU call for a change under test: the named GPU tests (TESTS, pytest paths / node ids;
# TEST_K: a -k expression), then a same-box context-kwarg sweep of the bench (SWEEP, as
# tools/ctx_sweep.sh).  Stops at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS ${TEST_K:+-k "$TEST_K"} -x -v \
    --timeout 200 --timeout-method thread > gpurun_out/check_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/check_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$SWEEP" ]; then
  bash tools/ctx_sweep.sh > gpurun_out/check_sweep.log 2>&1
  rc=$?
  tail -${SWEEP_TAIL:-12} gpurun_out/check_sweep.log
  exit $rc
fi
