#!/bin/bash
# One GPU call: parity tests, smoke, short bench.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a gpurun_out/gpu_tests.log
tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
