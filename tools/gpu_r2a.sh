cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 60 ./build/pageable_probe > gpurun_out/pageable_probe.log 2>&1; cat gpurun_out/pageable_probe.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r2a.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r2a.log
