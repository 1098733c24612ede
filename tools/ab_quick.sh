cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py -k "two_pass or eight_coords" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_par.log
[ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--config c5" bash tools/ab.sh && python3 tools/ab_summary.py gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log
