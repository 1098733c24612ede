cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="tests/test_host_cpp.py::test_train_driver_sharded_loopback_matches_oracle tests/test_gpu_dist.py"
for i in 1 2 3 4; do
  timeout -k 10 200 python -m pytest $T -m gpu -q --timeout 150 > gpurun_out/stress_$i.log 2>&1; echo "run $i rc=$? $(tail -1 gpurun_out/stress_$i.log)"
done
