cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=tests/test_host_cpp.py::test_train_driver_sharded_loopback_matches_oracle
for v in NONE DFX_NO_SEGS_PULL DFX_NO_INITV_GATE; do
  env $v=1 timeout -k 10 120 python -m pytest "$T" -m gpu -x -q --timeout 100 > gpurun_out/bis_$v.log 2>&1; echo "$v rc=$?"
done
