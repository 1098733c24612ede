bash tools/gpu_round.sh && CONFIGS="b1e5 c2 c5 c4shard b1e4" bash tools/bench_configs.sh > gpurun_out/cfg_all.log 2>&1; rc=$?; cat gpurun_out/cfg_all.log; exit $rc
