export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_split.py -k "cpp" > gpurun_out/cpp_split.log 2>&1 || { echo TESTFAIL; exit 1; }
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --sharded --force-collectives --steps 40 --no-cpu-baseline > gpurun_out/cpp_f.log 2>&1 || { echo BENCHF; exit 1; }
timeout -k 10 200 python bench.py --sharded --steps 40 --no-cpu-baseline > gpurun_out/cpp_n.log 2>&1 || { echo BENCHN; exit 1; }
echo ok
