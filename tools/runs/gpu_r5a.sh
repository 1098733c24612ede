cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5 && \
timeout -k 10 240 ./tools/membench/spanbench 10 > gpurun_out/r5/spanbench.txt 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench_base20.json 2> gpurun_out/r5/bench_base20.err && \
timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_base100.json 2> gpurun_out/r5/bench_base100.err
