cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4a_fused -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r4a_fused.log 2>&1 && \
DFX_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4a_serial -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r4a_serial.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4a_lsd -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --ctx loc_bucket=0 > gpurun_out/prof_r4a_lsd.log 2>&1
