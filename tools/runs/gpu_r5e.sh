#!/bin/bash
# round 5: tile chunks (hot keys summed per row tile) — parity, then C5's bench and kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r3.py tests/test_gpu_fullsize.py -x -q \
  --timeout 300 --timeout-method thread -k "tile or c5 or zipf or hot or walk or split" \
  > gpurun_out/r5/t_r5e.log 2>&1 || { tail -40 gpurun_out/r5/t_r5e.log; exit 1; }
tail -2 gpurun_out/r5/t_r5e.log
grep -E "tile chunks d=|C5 per-step" gpurun_out/r5/t_r5e.log | head
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/r5/c5_$i.json 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_c5 -o trace \
  --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/prof_r5_c5.log 2>&1 || exit 1
python3 - <<'PY'
import json
for i in (1, 2):
    d = json.loads(open('gpurun_out/r5/c5_%d.json' % i).read().strip().split('\n')[-1])
    print('c5', round(d['value'] / 1e6, 2), d['ms_per_step'], d['phases_ms_per_step'])
PY
