#!/bin/bash
# C5 with 128-occurrence chunks and the parallel hot-key pre-sum: the chunk parity tests, the
# bench line and a kernel trace of the same command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_r3.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "c5 or chunk or hot or zipf" \
  > gpurun_out/r5/t_r5h.log 2>&1 || { tail -40 gpurun_out/r5/t_r5h.log; exit 1; }
tail -1 gpurun_out/r5/t_r5h.log
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5/c5_c128c.json 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_c5c128c -o trace \
  --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/prof_r5_c5c128c.log 2>&1 || exit 1
python3 - <<'PY'
import json, csv
d = json.loads(open('gpurun_out/r5/c5_c128c.json').read().strip().split('\n')[-1])
print('c5 c128', round(d['value'] / 1e6, 2), d['ms_per_step'], d['phases_ms_per_step'])
for r in list(csv.DictReader(open('gpurun_out/prof_r5_c5c128c/trace_kernel_stats.csv')))[:14]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
