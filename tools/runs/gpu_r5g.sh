#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py -x -q --timeout 300 --timeout-method thread -k "tile" \
  > gpurun_out/r5/t_r5g.log 2>&1 || { tail -40 gpurun_out/r5/t_r5g.log; exit 1; }
tail -1 gpurun_out/r5/t_r5g.log
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5/c5_t64.json 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_c5t64 -o trace \
  --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/prof_r5_c5t64.log 2>&1 || exit 1
python3 - <<'PY'
import json, csv
d = json.loads(open('gpurun_out/r5/c5_t64.json').read().strip().split('\n')[-1])
print('c5 t64', round(d['value'] / 1e6, 2), d['ms_per_step'], d['phases_ms_per_step'])
for r in list(csv.DictReader(open('gpurun_out/prof_r5_c5t64/trace_kernel_stats.csv')))[:12]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
