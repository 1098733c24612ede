#!/bin/bash
# the bucket Localizer's splitter map (Zipf keys): Localizer parity and C5 tests, then C5 / C3
# bench lines and a C5 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r3.py tests/test_gpu_fullsize.py -x -q \
  --timeout 300 --timeout-method thread -k "bucket or c5 or chunk" \
  > gpurun_out/r5/t_r5i.log 2>&1 || { tail -40 gpurun_out/r5/t_r5i.log; exit 1; }
tail -1 gpurun_out/r5/t_r5i.log
for c in c5 c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5/${c}_split.json 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_c5split -o trace \
  --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/prof_r5_c5split.log 2>&1 || exit 1
python3 - <<'PY'
import json, csv
for c in ('c5', 'c3'):
    d = json.loads(open('gpurun_out/r5/%s_split.json' % c).read().strip().split('\n')[-1])
    print(c, round(d['value'] / 1e6, 2), d['ms_per_step'], d['phases_ms_per_step'], d['lanes_ms'])
for r in list(csv.DictReader(open('gpurun_out/prof_r5_c5split/trace_kernel_stats.csv')))[:18]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
