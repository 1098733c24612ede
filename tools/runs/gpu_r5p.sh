#!/bin/bash
# B = 10^4 (SURVEY's per-GPU C3 batch): bench lines, then kernel traces as run and serialised
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --batch 10000 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/r5/b1e4_$i.json 2>&1 || exit 1
done
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r5/b1e5.json 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_b1e4 -o trace --output-format csv \
  -- python3 bench.py --batch 10000 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r5_b1e4.log 2>&1 || exit 1
DFX_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_b1e4s -o trace --output-format csv \
  -- python3 bench.py --batch 10000 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r5_b1e4s.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ('b1e4_1', 'b1e4_2', 'b1e5'):
    d = json.loads(open('gpurun_out/r5/%s.json' % f).read().strip().split('\n')[-1])
    print(f, round(d['value'] / 1e6, 2), d['ms_per_step'], d['phases_ms_per_step'], d['lanes_ms'], d.get('host_call_ms_idle_device'))
PY
