#!/bin/bash
# round 5: the whole GPU suite, smoke and the default bench on the pruned tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5/gpu_tests_d.log 2>&1; rc=$?
tail -5 gpurun_out/r5/gpu_tests_d.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r5/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench_d20.json 2> gpurun_out/r5/bench_d20.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r5/bench_d100.json 2> gpurun_out/r5/bench_d100.err || exit 1
python3 - <<'PY'
import json
for f in ['bench_d20', 'bench_d100']:
    d = json.loads(open('gpurun_out/r5/%s.json' % f).read().strip().split('\n')[-1])
    print(f, round(d['value'] / 1e6, 2), d['ms_per_step'], d['roofline']['frac'], d['phases_ms_per_step']['forward'], d['phases_ms_per_step']['backward_update'])
PY
