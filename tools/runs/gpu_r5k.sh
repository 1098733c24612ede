#!/bin/bash
# the C5 Localizer lane alone (tools/locbench zipf): radix vs bucket (splitter map), with traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
export TMPDIR=/tmp
for kw in "loc_bucket=0" ""; do
  timeout -k 10 60 ./build/locbench 100000 39 24 20 "$kw" zipf || exit $?
done
timeout -k 10 60 ./build/locbench 100000 39 24 20 "" || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_locz -o trace \
  --output-format csv -- ./build/locbench 100000 39 24 20 "" zipf > gpurun_out/prof_locz.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/prof_locz/trace_kernel_trace.csv')))
per = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('dfx::', '')
    per[n].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for n, v in per.items():
    v2 = sorted(v)
    print("%-40s n=%3d med=%7.1f" % (n[:40], len(v), v2[len(v2) // 2]))
PY
