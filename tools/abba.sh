#!/bin/bash
# Same-box A/B in ABBA order (a linear drift of the box over the run cancels): A = the library
# at $A_LIB (DFX_LIB_PATH), B = the in-tree build; ROUNDS (default 2) ABBA blocks of
# `bench.py --no-cpu-baseline $BENCH_ARGS`; logs under gpurun_out/$TAG/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-abba}; mkdir -p gpurun_out/$TAG
run() {  # A|B, index
  local log=gpurun_out/$TAG/$1_$2.log
  if [ $1 = A ]; then
    DFX_LIB_PATH=$PWD/${A_LIB:-build/ab/libdifacto_amd.so} timeout -k 10 300 python3 bench.py --no-cpu-baseline $BENCH_ARGS > $log 2>&1 || exit 1
  else
    timeout -k 10 300 python3 bench.py --no-cpu-baseline $BENCH_ARGS > $log 2>&1 || exit 1
  fi
  python3 tools/bline.py $log $1_$2
}
n=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for x in A B B A; do n=$((n + 1)); run $x $n; done
done
python3 - gpurun_out/$TAG <<'PY'
import glob, json, sys
v = {"A": [], "B": []}
for f in sorted(glob.glob(sys.argv[1] + "/[AB]_*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    v[f.split("/")[-1][0]].append(d["value"] / 1e6)
for k in v:
    print(k, "mean %.2f M ex/s over %d:" % (sum(v[k]) / len(v[k]), len(v[k])), [round(x, 2) for x in v[k]])
PY
