#!/bin/bash
# round 6: the mid-grouped bucket scatter layout (locbucket.hip lb_mid_on): the GPU suite (the
# bucket Localizer is held bit-exact to the radix one and the oracle), then the driver's
# command A = build/ab (the same tree, layout off) against B = the tree, 3 interleaved rounds,
# then the Localizer lane's FETCH / WRITE per launch for both (separate --pmc passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6g
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6g/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6g/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6g/A$i.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6g/A$i.log A$i
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6g/B$i.log 2>&1 || exit 1
  python3 tools/bline.py gpurun_out/r6g/B$i.log B$i
done
export TMPDIR=/tmp
for v in A B; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    if [ $v = A ]; then export DFX_LIB_PATH=$PWD/build/ab/libdifacto_amd.so; else unset DFX_LIB_PATH; fi
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d gpurun_out/r6g/pmc_${v}_$ctr -o pmc --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r6g/pmc_${v}_$ctr.log 2>&1 || exit $?
  done
  unset DFX_LIB_PATH
  python3 tools/pmc_json.py gpurun_out/r6g/pmc_${v}_FETCH_SIZE/pmc_counter_collection.csv \
    gpurun_out/r6g/pmc_${v}_WRITE_SIZE/pmc_counter_collection.csv gpurun_out/r6g/pmc_$v.json 3 r6g
  python3 - gpurun_out/r6g/pmc_$v.json $v <<'PY'
import json, sys
k = json.load(open(sys.argv[1]))["kernels"]
lb = {n: v for n, v in k.items() if n.startswith("k_lb_")}
tot = sum(v["fetch_size_kb_per_dispatch"] + v["write_size_kb_per_dispatch"] for v in lb.values())
print(sys.argv[2], "lane FETCH+WRITE MB %.1f" % (tot / 1024),
      {n.split("(")[0]: (round(v["fetch_size_kb_per_dispatch"] / 1024, 1), round(v["write_size_kb_per_dispatch"] / 1024, 1)) for n, v in lb.items()})
PY
done
