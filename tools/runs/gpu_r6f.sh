#!/bin/bash
# round 6: HBM traffic of the bucket scatter's write patterns (lb_diag, measurement only):
# FETCH_SIZE and WRITE_SIZE passes (separate --pmc runs) of base, 512 (cursors per 4 buckets,
# XCD-contiguous tiles) and 128 (contiguous by input position)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6f
export TMPDIR=/tmp
for v in base:0 mid4xcd:512 contig:128; do
  n=${v%%:*}; b=${v##*:}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d gpurun_out/r6f/pmc_${n}_$ctr -o pmc --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ctx lb_diag=$b > gpurun_out/r6f/pmc_${n}_$ctr.log 2>&1 || exit $?
  done
  python3 tools/pmc_json.py gpurun_out/r6f/pmc_${n}_FETCH_SIZE/pmc_counter_collection.csv \
    gpurun_out/r6f/pmc_${n}_WRITE_SIZE/pmc_counter_collection.csv gpurun_out/r6f/pmc_$n.json 3 r6f
  python3 - gpurun_out/r6f/pmc_$n.json $n <<'PY'
import json, sys
k = json.load(open(sys.argv[1]))["kernels"]
lb = {n: v for n, v in k.items() if n.startswith("k_lb_")}
tot = sum(v["fetch_size_kb_per_dispatch"] + v["write_size_kb_per_dispatch"] for v in lb.values())
print(sys.argv[2], "lane FETCH+WRITE MB %.1f" % (tot / 1024),
      {n.split("(")[0]: (round(v["fetch_size_kb_per_dispatch"] / 1024, 1), round(v["write_size_kb_per_dispatch"] / 1024, 1)) for n, v in lb.items()})
PY
done
