#!/bin/bash
# owner-side kernel times at N = 1, 2, 4, 8 loopback shards (tools/owner_bench.py under rocprofv3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in ${NS:-1 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_owner$n -o trace --output-format csv -- python3 -u tools/owner_bench.py $n 100000 3 > gpurun_out/owner$n.log 2>&1 || exit $?
  echo "n=$n done"
done
