#!/bin/bash
# round 6: the bucket scatter's write pattern (measurement only, wrong results): 128 items
# written contiguously by input position; 256 at tile-local positions (each tile's items grouped
# by bucket inside the tile's own range: no better than base); 512 cursors per 4 buckets (runs of
# ~30 items) with each XCD a contiguous range of tiles; C3, 3 interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6c
b() {  # label, bench args
  local lab=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 "$@" > gpurun_out/r6c/$lab.log 2>&1 || { tail -20 gpurun_out/r6c/$lab.log; exit 1; }
  python3 tools/bline.py gpurun_out/r6c/$lab.log $lab
}
for r in 1 2 3; do
  b base_$r
  b contig_$r --ctx lb_diag=128
  b mid4xcd_$r --ctx lb_diag=512
done
