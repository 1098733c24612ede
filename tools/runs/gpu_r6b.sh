#!/bin/bash
# round 6: what each Localizer-lane launch costs the main stream (lb_diag launch skips on a
# workspace that holds an earlier batch: 16 scatter, 32 per-bucket sort, 64 outputs; 128 the
# scatter's items written contiguously by input position to scratch; diag=noloc the whole lane,
# noauc the AUC lane) — measurement only, wrong results; C3, 2 interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r6b
b() {  # label, bench args
  local lab=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 "$@" > gpurun_out/r6b/$lab.log 2>&1 || { tail -20 gpurun_out/r6b/$lab.log; exit 1; }
  python3 tools/bline.py gpurun_out/r6b/$lab.log $lab
}
for r in 1 2; do
  b base_$r
  b skip_scatter_$r --ctx lb_diag=16
  b contig_scatter_$r --ctx lb_diag=128
  b noloc_$r --ctx diag=noloc
  b noauc_$r --ctx diag=noauc
done
