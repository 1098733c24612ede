#!/bin/bash
# tools/locbench on the GPU box: the Localizer alone, radix vs bucket and the bucket kernel's
# measurement switches (lb_diag), then a kernel trace of the default.  B=${LB_B:-100000}.
# LB_AUC=1: the AUC lane alone instead (radix / merge), and a trace of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${LB_B:-100000}
if [ -n "$LB_C2" ]; then  # C2's shape: 40 valued nnz per row over 2^20 ids
  for kw in "loc_bucket=0" "" "lb_gather=0" ${LB_VARIANTS:-}; do
    timeout -k 10 60 ./build/locbench $B 40 20 20 "$kw" valued || exit $?
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_locbench_c2 -o trace \
    --output-format csv -- ./build/locbench $B 40 20 20 "" valued > gpurun_out/prof_locbench_c2.log 2>&1
  exit $?
fi
if [ -n "$LB_AUC" ]; then
  for kw in "auc_sort=radix" "auc_sort=merge"; do
    timeout -k 10 60 ./build/locbench $B 39 24 20 "$kw" auc || exit $?
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aucbench -o trace \
    --output-format csv -- ./build/locbench $B 39 24 20 "" auc > gpurun_out/prof_aucbench.log 2>&1
  exit $?
fi
for kw in "loc_bucket=0" "" ${LB_VARIANTS:-"lb_diag=1" "lb_diag=4" "lb_diag=5"}; do
  timeout -k 10 60 ./build/locbench $B 39 24 20 "$kw" || exit $?
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_locbench -o trace \
  --output-format csv -- ./build/locbench $B 39 24 20 "" > gpurun_out/prof_locbench.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_locbench_lsd -o trace \
  --output-format csv -- ./build/locbench $B 39 24 20 "loc_bucket=0" > gpurun_out/prof_locbench_lsd.log 2>&1 || exit $?
# LB_TRACE="kw;kw": kernel traces of further variants (gpurun_out/prof_locbench_v<i>)
IFS=';' read -ra TR <<< "${LB_TRACE:-}"
i=0
for kw in "${TR[@]}"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_locbench_v$i -o trace \
    --output-format csv -- ./build/locbench $B 39 24 20 "$kw" > gpurun_out/prof_locbench_v$i.log 2>&1 || exit $?
  i=$((i+1))
done
