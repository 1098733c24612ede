#!/bin/bash
# rocprofv3 kernel-trace per bisection variant (same VARIANTS syntax as ab_multi.sh):
# name|libpath|ctx-kwargs. One trace directory per variant under gpurun_out/tv_<name>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline}
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  IFS='|' read -r name lib ctx <<< "$v"
  if [ -n "$lib" ]; then export DFX_LIB_PATH=$PWD/$lib; else unset DFX_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tv_$name -o trace \
    --output-format csv -- python3 bench.py --ctx "$ctx" $ARGS > gpurun_out/tv_$name.log 2>&1 || exit $?
  echo "trace $name ok"
done
