#!/bin/bash
# same-box sweep of context kwargs: SWEEP="base;k=v;k=v,k2=v2" (base = no extra kwargs), each
# config benched twice, interleaved; "k=v@--flag x" adds bench flags to one config
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
IFS=';' read -ra CFG <<< "$SWEEP"
logs=()
for i in 1 2; do
  n=0
  for c in "${CFG[@]}"; do
    x="${c%%@*}"; [ "$x" = "base" ] && x=""
    extra=""; [[ "$c" == *@* ]] && extra="${c#*@}"
    f=gpurun_out/sw_${n}_$i.log
    timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS $extra --ctx "$x" > $f 2>&1 || exit 1
    echo "$f = $c"
    logs+=($f)
    n=$((n+1))
  done
done
python3 tools/ab_summary.py "${logs[@]}"
