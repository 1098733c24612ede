#!/bin/bash
# the bench's other BASELINE configs and the small-batch regime, one bench line each
# (gpurun_out/cfg_<name>.log); BENCH_EXTRA: extra bench.py arguments for every line
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
run() {  # name, then bench arguments
  local name=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline $BENCH_EXTRA "$@" > gpurun_out/cfg_$name.log 2>&1 || exit $?
  python3 - gpurun_out/cfg_$name.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r, f = d["roofline"], d.get("roofline_forward", {})
print("%-10s %8.2f M ex/s  %.4f ms/step  bwd frac %.3f  fwd frac %.3f  host call %.4f ms  U %.0f U_V %s"
      % (sys.argv[1].split("cfg_")[1][:-4], d["value"] / 1e6, d["ms_per_step"], r["frac"],
         f.get("frac", 0), d.get("host_call_ms_idle_device", -1), d["mean_unique_keys"],
         d.get("mean_live_v_keys")))
PY
}
for c in ${CONFIGS:-b1e4 c2 c5 c4shard}; do
  case $c in
    b1e4) run b1e4 --batch 10000 --steps 300 --warmup 30 ;;
    b1e5) run b1e5 ;;
    *) run $c --config $c ;;
  esac
done
