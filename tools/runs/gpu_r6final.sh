#!/bin/bash
# round 6, the final tree: the GPU suite, the smoke, then the driver's bench command twice (CPU
# baseline included) and the --steps 100 secondary once; BOX names the log directory
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
D=gpurun_out/r6final_${BOX:-1}; mkdir -p $D
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
  tail -2 $D/tests.log
fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -2 $D/smoke.log
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/k20w5_$i.log 2>&1 || { tail -20 $D/k20w5_$i.log; exit 1; }
  python3 tools/bline.py $D/k20w5_$i.log k20w5_$i
done
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 > $D/k100w10.log 2>&1 || exit 1
python3 tools/bline.py $D/k100w10.log k100w10
