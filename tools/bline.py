#!/usr/bin/env python3
"""one summary line of a bench.py log (its last JSON line): value, ms/step, phases, lanes and
the step window's shape; usage: bline.py LOG [LABEL]"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lab = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
w = dict(d.get("step_window") or {})
w.pop("ms", None)
ph = d.get("phases_ms_per_step") or d.get("phases_ms_per_step_rank0") or {}
print("%-24s %8.2f M ex/s %.4f ms  K=%s W=%s | fwd %.4f bwd %.4f | lanes %s | window %s"
      % (lab, d["value"] / 1e6, d["ms_per_step"], d["steps"], d["warmup"],
         ph.get("forward", -1), ph.get("backward_update", -1), d.get("lanes_ms"), w), flush=True)
