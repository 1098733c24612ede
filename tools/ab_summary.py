"""one line per bench log: throughput, main-stream phases, lane times (fused bench), or the
owner phases of rank 0 (sharded bench)"""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    name = f.split("/")[-1]
    if "phases_ms_per_step" in d:
        p = d["phases_ms_per_step"]
        ln = d["lanes_ms"]
        print("%-22s %7.2f M ex/s  fwd %.3f bwd %.3f initv %.3f eval %.3f  loc %.3f auc %.3f "
              "frac %.3f" % (name, d["value"] / 1e6, p["forward"], p["backward_update"],
                             p["initv"], p["eval_auc"], ln["loc_ms"], ln["auc_ms"],
                             d["roofline"]["frac"]))
    else:
        p = d.get("phases_ms_per_step_rank0", {})
        print("%-22s %7.2f M ex/s  %s  frac %.3f" % (
            name, d["value"] / 1e6, " ".join("%s %.3f" % kv for kv in p.items()),
            d["roofline"]["frac"]))
