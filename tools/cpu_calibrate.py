#!/usr/bin/env python3
"""Calibrate the CPU baseline port (oracle/cpu_ref.cc) against the survey's measurement of the
reference itself (FM V_dim=16, 39 nnz/row, 2^24 uniform keys, B=10^4,
2 OpenMP threads: 35.8 k ex/s = 200 k rows over the SUM of its phases — Localizer 0.48 s, Get
1.0 s, Predict(+Eval+AUC) 0.59 s, CalcGrad 0.32 s, Update 3.2 s — i.e. timed sequentially), in
the container class the survey measured it in.  The survey does not record its updater settings,
so both are run: the bench's (l1=0, V_threshold=0: every key carries V) and the reference
defaults (l1=1, V_threshold=10: almost no key gets V).  Two schedules each: "sequential" (one
thread runs Compact then the executor per batch, the survey's method) and "pipelined" (the
reference's IterateData: Localizer on the reader thread beside the executor thread, as
bench.py's cpu_baseline runs it).  Prints one JSON object (profiles/r6/cpu_calibration.json)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from difacto_amd import data as D  # noqa: E402
from oracle import cpu_ref as C  # noqa: E402

SURVEY = {"ex_per_s": 35800.0,
          "s_per_200k_rows": {"localize": 0.48, "get": 1.0, "predict_eval_auc": 0.59,
                              "calcgrad": 0.32, "update": 3.2}}


def per200k(ph, n):
    s = 200_000 / n
    out = {"localize": ph["localize"] * s, "get": ph["get"] * s,
           "predict_eval_auc": (ph["predict"] + ph["evaluate_auc"]) * s,
           "calcgrad": ph["calcgrad"] * s, "update": ph["update"] * s}
    return {k: round(v, 3) for k, v in out.items()}


def main():
    rows = int(os.environ.get("CAL_ROWS", "200000"))
    B, k, kb, d = 10_000, 39, 24, 16
    nb = rows // B
    blocks = [D.synthetic(B, k, 1 << kb, seed=1000 + i) for i in range(nb)]
    out = {}
    for label, kw in (("all_V (bench settings)", dict(V_dim=d, V_threshold=0, l1=0, lr=.1,
                                                      V_lr=.01)),
                      ("reference defaults", dict(V_dim=d))):
        ref = C.CpuRef(2, **kw)
        for b in blocks:  # the count-push epoch (untimed), as bench.py
            ref.step(b, push_cnt=True)
        res = {}
        for nt in (2, 1):
            ref.nt = nt
            C.phases()
            t = time.perf_counter()
            for b in blocks:
                ref.step(b)
            dt = time.perf_counter() - t
            ph = per200k(C.phases(), nb * B)
            seq = {"ex_per_s": round(nb * B / dt, 1), "s_per_200k_rows": ph,
                   "vs_survey": round(nb * B / dt / SURVEY["ex_per_s"], 3),
                   "phase_vs_survey": {p: round(v / SURVEY["s_per_200k_rows"][p], 2)
                                       for p, v in ph.items()}}
            C.phases()
            dt, _, _, n = ref.iterate(blocks)
            pip = {"ex_per_s": round(n / dt, 1), "s_per_200k_rows": per200k(C.phases(), n),
                   "vs_survey": round(n / dt / SURVEY["ex_per_s"], 3)}
            res[str(nt)] = {"sequential": seq, "pipelined": pip}
        res["model_keys"] = ref.size()
        ref.close()
        out[label] = {"settings": kw, "by_threads": res}
    out["survey_reference"] = SURVEY
    out["host"] = {"cpus": os.cpu_count(), "where": "build container (the survey's host class)"}
    out["shape"] = ("B=10^4, 39 binary nnz/row, ids ~ U[0, 2^24), V_dim=16, %d rows after an "
                    "untimed count-push epoch over them" % (nb * B))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
