"""Summarise a rocprofv3 kernel trace (+ optional FETCH/WRITE PMC passes) over the bench's
timed steps, as markdown.

The timed window is the last N steps: it starts where the (N+1)-th-from-last step's
`k_step_finalize` ended and stops where the last one ended.  Per kernel: dispatches per step,
average duration, microseconds per step, and the busy fraction of the window.
usage: prof_summary.py trace.csv N [fetch_pmc.csv write_pmc.csv]
DFX_STEP_MARKER (default: k_step_finalize or k_initv_onepass — since round 6 a V_dim > 0 training
step finalizes in its InitV launch; the sharded store: k_dist_worker_finalize, the split:
k_split_worker_finalize; comma-separated alternatives) names the once-per-step kernel the window
is anchored on;
DFX_STEP_SKIP skips that many trailing steps (the bench's secondary schedule runs).
"""
import collections
import csv
import os
import sys


def short(name):
    s = name.split("(")[0]
    return s.replace("void ", "").replace("dfx::", "")[:56]


def load_pmc(path):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    trace, nsteps = sys.argv[1], int(sys.argv[2])
    fetch = load_pmc(sys.argv[3]) if len(sys.argv) > 3 else {}
    write = load_pmc(sys.argv[4]) if len(sys.argv) > 4 else {}
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(trace))]
    rows.sort()
    markers = os.environ.get("DFX_STEP_MARKER", "k_step_finalize,k_initv_onepass").split(",")
    fin = [e for s, e, k in rows if any(m in k for m in markers)]
    skip = int(os.environ.get("DFX_STEP_SKIP", "0"))
    if len(fin) < nsteps + 1 + skip:
        raise SystemExit("trace holds %d steps, need %d" % (len(fin), nsteps + 1 + skip))
    t0, t1 = fin[-nsteps - 1 - skip], fin[-1 - skip]
    per = collections.defaultdict(list)
    busy = 0
    for s, e, k in rows:
        if s >= t0 and e <= t1:
            per[k].append((e - s) / 1e3)
            busy += e - s
    wall_us = (t1 - t0) / 1e3
    out = sorted(((sum(v) / nsteps, k, v) for k, v in per.items()), reverse=True)
    print("window: %d steps, %.1f us/step wall, %.1f us/step inside kernels, %d dispatches/step"
          % (nsteps, wall_us / nsteps, busy / 1e3 / nsteps,
             sum(len(v) for v in per.values()) // nsteps))
    print()
    print("| kernel | calls/step | avg us/dispatch | us/step | % of step | FETCH_SIZE MB/dispatch "
          "| WRITE_SIZE MB/dispatch |")
    print("|---|---|---|---|---|---|---|")
    for us, k, v in out:
        cps = len(v) / nsteps
        f, w = fetch.get(k, []), write.get(k, [])
        n = max(1, int(round(cps)))
        fm = "%.1f" % (sum(f[-n:]) / len(f[-n:]) / 1024) if f else ""
        wm = "%.1f" % (sum(w[-n:]) / len(w[-n:]) / 1024) if w else ""
        print("| %s | %.2g | %.1f | %.1f | %.1f | %s | %s |" % (
            short(k), cps, sum(v) / len(v), us, 100 * us * nsteps / wall_us, fm, wm))


if __name__ == "__main__":
    main()
