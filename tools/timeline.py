"""Per-step timeline of a rocprofv3 kernel trace: for steps [s0, s0 + n) (a step ends at each
k_step_finalize), every kernel's start / end in microseconds relative to the step's first kernel,
with its stream, so the critical path across the main stream and the lanes can be read.
usage: timeline.py trace_kernel_trace.csv [first_step] [n_steps] [marker]"""
import csv
import sys


def main():
    path = sys.argv[1]
    s0 = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    marker = sys.argv[4] if len(sys.argv) > 4 else "k_step_finalize,k_initv_onepass"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                         r["Kernel_Name"].split("(")[0]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if any(m in r[3] for m in marker.split(","))]
    lo = ends[s0 - 1] + 1 if s0 > 0 else 0
    hi = ends[s0 + n - 1] + 1
    t0 = rows[lo][0]
    for st, en, sid, name in rows[lo:hi]:
        print("%8.1f %8.1f %6.1f  s%-3s %s" % ((st - t0) / 1e3, (en - t0) / 1e3, (en - st) / 1e3,
                                               sid, name[:60]))


if __name__ == "__main__":
    main()
