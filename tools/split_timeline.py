"""Where the split's exchanges run against its compute, from a rocprofv3 kernel trace of
tools/split_loopback.py: over a window of whole steps (N markers of k_split_worker_finalize
each), per stream its busy time in owner forwards, owner backwards, combines and exchange
copies (loopback exchanges are device copies, __amd_rocclr_copyBuffer), and how much of the
copy time overlaps a forward or backward running on another hardware queue.  Streams are told
apart by the trace's Queue_Id (its Stream_Id is 0 without runtime tracing, which made every
copy look serialised with every kernel).
usage: split_timeline.py trace.csv N [first_step] [steps]"""
import collections
import csv
import sys


def kind(name):
    if "fm_fwd" in name:
        return "forward"
    if "fm_bwd" in name:
        return "backward"
    if "combine" in name:
        return "combine"
    if "copyBuffer" in name:
        return "copy"
    return None


def main():
    path, N = sys.argv[1], int(sys.argv[2])
    s0 = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    ns = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                   r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    fin = [e for s, e, _, k in rows if "k_split_worker_finalize" in k]
    t0, t1 = fin[s0 * N - 1], fin[(s0 + ns) * N - 1]
    win = [(s, e, sid, kind(k)) for s, e, sid, k in rows if s >= t0 and e <= t1 and kind(k)]
    busy = collections.defaultdict(float)
    for s, e, sid, k in win:
        busy[(sid, k)] += (e - s) / 1e3
    comp = [(s, e, sid) for s, e, sid, k in win if k in ("forward", "backward")]
    copy_us = hidden = 0.0
    for s, e, sid, k in win:
        if k != "copy":
            continue
        copy_us += (e - s) / 1e3
        # the part of this copy during which some forward / backward of another stream ran
        cov = []
        for cs, ce, csid in comp:
            if csid != sid and ce > s and cs < e:
                cov.append((max(s, cs), min(e, ce)))
        cov.sort()
        last = s
        for a, b in cov:
            a = max(a, last)
            if b > a:
                hidden += (b - a) / 1e3
                last = b
    print("window: %d steps, %.1f us per step" % (ns, (t1 - t0) / 1e3 / ns))
    for (sid, k), us in sorted(busy.items()):
        print("  queue %-4s %-9s %9.1f us per step" % (sid, k, us / ns))
    print("exchange copies: %.1f us per step, %.0f %% of it beside a forward / backward of "
          "another queue" % (copy_us / ns, 100.0 * hidden / max(copy_us, 1e-9)))


if __name__ == "__main__":
    main()
