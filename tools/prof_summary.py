"""Summarise a rocprofv3 kernel trace (+ optional FETCH/WRITE PMC passes) per kernel over
the LAST n dispatches of each kernel (the bench's timed steps), as markdown."""
import csv
import collections
import sys


def load_trace(path):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(list)
    for r in rows:
        per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per


def load_pmc(path):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def short(name):
    s = name.split("(")[0]
    return s.replace("void ", "").replace("dfx::", "")[:48]


def main():
    trace, last = sys.argv[1], int(sys.argv[2])
    fetch = load_pmc(sys.argv[3]) if len(sys.argv) > 3 else {}
    write = load_pmc(sys.argv[4]) if len(sys.argv) > 4 else {}
    per = load_trace(trace)
    rows = []
    for k, v in per.items():
        calls_per_step = max(1, round(len(v) / max(1, len(per.get(next(
            n for n in per if "k_step_finalize" in n or "k_sum_parts" in n), [1])))))
        tail = v[-last * calls_per_step:]
        rows.append((sum(tail) / last, k, len(v), sum(tail) / len(tail), calls_per_step))
    rows.sort(reverse=True)
    print("| kernel | calls/step | avg us/dispatch (last %d steps) | us/step | FETCH_SIZE MB/dispatch | WRITE_SIZE MB/dispatch |" % last)
    print("|---|---|---|---|---|---|")
    for per_step, k, n, avg, cps in rows:
        f = fetch.get(k, [])
        w = write.get(k, [])
        fm = "%.1f" % (sum(f[-cps:]) / max(1, len(f[-cps:])) / 1024) if f else ""
        wm = "%.1f" % (sum(w[-cps:]) / max(1, len(w[-cps:])) / 1024) if w else ""
        print("| %s | %d | %.1f | %.1f | %s | %s |" % (short(k), cps, avg, per_step, fm, wm))


if __name__ == "__main__":
    main()
