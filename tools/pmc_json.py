"""profiles/<round>/pmc_hbm.json from the two rocprofv3 --pmc passes of tools/profile.sh:
per kernel, FETCH_SIZE and WRITE_SIZE (KB, as rocprofv3 reports them) averaged over the last
`n` dispatches.  bench.py reads it for the roofline's `traffic`.
usage: pmc_json.py fetch_counter_collection.csv write_counter_collection.csv out.json [n] [tag]
"""
import collections
import csv
import json
import sys

KERNELS = ("k_probe_keys", "k_fm_fwd", "k_fm_bwd", "k_chunk_hot", "k_loc_", "k_lb_",
           "k_os_scatter<", "k_initv", "k_dist_", "k_split_", "k_auc")


def load(path):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    fetch, write, out = load(sys.argv[1]), load(sys.argv[2]), sys.argv[3]
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    tag = sys.argv[5] if len(sys.argv) > 5 else "r1"
    res = {}
    for k in fetch:
        short = k.split("(")[0].replace("void ", "").replace("dfx::", "")
        if not any(short.startswith(p) for p in KERNELS):
            continue
        f, w = fetch[k][-n:], write.get(k, [0.0])[-n:]
        res[short] = {"fetch_size_kb_per_dispatch": sum(f) / len(f),
                      "write_size_kb_per_dispatch": sum(w) / len(w)}
    doc = {"_source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                      "bench.py --steps 3 --warmup 1 (tools/profile.sh %s); last %d dispatches "
                      "averaged; KB as rocprofv3 reports them (FETCH_SIZE = TCC_EA0_RDREQ x 64 B; "
                      "calibration: profiles/r1/pmc_calibration.json)" % (tag, n),
           "kernels": res}
    json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
