"""profiles/<round>/pmc_requests.json from the TCC_EA0_RDREQ_sum / TCC_EA0_WRREQ_sum pass of
tools/profile.sh: the L2's memory-side requests per launch of the hot kernels, and per unique
key (U) and per nnz, averaged over the last `n` dispatches.
usage: pmc_requests.py counter_collection.csv U nnz out.json [tag] [n]
"""
import collections
import csv
import json
import sys

KERNELS = ("k_probe_keys", "k_fm_fwd", "k_fm_bwd", "k_chunk_hot", "k_loc_write", "k_loc_transform",
           "k_initv", "k_os_scatter<")


def main():
    path, U, nnz, out = sys.argv[1], float(sys.argv[2]), float(sys.argv[3]), sys.argv[4]
    tag = sys.argv[5] if len(sys.argv) > 5 else "r2"
    n = int(sys.argv[6]) if len(sys.argv) > 6 else 3
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, ctr in per.items():
        short = k.split("(")[0].replace("void ", "").replace("dfx::", "")
        if not any(short.startswith(p) for p in KERNELS):
            continue
        rd = ctr.get("TCC_EA0_RDREQ_sum", [0.0])[-n:]
        wr = ctr.get("TCC_EA0_WRREQ_sum", [0.0])[-n:]
        r, w = sum(rd) / len(rd), sum(wr) / len(wr)
        res[short] = {"rdreq_per_launch": round(r), "wrreq_per_launch": round(w),
                      "rdreq_per_nnz": round(r / nnz, 3), "wrreq_per_nnz": round(w / nnz, 3),
                      "rdreq_per_key": round(r / U, 3), "wrreq_per_key": round(w / U, 3)}
    src = ("rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum (a separate pass; "
           "tools/profile.sh %s), bench.py --steps 3 --warmup 1, last %d dispatches averaged; "
           "the L2's memory-side requests (MI355X_MICROARCH.md: FETCH_SIZE = RDREQ x 64 B; "
           "Infinity-Cache hits counted). Per-unit ratios use the bench's mean unique keys per "
           "step U = %d and nnz = %d." % (tag, n, U, nnz))
    json.dump({"_source": src, "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
