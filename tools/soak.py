"""Soak run of the fused step: many bench-shaped batches under the reference's default
updater settings (l1 = 1, V_threshold = 10, lazy InitV every step, the table growing from a
small max_keys), a sync and an error check every `every` steps.  Prints the progress per
interval; a device error (failed insert, look-back timeout, ...) raises.
usage: python tools/soak.py [steps] [every] [rows] [key_bits]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import DevBatch  # noqa: E402
from difacto_amd import hotpath as H  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
    kb = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = H.Context(0, V_dim=16, max_keys=1 << 20, lr=.1, V_lr=.01)  # l1 = 1, V_threshold = 10
    pool = [DevBatch(torch, dev, B, 39, kb, seed=5000 + i) for i in range(16)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        H.train_step(ctx, pool[s % len(pool)], H.kTraining, push_cnt=(s < len(pool)))
        if (s + 1) % every == 0:
            p = H.progress(ctx)  # syncs: raises on a device error
            st = H.Store(ctx).stats()
            _, maxp, cap = H.Store(ctx).probe_stats()
            print("step %5d  loss/row %.5f  auc %.4f  keys %d  V rows %d  cap %d  max probe %d  "
                  "%.1f s" % (s + 1, p["loss"] / p["nrows"], p["auc"] / p["nrows"], st["n_keys"],
                              st["n_vrows"], cap, maxp, time.perf_counter() - t0), flush=True)
    ctx.close()
    print("soak ok: %d steps" % steps)


if __name__ == "__main__":
    main()
