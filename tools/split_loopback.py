"""The split store's C++ driver over the loopback transport: N shards on this one GPU (one
context each), every exchange a device copy on the stream that the RCCL transport would use.
Run it under rocprofv3 --kernel-trace and read the per-stream timeline with tools/timeline.py
(marker k_split_worker_finalize) to see where the exchanges sit against the compute: in the
pipelined schedule between each step's forward and backward, in the stale one beside the
other step's compute.  Measurement tool, not a test.
  python3 tools/split_loopback.py [N] [stale 0|1] [steps] [rows per worker]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difacto_amd import data as D  # noqa: E402
from difacto_amd import dist as DI  # noqa: E402
from difacto_amd import hotpath as H  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    stale = len(sys.argv) > 2 and sys.argv[2] == "1"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    rows = int(sys.argv[4]) if len(sys.argv) > 4 else 12500
    kw = dict(V_dim=16, V_threshold=0, l1=0.0, lr=0.1, V_lr=0.01)
    # one stream per shard, as each rank has its own (a Context takes the current torch
    # stream: on the default one all N shards' compute would queue on one stream)
    streams = [torch.cuda.Stream() for _ in range(N)]
    ctxs = []
    for r in range(N):
        with torch.cuda.stream(streams[r]):
            ctxs.append(H.Context(0, max_keys=1 << 22, push_agg="sum", **kw))
    shards = [DI.Shard(c, N) for c in ctxs]
    store = DI.SplitStore(shards, stale=stale)
    blocks = [[D.synthetic(rows, 39, 1 << 22, seed=1000 * s + r) for r in range(N)]
              for s in range(steps)]
    dev = [[H.DeviceRowBlock(ctxs[r], b[r]) for r in range(N)] for b in blocks]
    torch.cuda.synchronize()
    store.submit(dev[0], H.kTraining, push_cnt=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(1, steps):
        store.submit(dev[s], H.kTraining)
    store.flush()
    for c in ctxs:
        c.sync()
    dt = (time.perf_counter() - t0) / (steps - 1)
    print("split loopback N=%d %s: %.3f ms per step (%d rows per worker, %.1f M ex/s over all "
          "shards on one GPU)" % (N, "stale" if stale else "pipelined", dt * 1e3, rows,
                                   N * rows / dt / 1e6))
    store.close()
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
